"""Instruction mix of the loops of one kernel in a gfx950 .s file (hipcc --cuda-device-only -S):
python3 tools/loop_mix.py file.s <mangled-name-substring>"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
sym = [m for m in re.findall(r'^(_Z\S*):', s, re.M) if sys.argv[2] in m][0]
i = s.index(sym + ':')
j = s.index('.Lfunc_end', i)
body = s[i:j].splitlines()
labels = {}
for k, l in enumerate(body):
    m = re.match(r'^(\.LBB\S+):', l)
    if m:
        labels[m.group(1)] = k
for k, l in enumerate(body):
    m = re.search(r's_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)', l)
    if m:
        t = m.group(1) or m.group(2)
        if labels.get(t, 1e9) < k and k - labels[t] > 40:
            seg = body[labels[t]:k + 1]
            ins = [x.strip() for x in seg if x.startswith('\t') and not x.strip().startswith(('.', ';'))]
            c = Counter(x.split()[0] for x in ins)
            v = sum(n for op, n in c.items() if op.startswith('v_'))
            print(f"loop {t} len {len(ins)} valu {v} mem {sum(n for op, n in c.items() if op.startswith('global_'))} "
                  f"waitcnt {c['s_waitcnt']} f64 {sum(n for op, n in c.items() if 'f64' in op)} "
                  f"u64 {c['v_lshl_add_u64'] + c['v_mad_u64_u32']} mov {c['v_mov_b32_e32'] + c['v_mov_b64_e32']}")
            if len(sys.argv) > 3:
                for op, n in c.most_common(int(sys.argv[3])):
                    print(f"   {n:4d} {op}")
