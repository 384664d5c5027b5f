#!/bin/bash
# Round 5: FETCH_SIZE / WRITE_SIZE / SQ counters of the generated and the hand-written
# image_warping applies (tools/bench_families.py), each counter set its own rocprofv3 run:
#   tools/r05_gen_pmc.sh <outdir>
set -e
R=$(pwd)
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C -d $O/pmc_$C --output-format csv -- \
      python3 tools/bench_families.py --only ${CFGS:-iw4096,iw4096_generic} --steps 2 > $O/pmc_$C.log 2>&1
done
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES \
    -d $O/pmc_sq --output-format csv -- python3 tools/bench_families.py --only ${CFGS:-iw4096,iw4096_generic} --steps 2 > $O/pmc_sq.log 2>&1
python3 tools/pmc_summary.py $O/pmc.json $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE $O/pmc_sq > /dev/null
python3 - <<PY
import json
d = json.load(open("$O/pmc.json"))["kernels"]
for k, v in d.items():
    if "apply" not in k and "strip" not in k: continue
    wc = v.get("SQ_WAVE_CYCLES", 0)
    print(k.split("(")[0][:60], "B/px %.1f" % ((2 * v.get("FETCH_SIZE", 0) + v.get("WRITE_SIZE", 0)) * 1024 / 4096**2),
          "mem %.2f issue %.2f valu %.2f" % (v.get("SQ_WAIT_ANY", 0) / max(wc, 1), v.get("SQ_WAIT_INST_ANY", 0) / max(wc, 1),
                                             v.get("SQ_ACTIVE_INST_VALU", 0) / max(wc, 1)),
          "waves", v.get("SQ_WAVES"), "cyc/wave %.0f" % (wc / max(v.get("SQ_WAVES", 1), 1)))
PY
