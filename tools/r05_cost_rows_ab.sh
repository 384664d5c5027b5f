#!/bin/bash
# Round 5: iw_cost60 rows per wave (OPT_AMD_IW_COST_ROWS; 0 = the plan's 32) through the
# bench's own kernel timing, two interleaved rounds:
#   tools/r05_cost_rows_ab.sh ROWS ...
O=gpurun_out/costab; mkdir -p $O
for r in 1 2; do for cr in "$@"; do
  OPT_AMD_IW_COST_ROWS=$cr timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 10 \
      > $O/b$cr.$r.json 2> $O/b$cr.$r.err || exit 1
  python3 -c "
import json;d=json.loads(open('$O/b$cr.$r.json').read().strip().splitlines()[-1]);s=d['step_kernels']
print('rows $cr', round(s['iw_cost']['avg_us'],1), round(s['iw_pcg']['avg_us'],1), round(d['ms_per_step'],3))"
done; done
