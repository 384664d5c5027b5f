#!/bin/bash
# PMC passes over the headline bench (through gpurun): FETCH_SIZE, WRITE_SIZE and the SQ
# occupancy / wait counters, each in its own rocprofv3 run; summary -> <out>/pmc.json.
#   tools/pmc_iw.sh <outdir> [extra env for bench]
set -e
R=$(pwd)
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C -d $O/pmc_$C --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_$C.log 2>&1
done
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES \
    -d $O/pmc_sq --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_sq.log 2>&1
python3 tools/pmc_summary.py $O/pmc.json $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE $O/pmc_sq > /dev/null
python3 - <<PY
import json
d = json.load(open("$O/pmc.json"))["kernels"]
for k, v in d.items():
    if "iw_" not in k: continue
    n = k.split("(")[0].replace("void optamd::iw::", "")
    f, w = v.get("FETCH_SIZE", 0) * 2048, v.get("WRITE_SIZE", 0) * 1024
    wc = v.get("SQ_WAVE_CYCLES", 0)
    print(f"{n:45s} MB {f/1e6:8.1f} + {w/1e6:8.1f}  wait_any {v.get('SQ_WAIT_ANY',0)/max(wc,1):.2f} "
          f"valu_active {v.get('SQ_ACTIVE_INST_VALU',0)/max(wc,1):.2f} insts_valu/wave {v.get('SQ_INSTS_VALU',0)/max(v.get('SQ_WAVES',1),1):.0f}")
PY
