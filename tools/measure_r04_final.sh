#!/bin/bash
# Round-4 closing pass (through gpurun, from the repo root), in two calls:
#   tools/measure_r04_final.sh <outdir> tests   every -m gpu test and smoke()
#   tools/measure_r04_final.sh <outdir> bench   both bench lines with their kernel-trace
#        stats and FETCH_SIZE / WRITE_SIZE / SQ PMC passes (tools/measure_r04.sh), the
#        shape_from_shading apply cache study and the per-config table
set -e
R=$(pwd)
O=$R/gpurun_out/$1
mkdir -p $O
if [ "$2" = tests ]; then
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
  tail -1 $O/gpu_tests.txt
  timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
  tail -1 $O/smoke.txt
else
  bash tools/measure_r04.sh $1 image_warping
  bash tools/measure_r04.sh $1 shape_from_shading
  timeout -k 10 300 python3 tools/apply_cache_study.py > $O/cache_study.txt 2>&1
  timeout -k 10 600 python3 tools/bench_families.py --out $O/families.json > $O/families.log 2>&1
fi
echo DONE
