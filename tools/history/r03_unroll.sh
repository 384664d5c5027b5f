# Edge-loop unroll A/B for the generated graph gathers (round 3):
#   bash tools/r03_unroll.sh <tag>   (on the GPU box; outputs under gpurun_out/<tag>)
set -e
R=$(pwd)
O=$R/gpurun_out/${1:-r03_unroll}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_generic_gpu.py tests/test_reference_costs_gpu.py -x -q \
    --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
for i in 1 2; do
  for u in 1 2 4; do
    OPT_AMD_GEN_EDGE_UNROLL=$u timeout -k 10 300 python3 -u tools/bench_families.py --only arap_generic \
        --out $O/u${u}_$i.json > $O/u${u}_$i.log 2>&1
  done
done
OPT_AMD_GEN_EDGE_UNROLL=2 timeout -k 10 600 python3 -u -m pytest tests/test_generic_gpu.py -x -q -k "arap or graph" \
    --timeout 300 --timeout-method thread > $O/tests_u2.txt 2>&1
