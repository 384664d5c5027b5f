# Graph record cache A/B (round 3): generated-kernel GPU tests, then the generated ARAP
# bench row with OPT_AMD_GEN_GRAPH_CACHE=0 / 1 (twice each) and kernel stats with it on.
#   bash tools/r03_gcache.sh   (on the GPU box; outputs under gpurun_out/r03_gcache)
set -e
R=$(pwd)
O=$R/gpurun_out/${1:-r03_gcache}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_generic_gpu.py tests/test_reference_costs_gpu.py -x -q \
    --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
for i in 1 2; do
  for c in 0 1; do
    OPT_AMD_GEN_GRAPH_CACHE=$c timeout -k 10 300 python3 -u tools/bench_families.py --only arap_generic \
        --out $O/c${c}_$i.json > $O/c${c}_$i.log 2>&1
  done
done
bash tools/prof_family.sh arap_generic ${1:-r03_gcache}
