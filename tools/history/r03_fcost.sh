# Fused update + cost (round 3): image_warping GPU tests, then bench A/B
# (OPT_AMD_IW_FUSED_COST=0 / 1, twice each) and kernel stats of the default.
#   bash tools/r03_fcost.sh <tag>   (on the GPU box; outputs under gpurun_out/<tag>)
set -e
R=$(pwd)
O=$R/gpurun_out/${1:-r03_fcost}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_image_warping_gpu.py -x -q \
    --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
for i in 1 2; do
  for c in 0 1; do
    OPT_AMD_IW_FUSED_COST=$c timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/b${c}_$i.json 2> $O/b${c}_$i.log
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.log
