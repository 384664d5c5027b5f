# A/B of the ARAP apply variants (OPT_AMD_ARAP_APPLY): parity tests, then the family
# bench row per variant. Run through gpurun from the repo root.
set -e
mkdir -p gpurun_out/arapv
VARS=${VARS:-"0 4 5 6"}
for V in $VARS; do
  OPT_AMD_ARAP_APPLY=$V timeout -k 10 300 python -u -m pytest tests/test_arap_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/arapv/test_$V.log 2>&1
done
for V in $VARS; do
  OPT_AMD_ARAP_APPLY=$V timeout -k 10 200 python tools/bench_families.py --only arap,arap --steps 5 > gpurun_out/arapv/bench_$V.json 2> gpurun_out/arapv/bench_$V.err
done
echo DONE
