# A/B of streaming (nontemporal) PCG-vector access in iw_apply / iw_residual
# (OPT_AMD_IW_NT): image_warping parity tests with NT on, then bench.py twice per
# setting, interleaved. Run through gpurun from the repo root.
set -e
O=gpurun_out/iwnt
mkdir -p $O
OPT_AMD_IW_NT=7 timeout -k 10 300 python -u -m pytest tests/test_image_warping_gpu.py tests/test_decomposition_gpu.py \
    -x -q --timeout 120 --timeout-method thread > $O/test_nt7.log 2>&1
for k in 1 2; do
  for V in 0 2 4 6; do
    OPT_AMD_IW_NT=$V timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/bench_${V}_$k.json 2> $O/bench_${V}_$k.err
  done
done
echo DONE
