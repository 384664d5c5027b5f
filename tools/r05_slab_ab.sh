set -o pipefail
bash tools/run_gpu_tests.sh r05o tests/test_decomposition_gpu.py tests/test_config3_split_gpu.py tests/test_rccl_multirank_gpu.py tests/test_bench_launcher.py -x || exit 1
for v in "" "OPT_AMD_IW_FUSED_INIT=0 OPT_AMD_IW_APFREE=0" "" "OPT_AMD_IW_FUSED_INIT=0 OPT_AMD_IW_APFREE=0"; do
  echo "variant [$v]"
  env $v timeout -k 10 120 python3 tools/slab_step.py 8 4096 4096 10 || exit 1
  env $v timeout -k 10 120 python3 tools/slab_step.py 2 4096 1024 10 || exit 1
done
