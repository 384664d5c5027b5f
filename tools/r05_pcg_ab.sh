set -o pipefail
mkdir -p gpurun_out/r05e
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_image_warping_gpu.py -k "without_stored_ap or deferred_delta or double_precision_path or fused_residual or fused_init or test_gn_solve or far_past" > gpurun_out/r05e/tests.txt 2>&1 || exit 1
bash tools/ab_run.sh r05e tree@OPT_AMD_IW_APFREE=0 tree tree@OPT_AMD_IW_JTF_NT=0 tree@OPT_AMD_IW_PCG_NT=1
