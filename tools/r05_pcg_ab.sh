#!/bin/bash
# Round 5: iw_pcg parity tests, then the headline bench for the iw_pcg variants (A/B, two
# interleaved rounds on one box): tools/r05_pcg_ab.sh <outdir> [variants...]
set -o pipefail
O=$1; shift
mkdir -p gpurun_out/$O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_image_warping_gpu.py \
    -k "rec_layout or without_stored_ap or deferred_delta or double_precision_path or fused_residual or fused_init or test_gn_solve or far_past or bench_workload_matches" \
    > gpurun_out/$O/tests.txt 2>&1 || { tail -30 gpurun_out/$O/tests.txt; exit 1; }
tail -1 gpurun_out/$O/tests.txt
bash tools/ab_run.sh $O "$@"
