#!/bin/bash
# Deferred-delta A/B (through gpurun): the bitwise tests, then the headline bench with the
# per-iteration delta update (OPT_AMD_IW_DEFER=0) and the deferred one (=1), interleaved.
set -e
O=gpurun_out/${1:-r03_defer}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_image_warping_gpu.py -x -q -k "bitwise or fused" \
    --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
tail -2 $O/tests.txt
bash tools/ab_run.sh ${1:-r03_defer} tree tree@OPT_AMD_IW_RES_NT=3 tree@OPT_AMD_IW_RES_NT=0 tree@OPT_AMD_ROWS=16 tree@OPT_AMD_ROWS=64
