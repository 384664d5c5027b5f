#!/bin/bash
# Round-3 image_warping pass (through gpurun, from the repo root): the image_warping,
# decomposition and C-caller GPU tests, the headline bench line and its kernel-trace stats.
set -e
R=$(pwd)
O=$R/gpurun_out/${1:-r03_iw}
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_image_warping_gpu.py tests/test_decomposition_gpu.py \
    tests/test_c_caller_gpu.py -v --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1 || true
grep -q "Fatal\|core dumped\|Timeout" $O/gpu_tests.txt && exit 1
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/stats.log 2>&1
echo DONE
