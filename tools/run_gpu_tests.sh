#!/bin/bash
# Run a list of GPU test files (through gpurun): tools/run_gpu_tests.sh <outdir> <pytest args...>
R=$(pwd)
O=$R/gpurun_out/$1
shift
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest "$@" -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?
tail -3 $O/gpu_tests.txt
exit $rc
