#!/bin/bash
# Round 6: GPU tests (one pytest process), then the headline bench line for each A/B variant,
# twice, interleaved on one box:
#   tools/r06_ab.sh <outdir> "<pytest args or NONE>" [variants...]   (variants as tools/ab_run.sh)
set -o pipefail
O=$1; T=$2; shift 2
mkdir -p gpurun_out/$O
if [ "$T" != "NONE" ]; then
  timeout -k 10 1000 python -u -m pytest -x -q --timeout 400 --timeout-method thread $T \
      > gpurun_out/$O/tests.txt 2>&1 || { tail -40 gpurun_out/$O/tests.txt; exit 1; }
  tail -2 gpurun_out/$O/tests.txt
fi
[ $# -gt 0 ] && bash tools/ab_run.sh $O "$@"
exit 0
