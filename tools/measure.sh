#!/bin/bash
# One GPU measurement pass (run through gpurun from the repo root):
# bench line, kernel-trace stats, FETCH/WRITE PMC passes over the bench, and the
# per-config table (incl. the materialized-Jacobian rows). Outputs under gpurun_out/$TAG.
# (The FETCH_SIZE calibration, tools/fetchcal.hip, is a one-off: profiles/r01_fetchcal.json.)
set -e
R=$(pwd)
TAG=${1:-meas}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- \
    python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/stats.log 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -d $O/pmc_$C --output-format csv -- \
      python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_$C.log 2>&1
done
cd $R
python3 tools/pmc_summary.py $O/pmc.json $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE > /dev/null
timeout -k 10 600 python3 tools/bench_families.py --out $O/families.json > $O/families.log 2>&1
echo DONE
