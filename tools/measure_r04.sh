#!/bin/bash
# Round-4 measurement pass over ONE bench workload (through gpurun, from the repo root):
# the bench line, its rocprofv3 kernel-trace stats, and the FETCH_SIZE / WRITE_SIZE / SQ PMC
# passes (each its own run), summarised per kernel.
#   tools/measure_r04.sh <outdir> [image_warping|shape_from_shading]
set -e
R=$(pwd)
O=$R/gpurun_out/$1
WL=${2:-image_warping}
mkdir -p $O
timeout -k 10 300 python3 bench.py --workload $WL > $O/bench_$WL.json 2> $O/bench_$WL.err
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_$WL -o run --output-format csv -- \
    python3 bench.py --workload $WL --steps 10 --warmup 2 --no-cpu-baseline > $O/stats_$WL.log 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C -d $O/pmc_${WL}_$C --output-format csv -- \
      python3 bench.py --workload $WL --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_${WL}_$C.log 2>&1
done
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES \
    -d $O/pmc_${WL}_sq --output-format csv -- python3 bench.py --workload $WL --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_${WL}_sq.log 2>&1
python3 tools/pmc_summary.py $O/pmc_$WL.json $O/pmc_${WL}_FETCH_SIZE $O/pmc_${WL}_WRITE_SIZE $O/pmc_${WL}_sq > /dev/null
find $O/stats_$WL -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_$WL.csv \;
echo DONE $WL
