#!/bin/bash
# Round-3 measurement pass (through gpurun, from the repo root): the headline bench line,
# its rocprofv3 kernel-trace stats, and the FETCH_SIZE / WRITE_SIZE / SQ PMC passes.
set -e
R=$(pwd)
O=$R/gpurun_out/${1:-r03_measure}
mkdir -p $O
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/stats.log 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C -d $O/pmc_$C --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_$C.log 2>&1
done
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES \
    -d $O/pmc_sq --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_sq.log 2>&1
python3 tools/pmc_summary.py $O/pmc.json $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE $O/pmc_sq > /dev/null
echo DONE
