#!/bin/bash
# Round-3 measurement pass (through gpurun, from the repo root): every -m gpu test, smoke(),
# the two bench lines, the bench's kernel-trace stats, the FETCH_SIZE / WRITE_SIZE / SQ PMC
# passes over the bench, and the per-config table. Output: gpurun_out/${1:-r03_final}.
set -e
R=$(pwd)
O=$R/gpurun_out/${1:-r03_final}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
tail -1 $O/gpu_tests.txt
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python3 bench.py --workload shape_from_shading > $O/bench_sfs.json 2> $O/bench_sfs.err
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
timeout -k 10 600 python3 tools/bench_families.py --out $O/families.json > $O/families.log 2>&1
echo DONE
