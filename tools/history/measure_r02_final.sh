#!/bin/bash
# Closing round-2 pass (through gpurun, from the repo root): every -m gpu test, smoke(),
# the two bench lines, the bench's kernel-trace stats and the per-config table (the
# kernels the PMC summaries profiles/r02_pmc*.json were taken on are unchanged).
set -e
R=$(pwd)
O=$R/gpurun_out/r02_final
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 200 python3 bench.py --no-cpu-baseline --workload shape_from_shading > $O/bench_sfs.json 2> $O/bench_sfs.err
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/stats.log 2>&1
timeout -k 10 600 python3 tools/bench_families.py --out $O/families.json > $O/families.log 2>&1
echo DONE
