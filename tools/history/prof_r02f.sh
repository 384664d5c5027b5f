#!/bin/bash
# Round-2 measurement pass: bench lines (image_warping, shape_from_shading), kernel stats
# of the LM configs and ARAP, ARAP PMC, the two-rank RCCL test.
set -e
O=gpurun_out/r02f
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_rccl_multirank_gpu.py -m gpu -q -rs --timeout 240 --timeout-method thread > $O/rccl_test.txt 2>&1 || echo "rccl test rc=$?" >> $O/rccl_test.txt
timeout -k 10 150 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
timeout -k 10 150 python bench.py --no-cpu-baseline --workload shape_from_shading > $O/bench_sfs.json 2> $O/bench_sfs.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in sfs optical_flow arap; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- python tools/bench_families.py --only $c --steps 5 > $O/fam_$c.json 2> $O/fam_$c.err
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_arap_fetch -o run -- python tools/bench_families.py --only arap --steps 2 > $O/pmc1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_arap_write -o run -- python tools/bench_families.py --only arap --steps 2 > $O/pmc2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM --output-format csv -d $O/pmc_arap_sq -o run -- python tools/bench_families.py --only arap --steps 2 > $O/pmc3.log 2>&1
echo done
