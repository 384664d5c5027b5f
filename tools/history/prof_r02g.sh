#!/bin/bash
# GPU tests (all), family step times (arap / sfs / optical_flow), ARAP kernel stats + PMC
set -e
O=gpurun_out/r02g
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo "tests rc=$?" >> $O/gpu_tests.txt; }
timeout -k 10 300 python tools/bench_families.py --only arap,sfs,optical_flow --steps 5 > $O/fam.json 2> $O/fam.err
OPT_AMD_ARAP_EP=0 timeout -k 10 120 python tools/bench_families.py --only arap --steps 5 > $O/fam_arap_vpt.json 2>> $O/fam.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_arap -o run -- python tools/bench_families.py --only arap --steps 5 > $O/prof_arap.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_arap_fetch -o run -- python tools/bench_families.py --only arap --steps 2 > $O/pmc1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_arap_write -o run -- python tools/bench_families.py --only arap --steps 2 > $O/pmc2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS --output-format csv -d $O/pmc_arap_sq -o run -- python tools/bench_families.py --only arap --steps 2 > $O/pmc3.log 2>&1
echo done
