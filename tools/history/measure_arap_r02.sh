#!/bin/bash
# ARAP part of the round-2 measurement pass (tools/measure_r02.sh): kernel trace + the
# FETCH / WRITE / SQ / TA counter passes over the 1M-vertex config.
set -e
R=$(pwd)
O=$R/gpurun_out/${1:-r02t}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
B="python3 tools/bench_families.py --only arap --steps 5"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_arap -o run -- $B > $O/fam_arap.json 2> $O/fam_arap.err
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d $O/pmc_arap_$C -o run -- python3 tools/bench_families.py --only arap --steps 2 > $O/pmc_arap_$C.log 2>&1
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES \
    --output-format csv -d $O/pmc_arap_sq -o run -- python3 tools/bench_families.py --only arap --steps 2 > $O/pmc_arap_sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE \
    --output-format csv -d $O/pmc_arap_ta -o run -- python3 tools/bench_families.py --only arap --steps 2 > $O/pmc_arap_ta.log 2>&1
python3 tools/pmc_summary.py $O/pmc_arap.json $O/pmc_arap_FETCH_SIZE $O/pmc_arap_WRITE_SIZE $O/pmc_arap_sq $O/pmc_arap_ta > /dev/null
timeout -k 10 200 python3 tools/bench_families.py --only arap --steps 10 > $O/fam_arap_timed.json 2>&1
echo DONE
