#!/bin/bash
# Kernel-trace stats and PMC passes (FETCH_SIZE, WRITE_SIZE, SQ, TA/TD/TCP; each its own
# run) over one tools/bench_families.py config, summarised per kernel:
#   tools/pmc_family.sh <outdir> <config> [libopt_amd.so]   (through gpurun, repo root)
# -> gpurun_out/<outdir>/{kernel_stats_<config>.csv, pmc_<config>.json}
set -e
R=$(pwd)
O=$R/gpurun_out/$1
C=$2
[ -n "$3" ] && export OPT_AMD_LIB=$3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
B="python3 tools/bench_families.py --only $C --steps 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_$C -o run --output-format csv -- \
    $B --out $O/stats_$C.json > $O/stats_$C.log 2>&1
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $P -d $O/pmc_${C}_$P --output-format csv -- $B --out $O/p.json > $O/pmc_${C}_$P.log 2>&1
done
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES \
    -d $O/pmc_${C}_sq --output-format csv -- $B --out $O/p.json > $O/pmc_${C}_sq.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE \
    -d $O/pmc_${C}_ta --output-format csv -- $B --out $O/p.json > $O/pmc_${C}_ta.log 2>&1
python3 tools/pmc_summary.py $O/pmc_$C.json $O/pmc_${C}_FETCH_SIZE $O/pmc_${C}_WRITE_SIZE $O/pmc_${C}_sq $O/pmc_${C}_ta > /dev/null
find $O/stats_$C -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_$C.csv \;
echo DONE $C
