#!/bin/bash
# Round-2 measurement pass (through gpurun, from the repo root): the bench lines
# (image_warping headline, shape_from_shading leg), kernel-trace stats of the bench and
# of the LM / graph configs, FETCH_SIZE / WRITE_SIZE PMC passes (one counter group per
# run), the ARAP SQ / TA counters, and the per-config table. Outputs under
# gpurun_out/$TAG; the summaries worth keeping are copied to profiles/ afterwards.
set -e
R=$(pwd)
TAG=${1:-r02z}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 200 python3 bench.py --no-cpu-baseline --workload shape_from_shading > $O/bench_sfs.json 2> $O/bench_sfs.err
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/stats.log 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C -d $O/pmc_$C --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_$C.log 2>&1
done
for c in sfs optical_flow arap; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- \
      python3 tools/bench_families.py --only $c --steps 5 > $O/fam_$c.json 2> $O/fam_$c.err
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d $O/pmc_${c}_$C -o run -- \
        python3 tools/bench_families.py --only $c --steps 2 > $O/pmc_${c}_$C.log 2>&1
  done
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES \
    --output-format csv -d $O/pmc_arap_sq -o run -- python3 tools/bench_families.py --only arap --steps 2 > $O/pmc_arap_sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE \
    --output-format csv -d $O/pmc_arap_ta -o run -- python3 tools/bench_families.py --only arap --steps 2 > $O/pmc_arap_ta.log 2>&1
python3 tools/pmc_summary.py $O/pmc.json $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE > /dev/null
for c in sfs optical_flow; do
  python3 tools/pmc_summary.py $O/pmc_$c.json $O/pmc_${c}_FETCH_SIZE $O/pmc_${c}_WRITE_SIZE > /dev/null
done
python3 tools/pmc_summary.py $O/pmc_arap.json $O/pmc_arap_FETCH_SIZE $O/pmc_arap_WRITE_SIZE $O/pmc_arap_sq $O/pmc_arap_ta > /dev/null
timeout -k 10 600 python3 tools/bench_families.py --out $O/families.json > $O/families.log 2>&1
echo DONE
