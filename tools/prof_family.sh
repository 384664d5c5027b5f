# Kernel-trace stats of one family's bench row: bash tools/prof_family.sh <config> [tag]
set -e
R=$(pwd)
C=$1
O=$R/gpurun_out/prof_${2:-$C}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- \
    python3 $R/tools/bench_families.py --only $C --steps 5 > $O/log.txt 2>&1
