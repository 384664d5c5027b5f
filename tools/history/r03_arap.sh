#!/bin/bash
# ARAP apply pass (through gpurun): the ARAP GPU tests, then the arap config of
# tools/bench_families.py with 3 and 2 merged slots per batch, and a rocprofv3 kernel
# trace of the default.
set -e
O=gpurun_out/${1:-r03_arap}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_arap_gpu.py tests/test_reference_costs_gpu.py -x -q \
    --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
tail -2 $O/tests.txt
for eb in 3 2 3 2; do
  OPT_AMD_ARAP_EB=$eb timeout -k 10 300 python3 tools/bench_families.py --only arap --steps 10 --out $O/families_eb$eb.json > $O/families.log 2>&1
  python3 -c "import json; d=json.load(open('$O/families_eb$eb.json'))[0]; print('eb $eb', round(d['apply_us'],1), round(d['roofline']['frac'],3), round(d['step_ms'],3))"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- \
    python3 tools/bench_families.py --only arap --steps 10 > $O/stats.log 2>&1
echo DONE
