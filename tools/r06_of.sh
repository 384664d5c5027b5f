#!/bin/bash
# Round 6: optical_flow family strip apply — tests, then the families rows (strip / flat / generated)
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_optical_flow_gpu.py tests/test_materialized_gpu.py -k "optical or flow or of_" > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for v in "OPT_AMD_OF_STRIP=1" "OPT_AMD_OF_STRIP=0" "OPT_AMD_OF_ROWS=8" "OPT_AMD_OF_ROWS=32"; do
  env $v timeout -k 10 600 python -u tools/bench_families.py --only optical_flow --out $O/fam_$v.json > $O/fam_$v.log 2>&1 || { tail -20 $O/fam_$v.log; exit 1; }
  python3 -c "import json; r=json.load(open('$O/fam_$v.json'))[0]; print('$v', r['config'], round(r['apply_us'],1), round(r['step_ms'],3), r['cost_after'])"
done
exit 0
