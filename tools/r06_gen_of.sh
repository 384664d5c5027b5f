set -o pipefail
mkdir -p gpurun_out/r06n
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_generic_gpu.py tests/test_optical_flow_gpu.py tests/test_family_routing.py tests/test_generic_examples_gpu.py > gpurun_out/r06n/tests.txt 2>&1 || { tail -40 gpurun_out/r06n/tests.txt; exit 1; }
tail -2 gpurun_out/r06n/tests.txt
timeout -k 10 600 python -u tools/bench_families.py --only optical_flow,optical_flow_generic,sfs,sfs_generic --out gpurun_out/r06n/fam.json > gpurun_out/r06n/fam.log 2>&1 || { tail -20 gpurun_out/r06n/fam.log; exit 1; }
OPT_AMD_GEN_SAMPLE_CACHE=0 timeout -k 10 600 python -u tools/bench_families.py --only optical_flow_generic --out gpurun_out/r06n/fam_nocache.json > gpurun_out/r06n/fam_nocache.log 2>&1
python3 -c "
import json
for f in ['fam','fam_nocache']:
    for r in json.load(open('gpurun_out/r06n/%s.json'%f)): print(f, r['config'], round(r['apply_us'],1), r['apply_kernel'], round(r['step_ms'],3))
"
