#!/bin/bash
# Generated graph apply A/B (round 4): build_ab/base (HEAD before the change) against the
# tree (32-bit gather offsets, centred terms fused into gen_apply_graph) at edge-loop
# unroll 4 and 2, interleaved twice; then the tree's counters.
#   tools/r04_graph.sh <outdir>   (through gpurun, repo root)
set -e
R=$(pwd)
O=$R/gpurun_out/${1:-r04_graph}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_generic_gpu.py tests/test_reference_costs_gpu.py -x -q \
    --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
tail -1 $O/tests.txt
for i in 1 2; do
  for v in base tree tree@2 base@2; do
    n=${v%%@*}; u=${v#*@}; [ "$u" = "$v" ] && u=4
    lib=build_ab/$n/libopt_amd.so; [ $n = tree ] && lib=opt_amd/libopt_amd.so
    OPT_AMD_LIB=$lib OPT_AMD_GEN_EDGE_UNROLL=$u timeout -k 10 300 python3 tools/bench_families.py --only arap_generic \
        --out $O/${n}_u${u}_$i.json > $O/${n}_u${u}_$i.log 2>&1
    python3 -c "import json; d=json.load(open('$O/${n}_u${u}_$i.json'))[0]; print('$n u$u', $i, round(d['apply_us'],1), round(d['step_ms'],3), d.get('cost_after'))"
  done
done
bash tools/pmc_family.sh ${1:-r04_graph}/pmc_tree arap_generic
[ -n "$PMC_BASE" ] && bash tools/pmc_family.sh ${1:-r04_graph}/pmc_base arap_generic build_ab/base/libopt_amd.so
echo DONE
