#!/bin/bash
# Round-4 experiment batch (through gpurun, repo root): the hand-written ARAP apply
# variants, XCD-contiguous order for every generated loop, the factored fp64 dots of the
# image_warping passes; each an interleaved A/B against the tree, then the ARAP counters.
set -e
O=${1:-r04_batch}
mkdir -p gpurun_out/$O
timeout -k 10 300 python3 -u -m pytest tests/test_arap_gpu.py tests/test_image_warping_gpu.py -x -q --timeout 120 \
    --timeout-method thread -k "not depth and not fp64_truth" > gpurun_out/$O/tests.txt 2>&1
tail -1 gpurun_out/$O/tests.txt
bash tools/ab_family.sh $O/arap arap base tree dpf dpf@OPT_AMD_ARAP_EB=1 ownk
for c in optical_flow_generic iw4096_generic poisson_generic sfs_generic; do
  bash tools/ab_family.sh $O/$c $c tree xall
done
bash tools/ab_run.sh $O/iw tree nofact
bash tools/pmc_family.sh $O/pmc_arap arap
echo DONE
