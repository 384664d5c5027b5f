#!/bin/bash
# Fused PCGStep2+3 of the generic driver (through gpurun): the SFS / decomposition / config-3
# tests, then the shape_from_shading bench leg with OPT_AMD_FUSE23=0 and =1, interleaved.
set -e
O=gpurun_out/${1:-r03_fuse23}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_sfs_gpu.py \
    -x -q -k fused_pcg \
    --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
tail -2 $O/tests.txt
for round in 1 2; do
  for f in 0 1; do
    OPT_AMD_FUSE23=$f timeout -k 10 200 python3 bench.py --workload shape_from_shading --no-cpu-baseline \
        > $O/sfs_$f.$round.json 2> $O/sfs_$f.$round.err
    python3 -c "import json; d=json.load(open('$O/sfs_$f.$round.json')); print('fuse23=$f', $round, round(d['ms_per_step'],3), 'apply', round(d['roofline']['avg_us'],1))"
  done
done
