#!/bin/bash
# Round 5: generated applies under a fixed grid (OPT_AMD_GEN_BLOCKS; 0 = the resident-round
# rule), two interleaved rounds: tools/r05_gen_blocks_ab.sh <outdir> BLOCKS ...
O=gpurun_out/$1; shift
mkdir -p $O
for round in 1 2; do
  for b in "$@"; do
    if [ "$b" = 0 ]; then e=""; else e="OPT_AMD_GEN_BLOCKS=$b"; fi
    env $e timeout -k 10 200 python3 tools/bench_families.py --only iw4096_generic,sfs_generic \
        --out $O/gen_b$b.$round.json > $O/gen_b$b.$round.log 2>&1 || exit 1
    python3 -c "
import json
for e in json.load(open('$O/gen_b$b.$round.json')): print('blocks $b', $round, e['config'][:22], round(e['apply_us'], 1), round(e['step_ms'], 3))"
  done
done
