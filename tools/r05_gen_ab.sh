#!/bin/bash
# Round 5: generated image_warping / shape_from_shading applies under each codegen form
# (OPT_AMD_GEN_STRIP32: 0 64-bit indices, 1 32-bit, 2 32-bit opaque; OPT_AMD_GEN_WIDU:
# readfirstlane wave index), two interleaved rounds, plus the hand-written applies:
#   tools/r05_gen_ab.sh <outdir> "S W" ...   (pairs of STRIP32 WIDU)
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 200 python3 tools/bench_families.py --only iw4096,sfs --out $O/hand.json > $O/hand.log 2>&1 || exit 1
for round in 1 2; do
  for v in "$@"; do
    sv=${v% *}; wv=${v#* }
    tag=s${sv}w${wv}
    OPT_AMD_GEN_STRIP32=$sv OPT_AMD_GEN_WIDU=$wv OPT_AMD_GEN_FACTOR=${GEN_FACTOR:-1} timeout -k 10 200 python3 tools/bench_families.py \
        --only iw4096_generic,sfs_generic --out $O/gen_$tag.$round.json > $O/gen_$tag.$round.log 2>&1 || exit 1
    python3 -c "
import json
for e in json.load(open('$O/gen_$tag.$round.json')): print('$tag', $round, e['config'][:22], round(e['apply_us'], 1), round(e['step_ms'], 3))"
  done
done
python3 -c "
import json
for e in json.load(open('$O/hand.json')): print('hand', e['config'][:22], round(e['apply_us'], 1), round(e['step_ms'], 3))"
