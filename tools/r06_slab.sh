#!/bin/bash
# Round 6: one rank's slab (tools/slab_rank.py) for image_warping GN and shape_from_shading LM,
# with the rows-per-wave / side / FUSE23 A/B: tools/r06_slab.sh <outdir> [iw|sfs|both]
# (VARIANTS=closing: the round-6 closing set)
set -o pipefail
O=gpurun_out/$1; mkdir -p $O; WHICH=${2:-both}
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u tools/slab_rank.py $ARGS > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; };
  python3 -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['ms_per_step_slab'], d['ms_per_step_full_image'], d['slab_over_full_div_world'])"; }
if [ $WHICH != sfs ]; then
ARGS="image_warping 8 3 4096 4096 10"
if [ "$VARIANTS" = u2 ]; then   # one row per trip (fewer VGPRs) with fewer rows per wave
run iw_rows_auto OPT_AMD_X=0
run iw_u2off OPT_AMD_IW_PCG_U2=0
run iw_u2off_rows10 OPT_AMD_IW_PCG_U2=0 OPT_AMD_ROWS=10
run iw_u2off_rows8 OPT_AMD_IW_PCG_U2=0 OPT_AMD_ROWS=8
run iw_rows10 OPT_AMD_ROWS=10
elif [ "$VARIANTS" = closing ]; then   # round 6 closing set: the defaults, rows 12, forward-only kernels
run iw_rows_auto OPT_AMD_X=0
run iw_rows12 OPT_AMD_ROWS=12
run iw_rows_auto_norev OPT_AMD_IW_MALL_REV=0
else
run iw_rows_auto OPT_AMD_X=0
run iw_rows16 OPT_AMD_ROWS=16
run iw_rows24 OPT_AMD_ROWS=24
run iw_rows_auto_noside OPT_AMD_IW_PCG_SIDE=0
run iw_rows16_jtfside OPT_AMD_ROWS=16 OPT_AMD_IW_JTF_SIDE=1 OPT_AMD_IW_COST_SIDE=1
fi
fi
if [ $WHICH != iw ]; then
ARGS="shape_from_shading 8 3 4096 4096 10"
if [ "$VARIANTS" = sfsrows ]; then   # rows per wave of the once-per-step strips (cost, model cost, precompute)
run sfs_classic OPT_AMD_FUSE23=0
run sfs_cp16 OPT_AMD_FUSE23=0 OPT_AMD_SFS_COST_ROWS=16 OPT_AMD_SFS_PRE_ROWS=16
run sfs_cp12 OPT_AMD_FUSE23=0 OPT_AMD_SFS_COST_ROWS=12 OPT_AMD_SFS_PRE_ROWS=12
run sfs_cp8 OPT_AMD_FUSE23=0 OPT_AMD_SFS_COST_ROWS=8 OPT_AMD_SFS_PRE_ROWS=8
elif [ "$VARIANTS" = flat ]; then   # the flat PCG kernels' grid cap
run sfs_classic OPT_AMD_FUSE23=0
run sfs_flat8192 OPT_AMD_FUSE23=0 OPT_AMD_FLAT_BLOCKS=8192
run sfs_flat65536 OPT_AMD_FUSE23=0 OPT_AMD_FLAT_BLOCKS=65536
else
run sfs_classic OPT_AMD_FUSE23=0
[ "$VARIANTS" = closing ] || run sfs_fused OPT_AMD_FUSE23=1
fi
fi
exit 0
