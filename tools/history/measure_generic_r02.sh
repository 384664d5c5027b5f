# Generated-kernel measurement pass (round 2): bench rows with the default apply form
# (register strips where >= 2048 waves) and with the gather forced, plus rocprofv3 kernel
# stats of the generated image_warping and shape_from_shading steps.
#   bash tools/measure_generic_r02.sh   (on the GPU box; outputs under gpurun_out/)
set -e
R=$(pwd)
O=$R/gpurun_out/generic_r02
mkdir -p $O
timeout -k 10 300 python3 -u tools/bench_families.py --only iw4096_generic,sfs_generic,poisson_generic,arap_generic \
    --out $O/strip.json > $O/strip.log 2>&1
OPT_AMD_GEN_APPLY=gather timeout -k 10 300 python3 -u tools/bench_families.py \
    --only iw4096_generic,sfs_generic,poisson_generic --out $O/gather.json > $O/gather.log 2>&1
bash tools/prof_family.sh iw4096_generic generic_r02_iw
bash tools/prof_family.sh sfs_generic generic_r02_sfs
