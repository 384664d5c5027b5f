#!/bin/bash
# Build compile-time variants of libopt_amd.so for A/B runs on the GPU:
#   tools/ab_build.sh name1 "-DFOO=1" name2 "-DFOO=2" ...
# -> build_ab/<name>/libopt_amd.so (select with OPT_AMD_LIB=...; build_ab/ ships with gpurun: delete it after the A/B)
set -e
while [ $# -ge 2 ]; do
    n=$1; d=$2; shift 2
    make -s -j8 OBJ_DIR=build_ab/$n/obj LIB=build_ab/$n/libopt_amd.so EXTRA="$d" build_ab/$n/libopt_amd.so
    echo "built build_ab/$n ($d)"
done
