#!/bin/bash
# On the GPU box: the headline bench line for each A/B variant, twice, interleaved:
#   tools/ab_run.sh <outdir> v1 v2 ...
# a variant is <name> (build_ab/<name>/libopt_amd.so; "tree" = opt_amd/libopt_amd.so)
# optionally followed by @VAR=value[@VAR=value...] environment settings.
O=gpurun_out/$1; shift
mkdir -p $O
for round in 1 2; do
  for v in "$@"; do
    n=${v%%@*}
    lib=build_ab/$n/libopt_amd.so
    [ "$n" = tree ] && lib=opt_amd/libopt_amd.so
    envs=""
    [ "$v" != "$n" ] && envs=$(echo "${v#*@}" | tr '@' ' ')
    tag=$(echo "$v" | tr '@=/' '___')
    env $envs OPT_AMD_LIB=$lib timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline \
        > $O/$tag.$round.json 2> $O/$tag.$round.err || exit 1
    python3 -c "import json; d=json.load(open('$O/$tag.$round.json')); print('$v', $round, round(d['ms_per_step'],3), 'apply', round(d['roofline']['avg_us'],1), 'init', round(d.get('init_kernel',{}).get('avg_us',0),1))"
  done
done
