#!/bin/bash
# A/B of library variants on one tools/bench_families.py config, interleaved twice:
#   tools/ab_family.sh <outdir> <config> v1 v2 ...   (through gpurun, repo root)
# a variant is <name> (build_ab/<name>/libopt_amd.so, "tree" = opt_amd/libopt_amd.so)
# optionally followed by @VAR=value[@VAR=value...] environment settings.
O=gpurun_out/$1; C=$2; shift 2
mkdir -p $O
for round in 1 2; do
  for v in "$@"; do
    n=${v%%@*}
    lib=build_ab/$n/libopt_amd.so
    [ "$n" = tree ] && lib=opt_amd/libopt_amd.so
    envs=""
    [ "$v" != "$n" ] && envs=$(echo "${v#*@}" | tr '@' ' ')
    tag=$(echo "$v" | tr '@=/' '___')
    env $envs OPT_AMD_LIB=$lib timeout -k 10 300 python3 tools/bench_families.py --only $C \
        --out $O/$tag.$round.json > $O/$tag.$round.log 2>&1 || exit 1
    python3 -c "import json; d=json.load(open('$O/$tag.$round.json'))[0]; print('$v', $round, 'apply', round(d['apply_us'],2), 'frac', round(d['roofline']['frac'],3), 'step', round(d['step_ms'],4), d.get('cost_after'))"
  done
done
