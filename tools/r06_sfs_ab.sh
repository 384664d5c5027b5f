#!/bin/bash
# Round 6: the shape_from_shading bench leg for each A/B variant (env settings as tools/ab_run.sh:
# tree@VAR=value@...), twice, interleaved on one box:  tools/r06_sfs_ab.sh <outdir> v1 v2 ...
O=gpurun_out/$1; shift
mkdir -p $O
for round in 1 2; do
  for v in "$@"; do
    envs=""
    [ "$v" != "${v%%@*}" ] && envs=$(echo "${v#*@}" | tr '@' ' ')
    tag=$(echo "$v" | tr '@=/' '___')
    env $envs timeout -k 10 150 python3 bench.py --workload shape_from_shading --steps 10 --warmup 2 --no-cpu-baseline \
        > $O/$tag.$round.json 2> $O/$tag.$round.err || exit 1
    python3 -c "import json; d=json.load(open('$O/$tag.$round.json')); print('$v', $round, round(d['ms_per_step'],3), {k: round(x['avg_us'],1) for k, x in d.get('step_kernels', {}).items()})"
  done
done
