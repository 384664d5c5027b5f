# Fused update + cost variants under rocprofv3 (kernel stats per variant):
#   bash tools/r03_fcost_sweep.sh <tag> v1 v2 ...   (variant syntax as tools/ab_run.sh)
R=$(pwd)
O=$R/gpurun_out/$1; shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  n=${v%%@*}
  lib=$R/build_exp/$n/libopt_amd.so
  [ "$n" = tree ] && lib=$R/opt_amd/libopt_amd.so
  tag=$(echo "$v" | tr '@=/' '___')
  if [ "$v" != "$n" ]; then for kv in $(echo "${v#*@}" | tr '@' ' '); do export "$kv"; done; fi
  OPT_AMD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv -- \
      python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || exit 1
  if [ "$v" != "$n" ]; then for kv in $(echo "${v#*@}" | tr '@' ' '); do unset "${kv%%=*}"; done; fi
  python3 - "$O/$tag" "$v" <<'PY'
import csv, glob, sys, json
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
rows = {r["Name"].split("(")[0].replace("void optamd::iw::", ""): float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f))}
d = json.loads(open(sys.argv[1] + ".json").read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 3), {k: round(v, 1) for k, v in rows.items() if "cost" in k or "update" in k})
PY
done
