#!/bin/bash
# A/B of the default library against variants on one box, interleaved:
#   tools/ab_bench.sh TAG "bench args" var1 [var2 ...]   (variants: preganplus_amd/_lib/var/libpreganplus_<v>.so)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
TAG=$1; ARGS=$2; shift 2
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2 3; do
  for v in base "$@"; do
    if [ "$v" = base ]; then lib=$ROOT/preganplus_amd/_lib/libpreganplus.so; else lib=$ROOT/preganplus_amd/_lib/var/libpreganplus_$v.so; fi
    PGP_LIB=$lib timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline >"$OUT/$v.$rep.json" 2>"$OUT/$v.$rep.err" || { tail "$OUT/$v.$rep.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],4), round(d['value'],1), {k: round(v,4) for k,v in d.get('kernel_ms',{}).items()})" "$OUT/$v.$rep.json" "$v.$rep"
  done
done
