#!/bin/bash
# C2 A/B over library variants (PGP_LIB): the bench line's K2..K5 kernel times
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03_c2ab${1:-}
mkdir -p $OUT
shift || true
for v in base "$@"; do
  if [ "$v" = base ]; then lib=preganplus_amd/_lib/libpreganplus.so; else lib=preganplus_amd/_lib/var/libpreganplus_$v.so; fi
  PGP_LIB=$lib timeout -k 10 180 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c2_$v.json 2> $OUT/c2_$v.err; rc=$?
  [ $rc -eq 0 ] || { tail -5 $OUT/c2_$v.err; exit $rc; }
  python3 -c "import json,sys; d=json.load(open('$OUT/c2_$v.json')); print('$v', round(d['ms_per_step'],3), {k: round(x,3) for k,x in d['kernel_ms'].items()}, round(d['roofline']['frac'],3))"
done
echo done
