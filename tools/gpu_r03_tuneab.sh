#!/bin/bash
# C3 A/B over library variants (PGP_LIB): training tests on the default
# library, then the tune line per variant, twice.  usage: tools/gpu_r03_tuneab.sh TAG v1 [v2 ...]
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03_tuneab${1:-}
mkdir -p $OUT
shift || true
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_train.py tests/test_gpu_tunedp.py tests/test_gpu_dist.py > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in base "$@"; do
  if [ "$v" = base ]; then lib=preganplus_amd/_lib/libpreganplus.so; else lib=preganplus_amd/_lib/var/libpreganplus_$v.so; fi
  PGP_LIB=$lib timeout -k 10 180 python3 -u bench.py --config tune --steps 50 --warmup 5 --no-cpu-baseline > $OUT/t_$v.$rep.json 2> $OUT/t_$v.$rep.err; rc=$?
  [ $rc -eq 0 ] || { tail -5 $OUT/t_$v.$rep.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$OUT/t_$v.$rep.json')); print('$v', round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['tune_model_ms'].items()}, {k: round(x['ms'],4) for k,x in d['roofline']['fused_launches'].items()})"
done
done
echo done
