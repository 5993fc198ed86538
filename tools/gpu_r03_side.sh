#!/bin/bash
# C3 A/B: detect issue point (start / after the tuning forward), the
# backward's side work early (beside the fused launches) or in the tail, and
# the fused kernels at raised wave priority (variant "prio").
# usage: tools/gpu_r03_side.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
T=${1:-r03_side}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
TESTS="tests/test_gpu_train.py tests/test_gpu_tunedp.py tests/test_gpu_dist.py tests/test_gpu_plugin_graphs.py"
PGP_TUNE_SIDE_EARLY=1 timeout -k 10 300 python -u -m pytest $TESTS -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests_early.txt 2>&1; rc=$?; tail -1 $OUT/tests_early.txt; [ $rc -eq 0 ] || exit $rc
run() {  # name lib detect_at early
  local lib=preganplus_amd/_lib/libpreganplus.so
  [ "$2" = base ] || lib=preganplus_amd/_lib/var/libpreganplus_$2.so
  PGP_LIB=$lib PGP_BENCH_DETECT_AT=$3 PGP_TUNE_SIDE_EARLY=$4 timeout -k 10 200 python3 bench.py --config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline > $OUT/$1.json 2> $OUT/$1.err || { tail -3 $OUT/$1.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['stage_ms'].items()}, {k: round(v,4) for k,v in d['tune_model_ms'].items()}, round(d['roofline']['fused_total']['ms'],4))" $OUT/$1.json $1
}
for rep in 1 2; do
  run start_$rep base start 0 && run fwd_$rep base forward 0 && run fwd_early_$rep base forward 1 && run fwd_prio_$rep prio forward 0 && run fwd_early_prio_$rep prio forward 1 || exit 1
done | tee $OUT/ab.txt
