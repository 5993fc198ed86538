#!/bin/bash
# end-of-session evidence: GPU suite + smoke, the C2 line (CPU baseline
# included) with its kernel trace, the C3 line with its kernel trace, PMC
# passes (C2 traffic; C3 counters).  usage: tools/gpu_r03_end.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
T=${1:-r03_end}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py > $OUT/c2.json 2> $OUT/c2.err; rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2 -o c2 --output-format csv -- python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline > $OUT/prof_c2.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --config tune --hosts 50 --steps 50 --warmup 5 > $OUT/tune50.json 2> $OUT/tune50.err; rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof_tune -o tune --output-format csv -- python3 bench.py --config tune --hosts 50 --steps 60 --warmup 10 --no-cpu-baseline > $OUT/prof_tune.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r03_c2pmc.sh $T/c2pmc || exit $?
BENCH_ARGS="--config tune --hosts 50 --steps 3 --warmup 1 --no-cpu-baseline" bash tools/gpu_r03_pmc.sh $T/tunepmc || exit $?
echo done
