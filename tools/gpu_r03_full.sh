#!/bin/bash
# round-3 full check: every -m gpu test, smoke(), then the C2 line with its
# CPU baseline and a C2 kernel trace.  usage: tools/gpu_r03_full.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03_full}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py > $OUT/c2.json 2> $OUT/c2.err; rc=$?; cat $OUT/c2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c2 --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
echo done
