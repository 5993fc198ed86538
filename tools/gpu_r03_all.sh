#!/bin/bash
# full GPU suite + smoke, then the C2 line (no CPU baseline) and the C1 / C3 /
# loop lines.  usage: tools/gpu_r03_all.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03_all}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > $OUT/c2.json 2> $OUT/c2.err; rc=$?; cat $OUT/c2.json; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r03_c13.sh ${1:-r03_all}
