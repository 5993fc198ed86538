#!/bin/bash
# C3 tuning step: GPU tests of the training path, the bench line (with the
# live fused-kernel roofline and the CPU baseline) and a kernel trace
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03_tune${1:-}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_train.py tests/test_gpu_tunedp.py tests/test_gpu_dist.py > $OUT/tests.log 2>&1
rc=$?; grep -E "passed|failed|FAIL|Error" $OUT/tests.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 -u bench.py --config tune --hosts 50 --steps 50 --warmup 5 > $OUT/tune50.json 2> $OUT/tune50.err; rc=$?; cat $OUT/tune50.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --config tune --hosts 50 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
echo done
