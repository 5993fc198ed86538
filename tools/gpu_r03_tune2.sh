#!/bin/bash
# C3: the training-path GPU tests, the tune line and a kernel trace.  usage: tools/gpu_r03_tune2.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03_tune2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_train.py tests/test_gpu_tunedp.py tests/test_gpu_dist.py tests/test_gpu_plugin_graphs.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 -u bench.py --config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline > $OUT/tune50.json 2> $OUT/tune50.err; rc=$?; cat $OUT/tune50.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --config tune --hosts 50 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
echo done
