#!/bin/bash
# fused tuning encoder: A/B against the token-major build, training parity
# tests, then the C3 bench + kernel trace
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03_tf${1:-}
mkdir -p $OUT
export TMPDIR=/tmp
if [ -f preganplus_amd/_lib/var/libpreganplus_tm.so ]; then
  for H in 16 50; do
    timeout -k 10 120 python3 tools/tf_compare.py dump $OUT/new_h$H.npz $H 37 && \
    PGP_LIB=preganplus_amd/_lib/var/libpreganplus_tm.so timeout -k 10 120 python3 tools/tf_compare.py dump $OUT/old_h$H.npz $H 37 && \
    python3 tools/tf_compare.py compare $OUT/new_h$H.npz $OUT/old_h$H.npz > $OUT/compare_h$H.txt; rc=$?
    tail -3 $OUT/compare_h$H.txt; [ $rc -eq 0 ] || exit $rc
  done
fi
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_train.py tests/test_gpu_tunedp.py tests/test_gpu_dist.py > $OUT/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error" $OUT/tests.log | tail -40; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline > $OUT/tune50.json 2> $OUT/tune50.err; rc=$?; cat $OUT/tune50.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --config tune --hosts 50 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
echo done
