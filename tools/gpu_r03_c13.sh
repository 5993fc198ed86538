#!/bin/bash
# C1 plugin latency and the C3 tuning line (no tests).  usage: tools/gpu_r03_c13.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03_c13}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 python3 -u bench.py --config plugin > $OUT/plugin.json 2> $OUT/plugin.err; rc=$?; cat $OUT/plugin.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 -u bench.py --config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline > $OUT/tune50.json 2> $OUT/tune50.err; rc=$?; cat $OUT/tune50.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 -u bench.py --config loop --steps 50 --warmup 5 --no-cpu-baseline > $OUT/loop.json 2> $OUT/loop.err; rc=$?; cat $OUT/loop.json; [ $rc -eq 0 ] || exit $rc
echo done
