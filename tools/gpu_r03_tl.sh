#!/bin/bash
# C3 kernel timeline: a kernel trace of the tune bench, cut into steps by
# tools/tune_timeline.py.  usage: tools/gpu_r03_tl.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
T=${1:-r03_tl}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $OUT/prof -o tune --output-format csv -- python3 bench.py --config tune --hosts 50 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/tune.json 2> $OUT/tune.err; rc=$?; [ $rc -eq 0 ] || exit $rc
f=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
python3 tools/tune_timeline.py "$f" 8 > $OUT/timeline.txt 2>&1

sed -n 1,90p $OUT/timeline.txt
