#!/bin/bash
# GPU session for the tuning step (C3): parity tests, bench at H=50/16, kernel trace.
# usage: tools/gpu_tune_session.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/${1:-tune}
mkdir -p "$OUT"
export TMPDIR=/tmp
stop() { echo "[$1] rc=$2"; if [ "$2" -ne 0 ] && [ "$2" -ne 1 ]; then echo "fatal -> stop"; exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > "$OUT/tests.log" 2>&1
rc=$?; tail -25 "$OUT/tests.log"; stop tests $rc
for H in 50 16; do
  timeout -k 10 300 python bench.py --config tune --hosts $H --steps 20 --warmup 3 > "$OUT/bench_tune$H.json" \
    2> "$OUT/bench_tune$H.err"
  rc=$?; cat "$OUT/bench_tune$H.json"; stop bench$H $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
  -- python3 bench.py --config tune --hosts 50 --steps 10 --warmup 2 > "$OUT/prof.log" 2>&1
rc=$?; stop prof $rc
find "$OUT/prof" -name "*kernel_stats.csv" -exec head -45 {} \;
