#!/bin/bash
# Quick GPU iteration: forward parity tests, then the C2 and fleet benches (no CPU
# baseline) and a kernel-trace summary of the fleet config.  Stops at the first
# failing step.  usage: tools/gpu_quick.sh TAG [pytest-targets...]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
TAG=${1:-quick}
shift || true
TESTS=${*:-tests/test_gpu_parity.py}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $TESTS -x -q -p no:cacheprovider --timeout 120 --timeout-method thread >"$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 300 python bench.py --no-cpu-baseline >"$OUT/bench_c2.json" 2>"$OUT/bench_c2.err" || { tail "$OUT/bench_c2.err"; exit 1; }
cat "$OUT/bench_c2.json"
timeout -k 10 300 python bench.py --config fleet --steps 20 --warmup 3 >"$OUT/bench_fleet.json" 2>"$OUT/bench_fleet.err" || { tail "$OUT/bench_fleet.err"; exit 1; }
cat "$OUT/bench_fleet.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_fleet" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --config fleet --steps 10 --warmup 2 >"$OUT/prof_fleet.log" 2>&1 || exit 1
grep -o '"void pgp[^"]*",[0-9]*,[0-9]*,[0-9.]*' "$OUT/prof_fleet/run_kernel_stats.csv"
