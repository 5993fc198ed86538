#!/bin/bash
# One GPU-box session: build, parity tests, smoke, bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; the script stops at the first step that
# faults, aborts or times out (anything but exit 0/1).
# usage: tools/gpu_session.sh [tag] [steps...]   steps: test smoke bench prof pmc
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
TAG=${1:-r01}
shift || true
STEPS=${*:-"test smoke bench prof"}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

ok_or_stop() {  # $1 = rc, $2 = name
  local rc=$1
  echo "[$2] rc=$rc" | tee -a "$OUT/status.txt"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
    echo "[$2] fatal rc=$rc -> stopping session" | tee -a "$OUT/status.txt"
    exit "$rc"
  fi
}

make -s >"$OUT/build.log" 2>&1 || { echo "build failed"; cat "$OUT/build.log"; exit 3; }

for st in $STEPS; do
  case $st in
    test)
      timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider >"$OUT/gpu_tests.log" 2>&1
      ok_or_stop $? test; tail -5 "$OUT/gpu_tests.log";;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" >"$OUT/smoke.log" 2>&1
      ok_or_stop $? smoke; tail -3 "$OUT/smoke.log";;
    bench)
      timeout -k 10 600 python bench.py >"$OUT/bench.json" 2>"$OUT/bench.err"
      ok_or_stop $? bench; cat "$OUT/bench.json";;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
        -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline >"$OUT/prof.log" 2>&1
      ok_or_stop $? prof
      find "$OUT/prof" -name "*kernel_stats.csv" -exec cat {} \; | head -20;;
    pmc)
      for C in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 600 rocprofv3 --pmc $C -d "$OUT/pmc_$C" -o run --output-format csv \
          -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline >"$OUT/pmc_$C.log" 2>&1
        ok_or_stop $? "pmc_$C"
      done;;
    fpetest)
      timeout -k 10 600 python -m pytest tests/test_gpu_fpe.py -x -q -p no:cacheprovider >"$OUT/gpu_fpe_tests.log" 2>&1
      ok_or_stop $? fpetest; tail -15 "$OUT/gpu_fpe_tests.log";;
    fpebench)
      timeout -k 10 600 python bench.py --config fpe >"$OUT/bench_fpe.json" 2>"$OUT/bench_fpe.err"
      ok_or_stop $? fpebench; cat "$OUT/bench_fpe.json";;
    fpeprof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_fpe" -o run --output-format csv \
        -- python3 "$ROOT/bench.py" --config fpe --steps 10 --warmup 2 --no-cpu-baseline >"$OUT/prof_fpe.log" 2>&1
      ok_or_stop $? fpeprof
      find "$OUT/prof_fpe" -name "*kernel_stats.csv" -exec cat {} \; | head -20;;
    *) echo "unknown step $st";;
  esac
done
echo "session done"
