#!/bin/bash
# One profiling session of the headline config (C2): the bench line, the
# rocprofv3 kernel-trace summary of the SAME command, then PMC passes (each in
# its own run, --pmc only): HBM FETCH_SIZE, WRITE_SIZE, and the stall split.
# usage: tools/prof_session.sh TAG [bench args...]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
TAG=${1:-prof}
shift || true
ARGS=${*:-}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py $ARGS >"$OUT/bench.json" 2>"$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" $ARGS >"$OUT/trace_bench.json" 2>"$OUT/trace.err" || { tail "$OUT/trace.err"; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/pmc$i" -o run --output-format csv \
     -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline $ARGS >"$OUT/pmc$i.log" 2>&1
  rc=$?
  echo "[pmc$i] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
echo done
