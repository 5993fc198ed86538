#!/bin/bash
# Full GPU check of the committed tree: every -m gpu test (one process, per-test
# time limit), then smoke().  Stops at the first failing step.
# usage: tools/gpu_suite.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/${1:-suite}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  >"$OUT/gpu_tests.log" 2>&1
rc=$?
tail -3 "$OUT/gpu_tests.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" >"$OUT/smoke.log" 2>&1
rc=$?
tail -2 "$OUT/smoke.log"
exit $rc
