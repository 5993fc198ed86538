#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --pmc only with --kernel-trace-free
# collection as MI355X_MICROARCH.md prescribes).  usage: tools/pmc_session.sh TAG "grp1" "grp2" ...
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
TAG=$1; shift
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
make -s >"$OUT/build.log" 2>&1 || exit 3
BENCH_ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu-baseline"}
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d "$OUT/pmc$i" -o run --output-format csv \
     -- python3 "$ROOT/bench.py" $BENCH_ARGS >"$OUT/pmc$i.log" 2>&1
  rc=$?
  echo "[pmc$i: $grp] rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/pmc$i.log"; exit $rc; fi
done
echo done
