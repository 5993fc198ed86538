#!/bin/bash
# Every bench config once on one box (1 GPU), JSON lines into gpurun_out/<tag>/.
# usage: tools/all_configs.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/${1:-all}
mkdir -p "$OUT"
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python bench.py "$@" >"$OUT/$n.json" 2>"$OUT/$n.err"
  local rc=$?
  echo "[$n] rc=$rc $(cut -c1-160 "$OUT/$n.json")"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$n.err"; exit $rc; fi
}
run c2
run fleet --config fleet
run tune50 --config tune
run tune16 --config tune --hosts 16
run fpe --config fpe
run plugin --config plugin
run gobi --config gobi
run sim --config sim
run loop --config loop
