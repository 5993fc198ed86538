#!/bin/bash
# C2 HBM traffic per kernel: FETCH_SIZE and WRITE_SIZE passes (separate runs,
# counters only).  usage: tools/gpu_r03_c2pmc.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03_c2pmc}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc$i.log 2>&1
  rc=$?; echo "[pmc$i: $grp] rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/pmc$i.log; exit $rc; }
done
echo done
