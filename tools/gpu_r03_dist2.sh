#!/bin/bash
# two-rank rehearsal (gloo, both ranks on the one GPU) of the C2, C3, fleet and
# loop bench paths via `bench.py --gpus 2` (the launcher starts the ranks)
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03_dist2}
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in c2 tune fleet loop; do
  PGP_DIST_BACKEND=gloo PGP_DEVICE=0 timeout -k 10 300 python3 bench.py --config $cfg --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline \
    > $OUT/dist2_$cfg.json 2> $OUT/dist2_$cfg.err; rc=$?; tail -c 300 $OUT/dist2_$cfg.json; echo; [ $rc -eq 0 ] || { tail -5 $OUT/dist2_$cfg.err; exit $rc; }
done
echo done
