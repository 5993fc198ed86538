#!/bin/bash
# two-rank C3 rehearsal variants: library side stream off / bench GAN stream off
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03_dist2t
mkdir -p $OUT
for v in "A PGP_TUNE_SIDE_STREAM=1 PGP_BENCH_ONE_STREAM=0" "B PGP_TUNE_SIDE_STREAM=0 PGP_BENCH_ONE_STREAM=0" "C PGP_TUNE_SIDE_STREAM=1 PGP_BENCH_ONE_STREAM=1" "D PGP_TUNE_SIDE_STREAM=0 PGP_BENCH_ONE_STREAM=1"; do
  set -- $v
  n=$1; shift
  env "$@" PGP_DIST_BACKEND=gloo PGP_DEVICE=0 timeout -k 10 200 python3 bench.py --config tune --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline \
    > $OUT/t_$n.json 2> $OUT/t_$n.err; rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/t_$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$OUT/t_$n.json')); print('$n $*', round(d['ms_per_step'],3), {k: round(x,3) for k,x in d['stage_ms'].items()})"
done
echo done
