#!/bin/bash
# round 3 session 1: MFMA rate micro, save_gan / census tests, C1 bench, --gpus 2 rehearsal
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03_s1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 ./tools/micro/mfma_rate > $OUT/mfma_rate.txt 2>&1; rc=$?; cat $OUT/mfma_rate.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_checkpoint.py "tests/test_gpu_parity.py::test_full_size_census" > $OUT/tests.log 2>&1
rc=$?; tail -15 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/census_*.json $OUT/ 2>/dev/null
timeout -k 10 300 python3 bench.py --config plugin --steps 200 --warmup 10 --no-cpu-baseline > $OUT/plugin.json 2> $OUT/plugin.err; rc=$?; cat $OUT/plugin.json; [ $rc -eq 0 ] || exit $rc
for cfg in c2 tune fleet; do
  PGP_DIST_BACKEND=gloo PGP_DEVICE=0 timeout -k 10 300 python3 bench.py --config $cfg --gpus 2 --steps 10 --warmup 2 \
    > $OUT/dist2_$cfg.json 2> $OUT/dist2_$cfg.err; rc=$?; tail -1 $OUT/dist2_$cfg.json; [ $rc -eq 0 ] || exit $rc
done
echo done
