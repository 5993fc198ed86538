#!/bin/bash
# training-path GPU tests, then the C3 line with the GAN step issued after
# the tuning step (0) or right after detect (1), interleaved; then a timeline.
# usage: tools/gpu_r03_s3b.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
T=${1:-r03_s3b}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
TESTS="tests -m gpu"
timeout -k 10 600 python -u -m pytest $TESTS -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?; tail -1 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for ge in 0; do
    PGP_BENCH_GAN_EARLY=$ge timeout -k 10 200 python3 bench.py --config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline > $OUT/tune_g${ge}_$rep.json 2> $OUT/tune_g${ge}_$rep.err || { tail -3 $OUT/tune_g${ge}_$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['stage_ms'].items()}, {k: round(v,4) for k,v in d['tune_model_ms'].items()}, round(d['roofline']['fused_total']['ms'],4))" $OUT/tune_g${ge}_$rep.json g${ge}_$rep
  done
done
timeout -k 10 180 rocprofv3 --kernel-trace -d $OUT/prof -o tune --output-format csv -- python3 bench.py --config tune --hosts 50 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/tl_tune.json 2> $OUT/tl_tune.err; rc=$?; [ $rc -eq 0 ] || exit $rc
f=$(find $OUT/prof -name '*kernel_trace.csv')
python3 tools/tune_timeline.py "$f" 8 > $OUT/timeline.txt 2>&1
sed -n 1,2p $OUT/timeline.txt
