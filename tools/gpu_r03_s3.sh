#!/bin/bash
# session 3 check: the GPU suite, the C3 line twice, a C3 kernel timeline.
# usage: tools/gpu_r03_s3.sh TAG [quick]
set -u
cd "$GRAFT_REPO_ROOT"
T=${1:-r03_s3}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${2:-}" = quick ]; then
  TESTS="tests/test_gpu_train.py tests/test_gpu_tunedp.py tests/test_gpu_dist.py tests/test_gpu_plugin_graphs.py"
else
  TESTS="tests -m gpu"
fi
timeout -k 10 900 python -u -m pytest $TESTS -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?; tail -1 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 200 python3 bench.py --config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline > $OUT/tune_$rep.json 2> $OUT/tune_$rep.err || { tail -3 $OUT/tune_$rep.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['stage_ms'].items()}, {k: round(v,4) for k,v in d['tune_model_ms'].items()}, round(d['roofline']['fused_total']['ms'],4))" $OUT/tune_$rep.json tune_$rep
done
timeout -k 10 180 rocprofv3 --kernel-trace -d $OUT/prof -o tune --output-format csv -- python3 bench.py --config tune --hosts 50 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/tl_tune.json 2> $OUT/tl_tune.err; rc=$?; [ $rc -eq 0 ] || exit $rc
f=$(find $OUT/prof -name '*kernel_trace.csv')
python3 tools/tune_timeline.py "$f" 8 > $OUT/timeline.txt 2>&1
sed -n 1,2p $OUT/timeline.txt
