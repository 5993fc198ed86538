#!/bin/bash
# session-3 close: GPU suite + smoke, the C2 line, the C3 line and its kernel
# stats.  usage: tools/gpu_r03_s3end.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
T=${1:-r03_s3end}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1
rc=$?; tail -1 $OUT/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py > $OUT/c2.json 2> $OUT/c2.err; rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --config tune --hosts 50 --steps 50 --warmup 5 > $OUT/tune50.json 2> $OUT/tune50.err; rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof_tune -o tune --output-format csv -- python3 bench.py --config tune --hosts 50 --steps 60 --warmup 10 --no-cpu-baseline > $OUT/prof_tune.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.load(open('$OUT/c2.json')); print('c2', d['ms_per_step'], d['value'], d['roofline']['frac'])"
python3 -c "import json; d=json.load(open('$OUT/tune50.json')); print('tune', d['ms_per_step'], d['value'], d['tune_model_ms'])"
