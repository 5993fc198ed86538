#!/bin/bash
# stream-overlap check: the plugin / training GPU tests, then the C1, C3 and
# loop lines.  usage: tools/gpu_r03_ovl.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03_ovl}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_train.py tests/test_gpu_tunedp.py tests/test_gpu_dist.py tests/test_gpu_checkpoint.py \
  tests/test_gpu_plugin_graphs.py tests/test_gpu_repack.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r03_c13.sh ${1:-r03_ovl}
