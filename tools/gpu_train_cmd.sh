set -u
cd $GRAFT_REPO_ROOT
make -s > gpurun_out/train_build.log 2>&1 || exit 3
mkdir -p gpurun_out/r01t
timeout -k 10 900 python -m pytest tests/test_gpu_train.py tests/test_gpu_parity.py -x -q -p no:cacheprovider > gpurun_out/r01t/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -30 gpurun_out/r01t/tests.log
