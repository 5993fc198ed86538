set -u
cd $GRAFT_REPO_ROOT
make -s > gpurun_out/bm_build.log 2>&1 || exit 3
mkdir -p gpurun_out/r01bm
timeout -k 10 300 python bench.py --config fleet --steps 20 --warmup 2 > gpurun_out/r01bm/fleet.json 2> gpurun_out/r01bm/fleet.err; echo "fleet rc=$?"; cat gpurun_out/r01bm/fleet.json
timeout -k 10 300 python bench.py --config tune --hosts 16 --steps 10 --warmup 2 > gpurun_out/r01bm/tune16.json 2> gpurun_out/r01bm/tune16.err; echo "tune16 rc=$?"; cat gpurun_out/r01bm/tune16.json
timeout -k 10 300 python bench.py --config tune --hosts 50 --steps 5 --warmup 1 > gpurun_out/r01bm/tune50.json 2> gpurun_out/r01bm/tune50.err; echo "tune50 rc=$?"; cat gpurun_out/r01bm/tune50.json; tail -3 gpurun_out/r01bm/tune50.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r01bm/prof_tune -o run --output-format csv -- python3 bench.py --config tune --hosts 50 --steps 3 --warmup 1 > gpurun_out/r01bm/prof_tune.log 2>&1; echo "prof rc=$?"
cat gpurun_out/r01bm/prof_tune/run_kernel_stats.csv | cut -c1-200 | head -12
