set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03_base
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline > $OUT/tune50.json 2> $OUT/tune50.err && cat $OUT/tune50.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_tune -o run --output-format csv -- python3 bench.py --config tune --hosts 50 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof_tune.log 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline > $OUT/c2.json 2> $OUT/c2.err && cat $OUT/c2.json
