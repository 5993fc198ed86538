#!/bin/bash
# Round-5 GPU session steps.  usage: tools/gpu_r05.sh TAG STEP...
#   tests   GPU suite (+ smoke)
#   c2      C2 line (CPU baseline included) + rocprofv3 kernel stats
#   c2pmc   C2 FETCH_SIZE / WRITE_SIZE passes (traffic of K1, K2, K2b, K3)
#   c2stall C2 stall / MFMA-busy passes (K2, K3)
#   fleet   C5 line + FETCH / WRITE passes at its batch
#   tune    C3 lines (H=50, H=16) + rocprofv3 kernel stats of H=50
#   tunepmc C3 stall passes (H=50)
#   graphc  HIP graph branch concurrency / launch-cost probe
#   others  C4, C1, loop lines
# every GPU step runs under its own timeout; the script stops at the first failure
set -u
cd "$GRAFT_REPO_ROOT"
T=${1:?tag}
shift
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run NAME SECONDS CMD...
  local name=$1 secs=$2
  shift 2
  echo "[$name] $(date +%T) start"
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?
  echo "[$name] $(date +%T) rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $OUT/$name.err; tail -5 $OUT/$name.out; exit $rc; fi
}
pmc() {  # pmc NAME COUNTERS BENCH_ARGS...
  local name=$1 ctr=$2
  shift 2
  echo "[$name] $(date +%T) start"
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d $OUT/$name -o run --output-format csv -- python3 bench.py "$@" \
    > $OUT/$name.log 2>&1
  local rc=$?
  echo "[$name] $(date +%T) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
STALL1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
STALL2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
for step in "$@"; do
  case $step in
    tests)
      run gpu_tests 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
      tail -2 $OUT/gpu_tests.out
      run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
      ;;
    ttrain)
      run t_train 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_bench_modes.py tests/test_gpu_dist.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
      tail -2 $OUT/t_train.out
      ;;
    tc3)
      run t_c3 600 python -u -m pytest tests/test_gpu_c3step.py tests/test_gpu_tunedp.py tests/test_gpu_dist.py tests/test_gpu_plugin_graphs.py tests/test_gpu_train.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
      tail -2 $OUT/t_c3.out
      ;;
    tfpe)
      run t_fpe 600 python -u -m pytest tests/test_gpu_fpetrain.py tests/test_gpu_checkpoint.py -v -p no:cacheprovider --timeout 300 --timeout-method thread
      tail -2 $OUT/t_fpe.out
      ;;
    c2)
      run c2 400 python3 -u bench.py
      run prof_c2 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2 -o c2 --output-format csv -- python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline
      ;;
    c2pmc)
      pmc c2pmc1 FETCH_SIZE --steps 3 --warmup 1 --no-cpu-baseline
      pmc c2pmc2 WRITE_SIZE --steps 3 --warmup 1 --no-cpu-baseline
      ;;
    c2stall)
      pmc c2stall1 "$STALL1" --steps 3 --warmup 1 --no-cpu-baseline
      pmc c2stall2 "$STALL2" --steps 3 --warmup 1 --no-cpu-baseline
      ;;
    fleet)
      run fleet 400 python3 -u bench.py --config fleet --steps 100 --warmup 5
      pmc fleetpmc1 FETCH_SIZE --config fleet --steps 3 --warmup 1 --no-cpu-baseline
      pmc fleetpmc2 WRITE_SIZE --config fleet --steps 3 --warmup 1 --no-cpu-baseline
      ;;
    tune)
      run tune50 400 python3 -u bench.py --config tune --hosts 50 --steps 50 --warmup 5
      run tune16 400 python3 -u bench.py --config tune --hosts 16 --steps 50 --warmup 5
      run prof_tune 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_tune -o tune --output-format csv -- python3 bench.py --config tune --hosts 50 --steps 60 --warmup 10 --no-cpu-baseline
      run prof_tune16 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_tune16 -o tune --output-format csv -- python3 bench.py --config tune --hosts 16 --steps 60 --warmup 10 --no-cpu-baseline
      ;;
    tunepmc)
      pmc tunestall1 "$STALL1" --config tune --hosts 50 --steps 3 --warmup 1 --no-cpu-baseline
      pmc tunestall2 "$STALL2" --config tune --hosts 50 --steps 3 --warmup 1 --no-cpu-baseline
      ;;
    graphc)
      run graphc 120 python3 -u tools/graph_concurrency.py
      cat $OUT/graphc.out
      ;;
    abtune)
      grep median $OUT/ab16.out
      grep median $OUT/ab50.out
      ;;
    abtune2)
      grep median $OUT/ab16b.out
      grep median $OUT/ab50b.out
      ;;
    abdma)
      run abc2 600 python3 -u tools/ab_bench.py --rounds 3 --args "--steps 100 --warmup 10 --no-cpu-baseline" new= old=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_olddma.so
      grep median $OUT/abc2.out
      ;;
    abdw)
      run abdw 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" base= dw64=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_dw64.so dw64a=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_dw64a.so
      grep median $OUT/abdw.out
      run prof_dw 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_dw -o tune --output-format csv -- python3 bench.py --config tune --hosts 50 --steps 30 --warmup 5 --no-cpu-baseline
      PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_dw64a.so run prof_dw64a 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_dw64a -o tune --output-format csv -- python3 bench.py --config tune --hosts 50 --steps 30 --warmup 5 --no-cpu-baseline
      ;;
    abprev)
      run abp50 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" new= prev=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_prev.so
      grep median $OUT/abp50.out
      run abp16 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 16 --steps 100 --warmup 10 --no-cpu-baseline" new= prev=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_prev.so
      grep median $OUT/abp16.out
      ;;
    abpp)
      run pp_quick_base 180 python -u -m pytest tests/test_gpu_parity.py -k "not census" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
      PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_k2pp.so run pp_quick 180 python -u -m pytest tests/test_gpu_parity.py -k "not census" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
      PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_k3pp.so run pp_quick_k3 180 python -u -m pytest tests/test_gpu_parity.py -k "not census" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
      tail -2 $OUT/pp_quick.out
      run abpp 600 python3 -u tools/ab_bench.py --rounds 3 --args "--steps 100 --warmup 10 --no-cpu-baseline" base= k2pp=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_k2pp.so k3pp=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_k3pp.so
      grep median $OUT/abpp.out
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); [print(k, [{kk: round(vv, 4) for kk, vv in e['kernel_ms'].items()} for e in v]) for k, v in d['extra'].items()]" $OUT/abpp.out
      run abtfpp 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" base= tfpp=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_tfpp.so
      grep median $OUT/abtfpp.out
      ;;
    abfull)
      run abfull50 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" base= fullreg=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_fullreg.so
      grep median $OUT/abfull50.out
      run abfull16 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 16 --steps 100 --warmup 10 --no-cpu-baseline" base= fullreg=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_fullreg.so
      grep median $OUT/abfull16.out
      PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_fullreg.so run prof_full 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_full -o tune --output-format csv -- python3 bench.py --config tune --hosts 50 --steps 30 --warmup 5 --no-cpu-baseline
      ;;
    abloop)
      grep median $OUT/abloop.out
      ;;
    profloop)
      run prof_loop 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_loop -o loop --output-format csv -- python3 bench.py --config loop --steps 20 --warmup 3 --no-cpu-baseline
      PGP_BENCH_ONE_STREAM=1 run prof_loop1 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_loop1 -o loop --output-format csv -- python3 bench.py --config loop --steps 20 --warmup 3 --no-cpu-baseline
      ;;
    loop)
      run loop 300 python3 -u bench.py --config loop --steps 20 --warmup 3
      ;;
    abgraph)
      run abg16 600 python3 -u tools/ab_bench.py --rounds 4 --args "--config tune --hosts 16 --steps 100 --warmup 10 --no-cpu-baseline" eager= graph=PGP_BENCH_GRAPH=1
      grep median $OUT/abg16.out
      run abg50 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" eager= graph=PGP_BENCH_GRAPH=1
      grep median $OUT/abg50.out
      ;;
    gobi)
      run tgobi 300 python3 -u -m pytest tests/test_gpu_gobi.py -x -v --timeout 120 --timeout-method thread -m gpu
      run gobi1 120 python3 -u bench.py --config gobi --steps 50 --warmup 5 --no-cpu-baseline
      run gobi2 120 python3 -u bench.py --config gobi --steps 50 --warmup 5 --no-cpu-baseline
      run loopg 300 python3 -u bench.py --config loop --steps 20 --warmup 3 --no-cpu-baseline
      grep -h -o '"ms_per_step": [0-9.]*\|"mean_iterations": [0-9.]*' $OUT/gobi1.out $OUT/gobi2.out $OUT/loopg.out
      ;;
    abspread)
      run tbal 600 python3 -u -m pytest tests/test_gpu_c3step.py tests/test_gpu_tunedp.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread -m gpu
      run abs50 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" balanced= spread=PGP_TF_SPREAD=1
      grep median $OUT/abs50.out
      run abs16 600 python3 -u tools/ab_bench.py --rounds 4 --args "--config tune --hosts 16 --steps 100 --warmup 10 --no-cpu-baseline" balanced= spread=PGP_TF_SPREAD=1
      grep median $OUT/abs16.out
      run absloop 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config loop --steps 20 --warmup 3 --no-cpu-baseline" balanced= spread=PGP_TF_SPREAD=1
      grep median $OUT/absloop.out
      ;;
    abres)
      grep median $OUT/abr16.out
      grep median $OUT/abr50.out
      grep median $OUT/abrloop.out
      ;;
    abside2)
      PGP_TUNE_SIDE_EARLY=15 run tside2 600 python3 -u -m pytest tests/test_gpu_c3step.py tests/test_gpu_tunedp.py -x -q --timeout 120 --timeout-method thread -m gpu
      run abe2 900 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" e3= e7=PGP_TUNE_SIDE_EARLY=7 e11=PGP_TUNE_SIDE_EARLY=11 e15=PGP_TUNE_SIDE_EARLY=15
      grep median $OUT/abe2.out
      ;;
    cprof)
      run cprof16 300 python3 -u -m cProfile -o $OUT/cprof16.pstats bench.py --config tune --hosts 16 --steps 400 --warmup 10 --no-cpu-baseline
      python3 -c "import pstats; p=pstats.Stats('$OUT/cprof16.pstats'); p.sort_stats('tottime').print_stats(40)" > $OUT/cprof16_tottime.txt
      python3 -c "import pstats; p=pstats.Stats('$OUT/cprof16.pstats'); p.sort_stats('cumtime').print_stats(60)" > $OUT/cprof16_cumtime.txt
      ;;
    host)
      run thost 600 python3 -u -m pytest tests/test_gpu_c3step.py tests/test_gpu_tunedp.py tests/test_gpu_train.py tests/test_gpu_bench_modes.py -x -q --timeout 120 --timeout-method thread -m gpu
      run h16a 120 python3 -u bench.py --config tune --hosts 16 --steps 200 --warmup 10 --no-cpu-baseline
      run h16b 120 python3 -u bench.py --config tune --hosts 16 --steps 200 --warmup 10 --no-cpu-baseline
      run h50a 120 python3 -u bench.py --config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline
      run hloop 300 python3 -u bench.py --config loop --steps 20 --warmup 3 --no-cpu-baseline
      grep -h -o '"ms_per_step": [0-9.]*\|"host_issue_ms_per_step": [0-9.]*' $OUT/h16a.out $OUT/h16b.out $OUT/h50a.out $OUT/hloop.out
      ;;
    late)
      PGP_C3_GAN_LATE=1 run tlate 600 python3 -u -m pytest tests/test_gpu_c3step.py tests/test_gpu_bench_modes.py -x -q --timeout 120 --timeout-method thread -m gpu
      run abl16 600 python3 -u tools/ab_bench.py --rounds 4 --args "--config tune --hosts 16 --steps 100 --warmup 10 --no-cpu-baseline" early= late=PGP_C3_GAN_LATE=1
      grep median $OUT/abl16.out
      run abl50 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" early= late=PGP_C3_GAN_LATE=1
      grep median $OUT/abl50.out
      run cprofloop 300 python3 -u -m cProfile -o $OUT/cprofloop.pstats bench.py --config loop --steps 40 --warmup 3 --no-cpu-baseline
      python3 -c "import pstats; p=pstats.Stats('$OUT/cprofloop.pstats'); p.sort_stats('tottime').print_stats(50)" > $OUT/cprofloop_tottime.txt
      python3 -c "import pstats; p=pstats.Stats('$OUT/cprofloop.pstats'); p.sort_stats('cumtime').print_stats('preganplus_amd|bench', 60)" > $OUT/cprofloop_cumtime.txt
      ;;
    abdec)
      run tdec 600 python3 -u -m pytest tests/test_gpu_c3step.py tests/test_gpu_tunedp.py tests/test_gpu_tune1.py tests/test_gpu_train_model.py -x -q --timeout 120 --timeout-method thread -m gpu
      run abd50 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" new= prev=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_prevdec.so
      grep median $OUT/abd50.out
      run abd16 600 python3 -u tools/ab_bench.py --rounds 4 --args "--config tune --hosts 16 --steps 100 --warmup 10 --no-cpu-baseline" new= prev=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_prevdec.so
      grep median $OUT/abd16.out
      run prof_dec 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_dec -o tune --output-format csv -- python3 bench.py --config tune --hosts 50 --steps 30 --warmup 5 --no-cpu-baseline
      ;;
    abzero)
      run tzero 600 python3 -u -m pytest tests/test_gpu_c3step.py tests/test_gpu_bench_modes.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread -m gpu
      run abz16 600 python3 -u tools/ab_bench.py --rounds 4 --args "--config tune --hosts 16 --steps 100 --warmup 10 --no-cpu-baseline" zside= zmain=PGP_C3_ZERO_SIDE=0
      grep median $OUT/abz16.out
      run abz50 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" zside= zmain=PGP_C3_ZERO_SIDE=0
      grep median $OUT/abz50.out
      ;;
    abmin)
      run abm16 600 python3 -u tools/ab_bench.py --rounds 4 --args "--config tune --hosts 16 --steps 100 --warmup 10 --no-cpu-baseline" nofork= fork=PGP_TUNE_SIDE_MIN_TOKENS=1
      grep median $OUT/abm16.out
      ;;
    abdws)
      PGP_TUNE_DEC_DWS=1 run tdws 600 python3 -u -m pytest tests/test_gpu_c3step.py tests/test_gpu_tunedp.py -x -q --timeout 120 --timeout-method thread -m gpu
      run abdws50 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" p4= p2=PGP_TUNE_DEC_DWS=2 p1=PGP_TUNE_DEC_DWS=1
      grep median $OUT/abdws50.out
      ;;
    state)
      run tstate 600 python3 -u -m pytest tests/test_gpu_tunedp.py tests/test_gpu_c3step.py tests/test_gpu_train.py tests/test_gpu_dist.py tests/test_gpu_plugin_graphs.py -x -q --timeout 120 --timeout-method thread -m gpu
      run st50 120 python3 -u bench.py --config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline
      run st16 120 python3 -u bench.py --config tune --hosts 16 --steps 100 --warmup 10 --no-cpu-baseline
      run prof_st 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_st -o tune --output-format csv -- python3 bench.py --config tune --hosts 50 --steps 30 --warmup 5 --no-cpu-baseline
      grep -h -o '"ms_per_step": [0-9.]*' $OUT/st50.out $OUT/st16.out
      ;;
    ds)
      run tds 600 python3 -u -m pytest tests/test_gpu_tunedp.py tests/test_gpu_c3step.py tests/test_gpu_train.py tests/test_gpu_plugin_graphs.py -x -q --timeout 120 --timeout-method thread -m gpu
      run ds50 120 python3 -u bench.py --config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline
      run ds16 120 python3 -u bench.py --config tune --hosts 16 --steps 100 --warmup 10 --no-cpu-baseline
      run prof_ds 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_ds -o tune --output-format csv -- python3 bench.py --config tune --hosts 50 --steps 30 --warmup 5 --no-cpu-baseline
      run prof_ds16 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_ds16 -o tune --output-format csv -- python3 bench.py --config tune --hosts 16 --steps 30 --warmup 5 --no-cpu-baseline
      grep -h -o '"ms_per_step": [0-9.]*' $OUT/ds50.out $OUT/ds16.out
      ;;
    abflush)
      run tflush 600 python3 -u -m pytest tests/test_gpu_c3step.py tests/test_gpu_tunedp.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread -m gpu
      run abf50 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" early= late=PGP_TUNE_EARLY_FLUSH=0
      grep median $OUT/abf50.out
      ;;
    abe15)
      run abe15 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" e7= e15=PGP_TUNE_SIDE_EARLY=15
      grep median $OUT/abe15.out
      ;;
    roofchk)
      run rc50 120 python3 -u bench.py --config tune --hosts 50 --steps 20 --warmup 3 --no-cpu-baseline
      run rc16 120 python3 -u bench.py --config tune --hosts 16 --steps 50 --warmup 5 --no-cpu-baseline
      python3 -c "import json; [print(json.dumps({k: v for k, v in json.loads(open('$OUT/' + f + '.out').read().strip().splitlines()[-1])['roofline'].items() if k != 'basis'})) for f in ('rc50', 'rc16')]"
      ;;
    tunetraffic)
      pmc tunepmcf FETCH_SIZE --config tune --hosts 50 --steps 3 --warmup 1 --no-cpu-baseline
      pmc tunepmcw WRITE_SIZE --config tune --hosts 50 --steps 3 --warmup 1 --no-cpu-baseline
      ;;
    gp)
      run tgp 600 python3 -u -m pytest tests/test_gpu_tunedp.py tests/test_gpu_c3step.py tests/test_gpu_train.py tests/test_gpu_dist.py tests/test_gpu_plugin_graphs.py tests/test_gpu_tune1.py tests/test_gpu_train_model.py tests/test_gpu_bench_modes.py -x -q --timeout 120 --timeout-method thread -m gpu
      run gp50 120 python3 -u bench.py --config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline
      run gp16 120 python3 -u bench.py --config tune --hosts 16 --steps 100 --warmup 10 --no-cpu-baseline
      run prof_gp 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_gp -o tune --output-format csv -- python3 bench.py --config tune --hosts 50 --steps 30 --warmup 5 --no-cpu-baseline
      grep -h -o '"ms_per_step": [0-9.]*' $OUT/gp50.out $OUT/gp16.out
      ;;
    tc3q)
      run tc3q 600 python3 -u -m pytest tests/test_gpu_c3step.py tests/test_gpu_tunedp.py tests/test_gpu_train.py tests/test_gpu_dist.py tests/test_gpu_plugin_graphs.py tests/test_gpu_bench_modes.py -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider
      tail -2 $OUT/tc3q.out
      run q16 120 python3 -u bench.py --config tune --hosts 16 --steps 200 --warmup 10 --no-cpu-baseline
      run q50 120 python3 -u bench.py --config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline
      grep -h -o '"ms_per_step": [0-9.]*\|"host_issue_ms_per_step": [0-9.]*' $OUT/q16.out $OUT/q50.out
      python3 -c "import json; [print(f, json.loads(open('$OUT/' + f + '.out').read().strip().splitlines()[-1])['train_gan_alone']['ms']) for f in ('q16', 'q50')]"
      ;;
    prof16)
      run prof16 240 rocprofv3 --kernel-trace --stats -d $OUT/prof16 -o tune --output-format csv -- python3 bench.py --config tune --hosts 16 --steps 60 --warmup 10 --no-cpu-baseline
      PGP_BENCH_ONE_STREAM=1 run one16 120 python3 -u bench.py --config tune --hosts 16 --steps 200 --warmup 10 --no-cpu-baseline
      grep -h -o '"ms_per_step": [0-9.]*\|"host_issue_ms_per_step": [0-9.]*' $OUT/one16.out
      ;;
    prof50)
      run p50b 120 python3 -u bench.py --config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline
      grep -h -o '"ms_per_step": [0-9.]*' $OUT/p50b.out
      run prof50 240 rocprofv3 --kernel-trace --stats -d $OUT/prof50 -o tune --output-format csv -- python3 bench.py --config tune --hosts 50 --steps 40 --warmup 5 --no-cpu-baseline
      ;;
    ffn8)
      PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_ffn8.so run ffn8 120 python3 -u bench.py --config tune --hosts 50 --steps 30 --warmup 5 --no-cpu-baseline
      run ffn4 120 python3 -u bench.py --config tune --hosts 50 --steps 30 --warmup 5 --no-cpu-baseline
      python3 -c "import json; [print(f, json.dumps({k: round(v['ms'],4) for k, v in json.loads(open('$OUT/' + f + '.out').read().strip().splitlines()[-1])['roofline']['fused_launches'].items()})) for f in ('ffn8', 'ffn4')]"
      ;;
    native)
      run tnat 600 python3 -u -m pytest tests/test_gpu_c3step.py tests/test_gpu_dist.py -x -v --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider
      run n16 120 python3 -u bench.py --config tune --hosts 16 --steps 200 --warmup 10 --no-cpu-baseline
      run n50 120 python3 -u bench.py --config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline
      grep -h -o '"ms_per_step": [0-9.]*\|"host_issue_ms_per_step": [0-9.]*' $OUT/n16.out $OUT/n50.out
      run prof_n16 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_n16 -o tune --output-format csv -- python3 bench.py --config tune --hosts 16 --steps 60 --warmup 10 --no-cpu-baseline
      ;;
    base)
      run b16 120 python3 -u bench.py --config tune --hosts 16 --steps 200 --warmup 10 --no-cpu-baseline
      run b50 120 python3 -u bench.py --config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline
      run bc2 200 python3 -u bench.py --steps 100 --warmup 10 --no-cpu-baseline
      grep -h -o '"ms_per_step": [0-9.]*\|"host_issue_ms_per_step": [0-9.]*' $OUT/b16.out $OUT/b50.out $OUT/bc2.out
      ;;
    ckpt)
      run ckpt 300 python3 -u -m pytest tests/test_gpu_checkpoint.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
      tail -3 $OUT/ckpt.out
      ;;
    abearly)
      L=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var
      run abearly 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" base= e5=PGP_LIB=$L/libpreganplus_e5.so e13=PGP_LIB=$L/libpreganplus_e13.so e15=PGP_LIB=$L/libpreganplus_e15.so
      tail -6 $OUT/abearly.out
      ;;
    gobidx)
      L=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var
      run gdx1 300 python3 -u tools/dbg/gobi_ab.py $L/libpreganplus_dxbase.so
      run gdx2 300 python3 -u tools/dbg/gobi_ab.py $L/libpreganplus_dxpref.so
      run gdx3 300 python3 -u tools/dbg/gobi_ab.py $L/libpreganplus_gobi7.so
      cat $OUT/gdx1.out $OUT/gdx2.out $OUT/gdx3.out
      ;;
    abgs2)
      L=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var
      run abgs16 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 16 --steps 100 --warmup 10 --no-cpu-baseline" base= gs2=PGP_LIB=$L/libpreganplus_gs2.so
      grep median $OUT/abgs16.out
      python3 -c "import json; d=json.loads(open('$OUT/abgs16.out').read().strip().splitlines()[-1]); print({k: [x.get('train_gan_alone') for x in v] for k, v in d.get('extra', {}).items()})"
      ;;
    abdx)
      L=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var
      run abdec50 600 python3 -u tools/ab_bench.py --rounds 4 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" new= old=PGP_LIB=$L/libpreganplus_decold.so
      run abdec16 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 16 --steps 100 --warmup 10 --no-cpu-baseline" new= old=PGP_LIB=$L/libpreganplus_decold.so
      grep median $OUT/abdec50.out $OUT/abdec16.out
      ;;
    dist2)  # the driver's N > 1 path rehearsed with two gloo ranks on the one GPU (c3_dp sub-record included)
      PGP_DIST_BACKEND=gloo PGP_DEVICE=0 run dist2 600 python3 -u bench.py --gpus 2 --steps 20 --warmup 3
      python3 -c "import json; d=json.loads(open('$OUT/dist2.out').read().strip().splitlines()[-1]); print(d['n_gpus'], d['ranks_seen'], d['ms_per_step'], {k: (v.get('ms_per_step'), v.get('ranks_seen')) for k, v in d.get('sub_records', d.get('sub', {})).items()} if isinstance(d.get('sub_records', d.get('sub', {})), dict) else list(d.keys()))"
      ;;
    abffn)
      L=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var
      run abffn50 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" base= f124=PGP_LIB=$L/libpreganplus_ffn124.so f132=PGP_LIB=$L/libpreganplus_ffn132.so
      run abffn16 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 16 --steps 100 --warmup 10 --no-cpu-baseline" base= f124=PGP_LIB=$L/libpreganplus_ffn124.so f132=PGP_LIB=$L/libpreganplus_ffn132.so
      grep median $OUT/abffn50.out $OUT/abffn16.out
      ;;
    fcal)  # FETCH_SIZE / WRITE_SIZE per access width (tools/micro/fetch_cal.hip)
      for c in FETCH_SIZE WRITE_SIZE; do
        echo "[fcal $c] $(date +%T)"
        timeout -s KILL 60 rocprofv3 --pmc $c -d $OUT/fcal_$c -o run --output-format csv -- ./tools/micro/fetch_cal \
          > $OUT/fcal_$c.log 2>&1 || { tail -5 $OUT/fcal_$c.log; exit 1; }
      done
      ;;
    gobiab)
      run gobitest 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_gobi.py
      run gobiab 300 python3 -u tools/dbg/gobi_ab.py $GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_gobi7.so
      cat $OUT/gobiab.out
      PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_gprof.so run gphase 120 python3 -u tools/gobi_phases.py
      cat $OUT/gphase.out
      run gobib 200 python3 -u bench.py --config gobi --steps 50 --warmup 5 --no-cpu-baseline
      run loopb 300 python3 -u bench.py --config loop --steps 20 --warmup 3 --no-cpu-baseline
      ;;
    gobi8ab)  # the in-tree GOBI against the round-5 v8 build (bit-identical results and timing), phases
      run gobitest 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_gobi.py
      run gobiab 300 python3 -u tools/dbg/gobi_ab.py $GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_gobi8.so
      cat $OUT/gobiab.out
      PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_gprof.so run gphase 120 python3 -u tools/gobi_phases.py
      cat $OUT/gphase.out
      ;;
    gobivs)  # the in-tree GOBI against variant $GOBI_VS (bit-identical results and timing)
      run gobivs 300 python3 -u tools/dbg/gobi_ab.py $GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_$GOBI_VS.so
      cat $OUT/gobivs.out
      ;;
    ginv)  # GOBI batch invariance probe, in-tree and variant $GOBI_VS
      run ginv 120 python3 -u tools/dbg/gobi_inv.py
      PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_$GOBI_VS.so run ginvvs 120 python3 -u tools/dbg/gobi_inv.py
      cat $OUT/ginv.out $OUT/ginvvs.out
      ;;
    abk3)  # C2 A/B: in-tree vs variant k3old, then the census parity tests
      L=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var
      run abk3 600 python3 -u tools/ab_bench.py --rounds 4 --args "--steps 100 --warmup 10 --no-cpu-baseline" new= old=PGP_LIB=$L/libpreganplus_k3old.so
      grep median $OUT/abk3.out
      run k3par 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_decide.py
      tail -2 $OUT/k3par.out
      ;;
    abt)  # C3 A/B, H = 16 and 50: in-tree vs variant $TV, then the C3 parity tests
      L=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var
      run abt16 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 16 --steps 100 --warmup 10 --no-cpu-baseline" new= old=PGP_LIB=$L/libpreganplus_$TV.so
      run abt50 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" new= old=PGP_LIB=$L/libpreganplus_$TV.so
      grep median $OUT/abt16.out $OUT/abt50.out
      run tc3par 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_c3step.py tests/test_gpu_tunedp.py tests/test_gpu_train.py
      tail -2 $OUT/tc3par.out
      ;;
    stalls)  # one PMC pass per config with tools/pmc_stalls.py's counter set: C3 H = 50 and C2
      SC="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
      pmc stall_tune50 "$SC" --config tune --hosts 50 --steps 3 --warmup 1 --no-cpu-baseline
      pmc stall_c2 "$SC" --steps 3 --warmup 1 --no-cpu-baseline
      for n in stall_tune50 stall_c2; do
        f=$(find $OUT/$n -name "*counter_collection.csv" | head -1)
        python3 tools/pmc_stalls.py "$f" > $OUT/$n.txt && cat $OUT/$n.txt
      done
      ;;
    trepack)  # the repack tests, then the loop line
      run trepack 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_repack.py tests/test_gpu_loop.py
      tail -2 $OUT/trepack.out
      run loopb 300 python3 -u bench.py --config loop --steps 20 --warmup 3 --no-cpu-baseline
      python3 -c "import json; d=json.loads(open('$OUT/loopb.out').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('stage_ms'))"
      ;;
    abk3w)  # K3 waves per workgroup at small batches: the loop line (1,024 windows) and the K3 tests
      L=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var
      run k3wpar 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_decide.py tests/test_gpu_loop.py
      tail -2 $OUT/k3wpar.out
      run abk3w 900 python3 -u tools/ab_bench.py --rounds 3 --args "--config loop --steps 20 --warmup 3 --no-cpu-baseline" w4= w1=PGP_LIB=$L/libpreganplus_k3w1.so w2=PGP_LIB=$L/libpreganplus_k3w2.so w8=PGP_LIB=$L/libpreganplus_k3w8.so w16=PGP_LIB=$L/libpreganplus_k3w16.so
      grep median $OUT/abk3w.out
      ;;
    abdws2)  # the decoder weight gradient's window split S: in-tree (4) vs 1 and 2
      L=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var
      run abdws50 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" s4= s1=PGP_LIB=$L/libpreganplus_dws1.so s2=PGP_LIB=$L/libpreganplus_dws2.so
      run abdws16 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 16 --steps 100 --warmup 10 --no-cpu-baseline" s4= s1=PGP_LIB=$L/libpreganplus_dws1.so s2=PGP_LIB=$L/libpreganplus_dws2.so
      grep median $OUT/abdws50.out $OUT/abdws16.out
      ;;
    abdeclate)  # the decoders' weight gradient forked after layer 1's FFN backward (variant declate) vs after the targets
      L=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var
      run abdl50 600 python3 -u tools/ab_bench.py --rounds 4 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" base= late=PGP_LIB=$L/libpreganplus_declate.so
      grep median $OUT/abdl50.out
      ;;
    abpack)  # the decoder weight packing forked after the layer-0 forward (variant packlate) vs after the dataset
      L=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var
      run abpk50 600 python3 -u tools/ab_bench.py --rounds 4 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" base= late=PGP_LIB=$L/libpreganplus_packlate.so
      grep median $OUT/abpk50.out
      ;;
    abearly2)  # the side-work mask after the round-5 moves: 7 (in-tree) vs 15 and 3
      L=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var
      run abe2 600 python3 -u tools/ab_bench.py --rounds 4 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" e7= e15=PGP_LIB=$L/libpreganplus_e15.so e3=PGP_LIB=$L/libpreganplus_e3.so
      grep median $OUT/abe2.out
      ;;
    gphase)
      PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_gprof.so run gphase 120 python3 -u tools/gobi_phases.py
      cat $OUT/gphase.out
      ;;
    gphase8)  # the same for the round-5 v8 kernel (variant gprof8)
      PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_gprof8.so run gphase8 120 python3 -u tools/gobi_phases.py
      cat $OUT/gphase8.out
      ;;
    others)
      run fpe 300 python3 -u bench.py --config fpe --steps 100 --warmup 5
      run plugin 300 python3 -u bench.py --config plugin --steps 50 --warmup 5
      run loop 300 python3 -u bench.py --config loop --steps 20 --warmup 3
      run gobi 300 python3 -u bench.py --config gobi --steps 50 --warmup 5
      ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo done
