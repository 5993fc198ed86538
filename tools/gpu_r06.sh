#!/bin/bash
# Round-6 GPU session steps.  usage: tools/gpu_r06.sh TAG STEP...
#   tests   GPU suite (+ smoke)
#   tfpe4   C4 GPU tests only (H=16 and H=50 fixtures, oracle, census)
#   fpe     C4 lines (H=50, H=16) + rocprofv3 kernel stats of both
#   fpepmc  K4 stall / VALU passes (H=50)
#   c2      C2 line (CPU baseline included) + rocprofv3 kernel stats
#   c2stall C2 stall / MFMA-busy passes (K2, K3)
#   tune    C3 lines (H=50, H=16) + rocprofv3 kernel stats
#   fleet   C5 lines (resident and streamed)
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
PYT="python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread"
for step in "$@"; do
  case $step in
    tests)
      run gpu_tests 1100 $PYT tests -m gpu
      tail -2 $OUT/gpu_tests.out
      run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
      ;;
    micro)
      run bf16split 120 tools/micro/bf16_split 256 7680
      cat $OUT/bf16split.out
      ;;
    tdec)
      run t_dec 900 $PYT tests/test_gpu_parity.py -m gpu -k "split or reference_fixtures or ragged or stage_split or census"
      tail -2 $OUT/t_dec.out
      ;;
    c2ab)
      run c2split 300 python3 -u bench.py --steps 100 --warmup 5 --no-cpu-baseline
      run c2fp32 300 python3 -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --fp32-decoder --fp32-gan
      run c2fp32g 300 python3 -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --fp32-gan
      grep -h -o "\"ms_per_step\": [0-9.]*\|\"decoder\": [0-9.]*\|\"gan\": [0-9.]*" $OUT/c2split.out $OUT/c2fp32.out $OUT/c2fp32g.out
      ;;
    traffic)  # FETCH / WRITE passes of the C2 kernels at H=50 and 16 (tools/pmc_traffic.py gpurun_out/T/trH B H)
      mkdir -p $OUT/tr50 $OUT/tr16
      pmc tr50/pmc_fetch FETCH_SIZE --steps 3 --warmup 1 --no-cpu-baseline
      pmc tr50/pmc_write WRITE_SIZE --steps 3 --warmup 1 --no-cpu-baseline
      pmc tr16/pmc_fetch FETCH_SIZE --hosts 16 --steps 3 --warmup 1 --no-cpu-baseline
      pmc tr16/pmc_write WRITE_SIZE --hosts 16 --steps 3 --warmup 1 --no-cpu-baseline
      ;;
    trtune)  # FETCH / WRITE passes of the fused tuning kernels (tools/pmc_traffic.py gpurun_out/T/trt50 1030 50)
      mkdir -p $OUT/trt50
      pmc trt50/pmc_fetch FETCH_SIZE --config tune --hosts 50 --steps 3 --warmup 1 --no-cpu-baseline
      pmc trt50/pmc_write WRITE_SIZE --config tune --hosts 50 --steps 3 --warmup 1 --no-cpu-baseline
      ;;
    stamps)  # phase stamps of the fused tuning kernels (profiling build st)
      PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_st.so run st50 300 python3 -u tools/tf_stamps.py 50 1030
      PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_st.so run st16 300 python3 -u tools/tf_stamps.py 16 1030
      cat $OUT/st16.out
      ;;
    tline)  # C3 kernel traces (H=50, 16) -> per-step timelines
      run tl50 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/tl50 -o tl -- python3 bench.py --config tune --hosts 50 --steps 40 --warmup 5 --no-cpu-baseline
      run tl16 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/tl16 -o tl -- python3 bench.py --config tune --hosts 16 --steps 100 --warmup 10 --no-cpu-baseline
      for h in 50 16; do python3 tools/tune_timeline.py $(find $OUT/tl$h -name "*kernel_trace.csv" | head -1) > $OUT/timeline$h.txt; head -3 $OUT/timeline$h.txt; done
      ;;
    abtf)  # fused tuning kernels: split-bf16 (default build) vs fp32 (variant tfs0)
      run abtf 900 python3 -u tools/ab_bench.py --rounds 4 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" split= fp32=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_tfs0.so
      grep median $OUT/abtf.out
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); [print(k, [{kk: round(vv, 4) for kk, vv in e['stage_ms'].items()} for e in v]) for k, v in d['extra'].items()]" $OUT/abtf.out
      ;;
    abatt)  # attention backward restructure (out_proj dW outside, Win^T split) vs the previous build (head)
      run abatt 900 python3 -u tools/ab_bench.py --rounds 4 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" new= head=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_head.so
      grep median $OUT/abatt.out
      ;;
    abdecpipe)  # decoder plane reads pinned a tile ahead (variant decpipe) vs the default build
      run abdp 900 python3 -u tools/ab_bench.py --rounds 5 --args "--steps 100 --warmup 5 --no-cpu-baseline" base= pipe=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_decpipe.so
      grep median $OUT/abdp.out
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); [print(k, [round(e['kernel_ms']['decoder'], 4) for e in v]) for k, v in d['extra'].items()]" $OUT/abdp.out
      ;;
    abdepth)  # decoder plane-read depth: 1 (default build) vs 2, 3
      run abdd 900 python3 -u tools/ab_bench.py --rounds 4 --args "--steps 100 --warmup 5 --no-cpu-baseline" d1= d2=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_dp2.so d3=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_dp3.so
      grep median $OUT/abdd.out
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); [print(k, [round(e['kernel_ms']['decoder'], 4) for e in v]) for k, v in d['extra'].items()]" $OUT/abdd.out
      ;;
    abdp0)  # decoder plane pipeline (default build) vs none (dp0); forward plane prefetch (fwdpf) on C3
      run abd0 900 python3 -u tools/ab_bench.py --rounds 4 --args "--steps 100 --warmup 5 --no-cpu-baseline" pipe= none=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_dp0.so
      grep median $OUT/abd0.out
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); [print(k, [round(e['kernel_ms']['decoder'], 4) for e in v]) for k, v in d['extra'].items()]" $OUT/abd0.out
      run abfpf 900 python3 -u tools/ab_bench.py --rounds 4 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" base= fwdpf=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_fwdpf.so
      grep median $OUT/abfpf.out
      ;;
    gobiab)  # GOBI: bit-identical trajectories and kernel time against the previous build (gobi0); GPU tests; lines
      run gobiab 600 python3 -u tools/dbg/gobi_ab.py $GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_gobi0.so
      tail -5 $OUT/gobiab.out
      run t_gobi 600 $PYT tests/test_gpu_gobi.py tests/test_gpu_loop.py -m gpu
      tail -2 $OUT/t_gobi.out
      run gobi 400 python3 -u bench.py --config gobi --steps 20 --warmup 3
      run loop 400 python3 -u bench.py --config loop --steps 50 --warmup 5
      ;;
    gobiph)  # GOBI phase timing (profiling build gprof)
      PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_gprof.so run gobiph 300 python3 -u tools/gobi_phases.py
      cat $OUT/gobiph.out
      ;;
    dist2)  # N=2 rehearsal on one GPU: two gloo ranks, the C2 line with its c3_dp sub-record
      PGP_DIST_BACKEND=gloo PGP_DEVICE=0 run dist2 600 python3 -u bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu-baseline
      grep "^{" $OUT/dist2.out | tail -1 | cut -c1-400
      ;;
    abencpipe)  # K2 split feed-forward planes pinned a (block, tile) ahead (variant encpipe)
      run abep 900 python3 -u tools/ab_bench.py --rounds 5 --args "--steps 100 --warmup 5 --no-cpu-baseline" base= pipe=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_encpipe.so
      grep median $OUT/abep.out
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); [print(k, [round(e['kernel_ms']['encoder'], 4) for e in v]) for k, v in d['extra'].items()]" $OUT/abep.out
      ;;
    abencf32)  # K2 fp32 GEMMs' A fragments one ahead (variant encf32): C2 (H=50) and fleet (H=16)
      run abef 900 python3 -u tools/ab_bench.py --rounds 5 --args "--steps 100 --warmup 5 --no-cpu-baseline" base= f32pf=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_encf32.so
      grep median $OUT/abef.out
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); [print(k, [round(e['kernel_ms']['encoder'], 4) for e in v]) for k, v in d['extra'].items()]" $OUT/abef.out
      run abeff 900 python3 -u tools/ab_bench.py --rounds 4 --args "--config fleet --steps 50 --warmup 5 --no-cpu-baseline" base= f32pf=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_encf32.so
      grep median $OUT/abeff.out
      ;;
    abbff)  # FFN backward split GEMMs' planes one ahead (variant bffpf)
      run abbff 900 python3 -u tools/ab_bench.py --rounds 5 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" base= bffpf=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_bffpf.so
      grep median $OUT/abbff.out
      ;;
    abtw)  # K3: two blocks of 16 windows per wave (default build) vs one (tw1)
      run abtw 900 python3 -u tools/ab_bench.py --rounds 4 --args "--steps 100 --warmup 5 --no-cpu-baseline" tw2= tw1=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_tw1.so
      grep median $OUT/abtw.out
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); [print(k, [round(e['kernel_ms']['gan'], 4) for e in v]) for k, v in d['extra'].items()]" $OUT/abtw.out
      ;;
    abk3pf)  # K3 one-hot containers: planes read a step ahead (default build) vs not (pf0); C2 at H=50 and H=16
      run abk3 900 python3 -u tools/ab_bench.py --rounds 4 --args "--steps 100 --warmup 5 --no-cpu-baseline" pf= pf0=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_pf0.so
      grep median $OUT/abk3.out
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); [print(k, [round(e['kernel_ms']['gan'], 4) for e in v]) for k, v in d['extra'].items()]" $OUT/abk3.out
      run abk316 900 python3 -u tools/ab_bench.py --rounds 3 --args "--hosts 16 --steps 100 --warmup 5 --no-cpu-baseline" pf= pf0=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_pf0.so
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); [print(k, [round(e['kernel_ms']['gan'], 4) for e in v]) for k, v in d['extra'].items()]" $OUT/abk316.out
      ;;
    abtouch)  # C3: prefetched unit inputs taken before the unit's stores (default build) vs not (touch0)
      run abtouch 900 python3 -u tools/ab_bench.py --rounds 4 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" touch= touch0=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_touch0.so
      grep median $OUT/abtouch.out
      run abtouch16 900 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 16 --steps 100 --warmup 10 --no-cpu-baseline" touch= touch0=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_touch0.so
      grep median $OUT/abtouch16.out
      ;;
    abdecready)  # K2b: each tile's planes waited for before the next tile's reads (default build) vs not (rd0); depth 2 (dp2)
      run abdr 900 python3 -u tools/ab_bench.py --rounds 4 --args "--steps 100 --warmup 5 --no-cpu-baseline" ready= rd0=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_rd0.so dp2=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_dp2.so
      grep median $OUT/abdr.out
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); [print(k, [round(e['kernel_ms']['decoder'], 4) for e in v]) for k, v in d['extra'].items()]" $OUT/abdr.out
      ;;
    abenc)
      run abenc 900 python3 -u tools/ab_bench.py --rounds 4 --args "--steps 100 --warmup 5 --no-cpu-baseline" split= fp32enc=ARGS=--fp32-encoder
      grep median $OUT/abenc.out
      ;;
    tfleet)
      run t_fleet 600 $PYT tests/test_gpu_fleet_stream.py -m gpu
      tail -2 $OUT/t_fleet.out
      run fleet 400 python3 -u bench.py --config fleet --steps 100 --warmup 5 --no-cpu-baseline
      ;;
    abissue)
      run t_c3 600 $PYT tests/test_gpu_c3step.py -m gpu
      run abi16 600 python3 -u tools/ab_bench.py --rounds 4 --args "--config tune --hosts 16 --steps 100 --warmup 10 --no-cpu-baseline" worker= serial=PGP_BENCH_SERIAL_ISSUE=1
      grep median $OUT/abi16.out
      run abi50 600 python3 -u tools/ab_bench.py --rounds 3 --args "--config tune --hosts 50 --steps 50 --warmup 5 --no-cpu-baseline" worker= serial=PGP_BENCH_SERIAL_ISSUE=1
      grep median $OUT/abi50.out
      ;;
    abbwd)
      PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_bwdfirst.so run t_bwd 600 $PYT tests/test_gpu_c3step.py -m gpu
      run abb16 600 python3 -u tools/ab_bench.py --rounds 4 --args "--config tune --hosts 16 --steps 100 --warmup 10 --no-cpu-baseline" base= bwd=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_bwdfirst.so
      grep median $OUT/abb16.out
      ;;
    tdist)
      run t_dist 600 $PYT tests/test_gpu_dist.py -m gpu
      tail -2 $OUT/t_dist.out
      ;;
    ttrain)
      run t_train 900 $PYT tests/test_gpu_train.py tests/test_gpu_c3step.py tests/test_gpu_dist.py -m gpu
      tail -2 $OUT/t_train.out
      ;;
    abdec)
      run abdec 900 python3 -u tools/ab_bench.py --rounds 5 --args "--steps 100 --warmup 5 --no-cpu-baseline" base= tw2=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_dectw2.so
      grep median $OUT/abdec.out
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); [print(k, [{kk: round(vv, 4) for kk, vv in e['kernel_ms'].items()} for e in v]) for k, v in d['extra'].items()]" $OUT/abdec.out
      ;;
    tbr)
      run t_br 600 $PYT tests/test_gpu_parity.py -m gpu -k "branches or split"
      tail -2 $OUT/t_br.out
      ;;
    tfpe4)
      run t_fpe4 900 $PYT tests/test_gpu_fpe.py -m gpu
      tail -2 $OUT/t_fpe4.out
      ;;
    fpe)
      run fpe50 400 python3 -u bench.py --config fpe --hosts 50 --steps 100 --warmup 5
      run fpe16 400 python3 -u bench.py --config fpe --hosts 16 --steps 100 --warmup 5
      run prof_fpe50 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_fpe50 -o fpe --output-format csv -- python3 bench.py --config fpe --hosts 50 --steps 60 --warmup 10 --no-cpu-baseline
      run prof_fpe16 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_fpe16 -o fpe --output-format csv -- python3 bench.py --config fpe --hosts 16 --steps 60 --warmup 10 --no-cpu-baseline
      ;;
    abpf)
      run abpf 900 python3 -u tools/ab_bench.py --rounds 5 --args "--steps 100 --warmup 5 --no-cpu-baseline" base= pf2=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_decpf2.so
      grep median $OUT/abpf.out
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); [print(k, [{kk: round(vv, 4) for kk, vv in e['kernel_ms'].items()} for e in v]) for k, v in d['extra'].items()]" $OUT/abpf.out
      ;;
    k3probe)
      run k3probe 900 python3 -u tools/ab_bench.py --rounds 2 --args "--steps 50 --warmup 5 --no-cpu-baseline" base= nop2=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_k3p1.so nop3=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_k3p2.so norow=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_k3p3.so oh0=PGP_LIB=$GRAFT_REPO_ROOT/preganplus_amd/_lib/var/libpreganplus_k3oh0.so
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); [print(k, [round(e['kernel_ms']['gan'], 4) for e in v]) for k, v in d['extra'].items()]" $OUT/k3probe.out
      ;;
    tmodes)
      run t_modes 600 $PYT tests/test_gpu_bench_modes.py tests/test_gpu_parity.py -m gpu -k "stream or split or branches or reference or ragged or onehot"
      tail -2 $OUT/t_modes.out
      ;;
    c2l2)
      pmc c2l2 "TCC_HIT_sum TCC_MISS_sum" --steps 3 --warmup 1 --no-cpu-baseline
      pmc c2fetch FETCH_SIZE --steps 3 --warmup 1 --no-cpu-baseline
      ;;
    fpepmc)
      pmc fpestall1 "$STALL1" --config fpe --hosts 50 --steps 3 --warmup 1 --no-cpu-baseline
      pmc fpestall2 "$STALL2" --config fpe --hosts 50 --steps 3 --warmup 1 --no-cpu-baseline
      ;;
    c2)
      run c2 400 python3 -u bench.py
      run prof_c2 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2 -o c2 --output-format csv -- python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline
      ;;
    c2stall)
      pmc c2stall1 "$STALL1" --steps 3 --warmup 1 --no-cpu-baseline
      pmc c2stall2 "$STALL2" --steps 3 --warmup 1 --no-cpu-baseline
      ;;
    tune)
      run tune50 400 python3 -u bench.py --config tune --hosts 50 --steps 50 --warmup 5
      run tune16 400 python3 -u bench.py --config tune --hosts 16 --steps 50 --warmup 5
      run prof_tune 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_tune -o tune --output-format csv -- python3 bench.py --config tune --hosts 50 --steps 60 --warmup 10 --no-cpu-baseline
      run prof_tune16 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_tune16 -o tune --output-format csv -- python3 bench.py --config tune --hosts 16 --steps 60 --warmup 10 --no-cpu-baseline
      ;;
    fleet)
      run fleet 400 python3 -u bench.py --config fleet --steps 100 --warmup 5
      run fleets 400 python3 -u bench.py --config fleet --stream --steps 20 --warmup 2 --no-cpu-baseline
      ;;
    tunestall)
      pmc tstall1 "$STALL1" --config tune --hosts 50 --steps 3 --warmup 1 --no-cpu-baseline
      pmc tstall2 "$STALL2" --config tune --hosts 50 --steps 3 --warmup 1 --no-cpu-baseline
      ;;
    lines)  # the other configs' lines: GOBI, the online loop, the plugin, the simulation
      run gobi 400 python3 -u bench.py --config gobi --steps 20 --warmup 3
      run loop 400 python3 -u bench.py --config loop --steps 50 --warmup 5
      run plugin 400 python3 -u bench.py --config plugin --steps 20 --warmup 3
      run sim 400 python3 -u bench.py --config sim --steps 50 --warmup 5
      ;;
    *)
      echo "unknown step $step"; exit 2
      ;;
  esac
done
echo DONE
