#!/bin/bash
# PMC passes over the C3 tuning step (one counter group per rocprofv3 run,
# counters only, as MI355X_MICROARCH.md prescribes).  usage: tools/gpu_r03_pmc.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03_pmc}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--config tune --hosts 50 --steps 3 --warmup 1 --no-cpu-baseline"}
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU" \
           "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc$i.log 2>&1
  rc=$?; echo "[pmc$i: $grp] rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/pmc$i.log; exit $rc; }
done
echo done
