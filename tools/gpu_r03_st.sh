#!/bin/bash
# phase stamps of the fused tuning-encoder kernels (profiling build)
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03_st${1:-}
mkdir -p $OUT
PGP_LIB=preganplus_amd/_lib/var/libpreganplus_st.so timeout -k 10 120 python3 -u tools/tf_stamps.py 50 1030 > $OUT/stamps.txt 2>&1; rc=$?; cat $OUT/stamps.txt; exit $rc
