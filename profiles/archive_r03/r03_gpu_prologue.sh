#!/bin/bash
# GRU forward prologue waiting for step 0 only: GRU / network tests, forward A/B vs the previous build, stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gru_fused_gpu.py tests/test_gnn_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03x_tests.log 2>&1 || { tail -40 gpurun_out/r03x_tests.log; exit 1; }
tail -1 gpurun_out/r03x_tests.log
LIBS="base" GRU_KERNELS=h2r GRU_CHECKSUM=1 bash profiles/r03_ab_multi.sh 4 profiles/gru_r_bench.py > gpurun_out/r03x_ab_prologue.log 2>&1 || exit 1
MARLSAT_LIB=$PWD/ab/libmarlsat_stamp2.so timeout -k 10 300 python3 profiles/gru_stamps.py > gpurun_out/r03x_gru_stamps.log 2>&1 || exit 1
grep '^{' gpurun_out/r03x_gru_stamps.log
