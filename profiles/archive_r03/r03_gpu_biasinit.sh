#!/bin/bash
# GRU forward accumulators initialised at the biases: GRU / network oracle tests, then forward A/B vs the
# previous build (ab/libmarlsat_base.so) on the round-2 kernel shapes, tape on and off
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gru_fused_gpu.py tests/test_gnn_gpu.py tests/test_mappo_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03v_tests.log 2>&1 || { tail -40 gpurun_out/r03v_tests.log; exit 1; }
tail -1 gpurun_out/r03v_tests.log
LIBS="base" GRU_KERNELS=h2r bash profiles/r03_ab_multi.sh 4 profiles/gru_r_bench.py > gpurun_out/r03v_ab_bias_init.log 2>&1 || exit 1
