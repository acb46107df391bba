#!/bin/bash
# h2s with linear weight-DMA addressing + uniform activation DMA: GRU tests, then A/B vs the previous build
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gru_fused_gpu.py -k "h2r or out_of_range" > gpurun_out/r03z_gru_tests.log 2>&1 || { tail -30 gpurun_out/r03z_gru_tests.log; exit 1; }
tail -2 gpurun_out/r03z_gru_tests.log
GRU_KERNELS=h2r bash profiles/r03_ab.sh 2 profiles/gru_r_bench.py > gpurun_out/r03z_ab.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03z_ab.log
