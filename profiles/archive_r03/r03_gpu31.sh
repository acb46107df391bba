#!/bin/bash
# GRU backward with fast gates + DPP wave reductions: backward / network parity tests, then A/B timing
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gru_fused_gpu.py tests/test_gnn_gpu.py -k "g4_backward or depth16 or uf200 or forward_backward" > gpurun_out/r03w_bwd_tests.log 2>&1 || { tail -40 gpurun_out/r03w_bwd_tests.log; exit 1; }
tail -2 gpurun_out/r03w_bwd_tests.log
bash profiles/r03_ab.sh 3 profiles/gru_bwd_only.py > gpurun_out/r03w_bwd_ab.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03w_bwd_ab.log
