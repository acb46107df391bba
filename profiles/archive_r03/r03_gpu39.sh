#!/bin/bash
# GRU backward with a wave-uniform row index: backward tests, then A/B vs HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gru_fused_gpu.py -k "g4_backward" > gpurun_out/r03h_tests.log 2>&1 || { tail -30 gpurun_out/r03h_tests.log; exit 1; }
tail -1 gpurun_out/r03h_tests.log
bash profiles/r03_ab.sh 4 profiles/gru_bwd_only.py > gpurun_out/r03h_ab.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03h_ab.log
