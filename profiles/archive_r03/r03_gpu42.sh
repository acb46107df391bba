#!/bin/bash
# GRU forward with the hidden steps last (h read from the slots at the epilogue, no h refetch) and two
# static step copies: GRU + network tests, A/B timing, PMC traffic
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gru_fused_gpu.py tests/test_gnn_gpu.py > gpurun_out/r03k_tests.log 2>&1 || { tail -40 gpurun_out/r03k_tests.log; exit 1; }
tail -1 gpurun_out/r03k_tests.log
GRU_KERNELS=h2r bash profiles/r03_ab.sh 3 profiles/gru_r_bench.py > gpurun_out/r03k_ab.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03k_ab.log
bash profiles/pmc_gru_traffic.sh > gpurun_out/r03k_pmc.log 2>&1 || { tail -20 gpurun_out/r03k_pmc.log; exit 1; }
cp gpurun_out/pmc_gru_traffic.json gpurun_out/r03k_pmc_gru.json
rm -rf gpurun_out/pmc_gru_traffic
grep -E "pmc_over|launch_us" gpurun_out/r03k_pmc_gru.json
