#!/bin/bash
# 32x32x16 one-wave-per-SIMD GRU forward (MARLSAT_GRU_WIDE=1): parity tests, then A/B timing vs the 16x16x32 kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
MARLSAT_GRU_WIDE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gru_fused_gpu.py -k "h2r or out_of_range" > gpurun_out/r03w_gru_tests.log 2>&1 || { tail -30 gpurun_out/r03w_gru_tests.log; exit 1; }
tail -3 gpurun_out/r03w_gru_tests.log
for i in 1; do for wd in 0 1; do
echo "== wide $wd" >> gpurun_out/r03w_gru_bench.log
MARLSAT_GRU_WIDE=$wd GRU_KERNELS=h2r timeout -k 10 120 python -u profiles/gru_r_bench.py >> gpurun_out/r03w_gru_bench.log 2>&1 || exit 1
done; done
cat gpurun_out/r03w_gru_bench.log
