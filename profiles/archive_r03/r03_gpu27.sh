#!/bin/bash
# SQ counters + timing: 32x32 one-wave-per-SIMD GRU forward (wide 1) vs the 16x16x32 kernel (wide 0)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for wd in 0 1; do
MARLSAT_GRU_WIDE=$wd GRU_KERNELS=h2r GRU_TAPE=False timeout -k 10 120 python -u profiles/gru_r_bench.py >> gpurun_out/r03x_gru_bench.log 2>&1 || exit 1
MARLSAT_GRU_WIDE=$wd GRU_KERNELS=h2r GRU_TAPE=False GRU_REPS=2 timeout -k 10 300 bash profiles/pmc_sq.sh gruw$wd $GRAFT_REPO_ROOT/profiles/gru_r_bench.py > gpurun_out/r03x_sq_w$wd.txt 2>&1 || exit 1
done
cat gpurun_out/r03x_gru_bench.log gpurun_out/r03x_sq_w*.txt
