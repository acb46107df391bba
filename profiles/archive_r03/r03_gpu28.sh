#!/bin/bash
# h2w ablations (clause + var, no tape): 1 product, 2 no epilogue, 3 no k-loop DMA, 4 no fragment reads; 0 = h2s
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for wd in 0 1 2 3 4; do
echo "== wide $wd" >> gpurun_out/r03y_abl.log
MARLSAT_GRU_WIDE=$wd GRU_KERNELS=h2r GRU_TAPE=False timeout -k 10 120 python -u profiles/gru_r_bench.py >> gpurun_out/r03y_abl.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/r03y_abl.log
