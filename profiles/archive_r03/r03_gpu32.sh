#!/bin/bash
# GRU backward scalar body (clause cell) variants: MSAT_BWD_MODE 0 old gates + shuffles, 1 fast gates, 2 DPP, 3 both
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for i in 1 2; do for m in 0 1 2 3; do
echo "== mode $m" >> gpurun_out/r03w_bwd_modes.log
MSAT_BWD_MODE=$m MSAT_BWD_VMODE=$m timeout -k 10 120 python -u profiles/gru_bwd_only.py >> gpurun_out/r03w_bwd_modes.log 2>&1 || exit 1
done; done
grep -v amdgpu.ids gpurun_out/r03w_bwd_modes.log
