#!/bin/bash
# round 3: N=2 rehearsals (gloo, shared GPU) of the mixed workload and uf200, parity report of the final kernels
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MARLSAT_DIST_BACKEND=gloo MARLSAT_SHARE_GPU=1 timeout -k 10 600 python bench.py --gpus 2 --workload mixed --envs 8192 \
    --steps 50 --warmup 10 --mappo uf200-860:4096:1 --mappo-micro-gb 100 --cpu-budget 6 > gpurun_out/r03d_dist2_mixed.json 2> gpurun_out/r03d_dist2_mixed.err &&
timeout -k 10 900 python -u -m pytest tests/test_gnn_gpu.py -k "depth16 or uf200" -s -q --timeout 300 --timeout-method thread > gpurun_out/r03d_parity_depth.txt 2>&1
