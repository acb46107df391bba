#!/bin/bash
# round 3, first GPU call: changed tests, parity profile of the defaults, N=2 bench rehearsal, default bench
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT tests/test_gnn_gpu.py -k "depth16 or uf200" -s > gpurun_out/r03_parity_depth.txt 2>&1 &&
timeout -k 10 600 $PYT tests/test_gemm_gpu.py -k wgrad_rot tests/test_learner_glue_gpu.py tests/test_comm_gpu.py \
    tests/test_dist_learner_gpu.py > gpurun_out/r03_tests1.txt 2>&1 &&
MARLSAT_DIST_BACKEND=gloo MARLSAT_SHARE_GPU=1 timeout -k 10 600 python bench.py --gpus 2 --steps 50 --warmup 10 \
    --mappo uf200-860:4096:1 --mappo-micro-gb 100 --cpu-budget 4 > gpurun_out/r03_dist2_uf200.json 2> gpurun_out/r03_dist2_uf200.err &&
timeout -k 10 900 python bench.py > gpurun_out/r03_bench_default.json 2> gpurun_out/r03_bench_default.err
