#!/bin/bash
# clause gather, two rows per wave (half-waves): gather tests, then A/B (split forward form and merged backward form)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gnn_gpu.py -k "gather" > gpurun_out/r03w_gather_tests.log 2>&1 || { tail -30 gpurun_out/r03w_gather_tests.log; exit 1; }
tail -1 gpurun_out/r03w_gather_tests.log
bash profiles/r03_ab.sh 3 profiles/gather_only.py > gpurun_out/r03w_gather_ab.log 2>&1 || exit 1
GATHER_MODE=bwd bash profiles/r03_ab.sh 3 profiles/gather_only.py > gpurun_out/r03w_gather_ab_bwd.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03w_gather_ab.log gpurun_out/r03w_gather_ab_bwd.log
