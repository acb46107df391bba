#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gathers_gpu.py tests/test_gnn_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03s_tests.log 2>&1 || { tail -30 gpurun_out/r03s_tests.log; exit 1; }
tail -1 gpurun_out/r03s_tests.log
LIBS="base" bash profiles/r03_ab_multi.sh 3 profiles/gather_only.py > gpurun_out/r03s_ab_gather_fwd.log 2>&1 || exit 1
GATHER_MODE=bwd LIBS="base" bash profiles/r03_ab_multi.sh 2 profiles/gather_only.py > gpurun_out/r03s_ab_gather_bwd.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03s_ab_gather_fwd.log gpurun_out/r03s_ab_gather_bwd.log
