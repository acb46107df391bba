#!/bin/bash
# round 4, call x: the 12-wave dual data gradient as the default -- GEMM tests, network / train-cycle parity
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_gnn_gpu.py tests/test_mappo_gpu.py tests/test_debug_build.py -q --timeout 350 --timeout-method thread -p no:cacheprovider > gpurun_out/r04x_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -3 gpurun_out/r04x_tests.log; exit $rc
