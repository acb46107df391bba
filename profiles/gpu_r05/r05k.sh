#!/bin/bash
# round 5, call k: planes weight gradient (fragments one slab ahead, 4-slot DMA rings with the row exponents) -- planes tests,
# then the dual products in both forms (clause / var shapes, three alternations)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T="python -u -m pytest -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T -v tests/test_planes_gpu.py > gpurun_out/r05k_planes_tests.log 2>&1
rc=$?; echo "planes tests rc $rc"; tail -3 gpurun_out/r05k_planes_tests.log
[ $rc -eq 0 ] || exit $rc
DUAL_ONLY=wgrad timeout -k 10 300 python -u profiles/dual_bench.py 1316000 10 256 3 > gpurun_out/r05k_dual_clause.log 2>&1 || exit 4
DUAL_ONLY=wgrad timeout -k 10 300 python -u profiles/dual_bench.py 560000 10 128 3 > gpurun_out/r05k_dual_var.log 2>&1 || exit 5
cat gpurun_out/r05k_dual_clause.log gpurun_out/r05k_dual_var.log
BWD_ALT=3 timeout -k 10 300 python -u profiles/gru_bwd_only.py 10 > gpurun_out/r05k_gru_bwd.log 2>&1 || exit 6
cat gpurun_out/r05k_gru_bwd.log
