#!/bin/bash
# round 5, call zc: the row exponents by scalar loads in the product build -- planes / gemm / GRU-backward / MAPPO /
# debug-build tests, both dual forms, and the MAPPO leg's kernel trace beside call w (planes, exponents by DMA)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T="python -u -m pytest -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T -q tests/test_planes_gpu.py tests/test_gemm_gpu.py tests/test_gru_bwd_reduction_gpu.py tests/test_mappo_gpu.py tests/test_debug_build.py > gpurun_out/r05zc_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -2 gpurun_out/r05zc_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u profiles/dual_bench.py 1316000 10 256 3 > gpurun_out/r05zc_dual_clause.log 2>&1 || exit 4
timeout -k 10 300 python -u profiles/dual_bench.py 560000 10 128 3 > gpurun_out/r05zc_dual_var.log 2>&1 || exit 5
grep '^{' gpurun_out/r05zc_dual_clause.log gpurun_out/r05zc_dual_var.log | cut -d: -f2- | cut -c1-110
timeout -k 10 900 bash profiles/collect_mappo.sh r05zc > gpurun_out/r05zc_collect.log 2>&1 || exit 6
grep -E "wgrad_w_dual|gemm_h2r16_dual|gru_ln_bwd" gpurun_out/keep/r05zc_mappo_uf100-430_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
grep -o '"s_min_med_max": \[[^]]*\]' gpurun_out/keep/r05zc_mappo_uf100-430_bench.json
