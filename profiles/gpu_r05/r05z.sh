#!/bin/bash
# round 5, call z: the planes in 64-byte chunks alternating hi and lo (a data-gradient row step reads one 128-byte line,
# the weight gradient's DMA chunks stay in 64-byte runs of one plane) -- tests, both dual forms, and the MAPPO leg's
# kernel trace beside calls w (two half-row planes), x (fp32 rows) and y (16-byte chunks)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T="python -u -m pytest -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T -q tests/test_planes_gpu.py tests/test_gemm_gpu.py tests/test_gru_bwd_reduction_gpu.py tests/test_mappo_gpu.py > gpurun_out/r05z_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -2 gpurun_out/r05z_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u profiles/dual_bench.py 1316000 10 256 3 > gpurun_out/r05z_dual_clause.log 2>&1 || exit 4
timeout -k 10 300 python -u profiles/dual_bench.py 560000 10 128 3 > gpurun_out/r05z_dual_var.log 2>&1 || exit 5
grep '^{' gpurun_out/r05z_dual_clause.log gpurun_out/r05z_dual_var.log | cut -d: -f2- | cut -c1-110
timeout -k 10 900 bash profiles/collect_mappo.sh r05z > gpurun_out/r05z_collect.log 2>&1 || exit 6
grep -E "wgrad_w_dual|gemm_h2r16_dual|gru_ln_bwd" gpurun_out/keep/r05z_mappo_uf100-430_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
grep -o '"s_min_med_max": \[[^]]*\]' gpurun_out/keep/r05z_mappo_uf100-430_bench.json
