#!/bin/bash
# round 5, call zg: on one box, hd (row exponents by one LDS-DMA piece per wave and slab, commit 3b96597) against q4
# (one exponent piece per wave and four slabs, 4.25 pieces per slab instead of 5, + the A split's low halves by
# v_fma_mix): q4's planes / gemm tests, the dual weight gradient (clause / var) and the MAPPO leg's kernel trace
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T="python -u -m pytest -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider"
D=$PWD/marl-sat_amd/marlsat/lib
MARLSAT_LIB=$D/libmarlsat_q4.so timeout -k 10 600 $T -q tests/test_planes_gpu.py tests/test_gemm_gpu.py > gpurun_out/r05zg_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -2 gpurun_out/r05zg_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do for L in hd q4; do
  DUAL_ONLY="wgrad planes" MARLSAT_LIB=$D/libmarlsat_$L.so timeout -k 10 200 python -u profiles/dual_bench.py 1316000 10 256 2 > gpurun_out/r05zg_clause_$L$i.log 2>&1 || exit 4
  DUAL_ONLY="wgrad planes" MARLSAT_LIB=$D/libmarlsat_$L.so timeout -k 10 200 python -u profiles/dual_bench.py 560000 10 128 2 > gpurun_out/r05zg_var_$L$i.log 2>&1 || exit 5
  echo "$L$i clause $(grep -o '"us": [0-9.]*' gpurun_out/r05zg_clause_$L$i.log | tr '\n' ' ') var $(grep -o '"us": [0-9.]*' gpurun_out/r05zg_var_$L$i.log | tr '\n' ' ')"
done; done
for L in hd q4; do
  MARLSAT_LIB=$D/libmarlsat_$L.so timeout -k 10 600 bash profiles/collect_mappo.sh r05zg_$L > gpurun_out/r05zg_collect_$L.log 2>&1 || exit 6
  echo "$L $(grep -E "wgrad_w_dual_pl" gpurun_out/keep/r05zg_${L}_mappo_uf100-430_kernel_stats.csv | cut -d, -f3-4) $(grep -o '"s_min_med_max": \[[^]]*\]' gpurun_out/keep/r05zg_${L}_mappo_uf100-430_bench.json)"
done
