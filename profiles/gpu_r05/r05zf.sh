#!/bin/bash
# round 5, call zf: on one box, three builds of the planes weight gradient -- hd (row exponents by LDS-DMA,
# commit 3b96597), hf (hd + the A split's low halves by v_fma_mix), fm (exponents by scalar loads + v_fma_mix):
# hf's planes / gemm tests, the dual weight gradient (clause / var shapes) and the MAPPO leg's kernel trace per build
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T="python -u -m pytest -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider"
D=$PWD/marl-sat_amd/marlsat/lib
MARLSAT_LIB=$D/libmarlsat_hf.so timeout -k 10 600 $T -q tests/test_planes_gpu.py tests/test_gemm_gpu.py > gpurun_out/r05zf_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -2 gpurun_out/r05zf_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do for L in hd hf fm; do
  DUAL_ONLY="wgrad planes" MARLSAT_LIB=$D/libmarlsat_$L.so timeout -k 10 200 python -u profiles/dual_bench.py 1316000 10 256 2 > gpurun_out/r05zf_clause_$L$i.log 2>&1 || exit 4
  DUAL_ONLY="wgrad planes" MARLSAT_LIB=$D/libmarlsat_$L.so timeout -k 10 200 python -u profiles/dual_bench.py 560000 10 128 2 > gpurun_out/r05zf_var_$L$i.log 2>&1 || exit 5
  echo "$L$i clause $(grep -o '"us": [0-9.]*' gpurun_out/r05zf_clause_$L$i.log | tr '\n' ' ') var $(grep -o '"us": [0-9.]*' gpurun_out/r05zf_var_$L$i.log | tr '\n' ' ')"
done; done
for L in hd hf fm; do
  MARLSAT_LIB=$D/libmarlsat_$L.so timeout -k 10 600 bash profiles/collect_mappo.sh r05zf_$L > gpurun_out/r05zf_collect_$L.log 2>&1 || exit 6
  echo "$L $(grep -E "wgrad_w_dual_pl" gpurun_out/keep/r05zf_${L}_mappo_uf100-430_kernel_stats.csv | cut -d, -f3-4) $(grep -o '"s_min_med_max": \[[^]]*\]' gpurun_out/keep/r05zf_${L}_mappo_uf100-430_bench.json)"
done
