#!/bin/bash
# round 5, call ze: the MAPPO leg's kernel trace on one box for three builds of the planes weight gradient:
# hd (row exponents by LDS-DMA, commit 3b96597), sx (by scalar loads), fm (sx + the A split's low halves by
# v_fma_mix) -- fm's planes / gemm tests first
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T="python -u -m pytest -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider"
D=$PWD/marl-sat_amd/marlsat/lib
MARLSAT_LIB=$D/libmarlsat_fm.so timeout -k 10 600 $T -q tests/test_planes_gpu.py tests/test_gemm_gpu.py > gpurun_out/r05ze_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -2 gpurun_out/r05ze_tests.log
[ $rc -eq 0 ] || exit $rc
for L in hd sx fm hd; do
  MARLSAT_LIB=$D/libmarlsat_$L.so timeout -k 10 600 bash profiles/collect_mappo.sh r05ze_$L > gpurun_out/r05ze_collect_$L.log 2>&1 || exit 6
  echo "$L $(grep -E "wgrad_w_dual_pl" gpurun_out/keep/r05ze_${L}_mappo_uf100-430_kernel_stats.csv | cut -d, -f1-4 | cut -c60-200) $(grep -o '"s_min_med_max": \[[^]]*\]' gpurun_out/keep/r05ze_${L}_mappo_uf100-430_bench.json)"
done
