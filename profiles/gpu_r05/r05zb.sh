#!/bin/bash
# round 5, call zb: the planes weight gradient's row exponents by scalar loads (4 LDS-DMA pieces per wave and slab,
# was 5) as libmarlsat_sx.so -- planes / gemm tests on it, then the dual weight gradient, default vs sx, alternated
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T="python -u -m pytest -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider"
SX=$PWD/marl-sat_amd/marlsat/lib/libmarlsat_sx.so
MARLSAT_LIB=$SX timeout -k 10 600 $T -q tests/test_planes_gpu.py tests/test_gemm_gpu.py > gpurun_out/r05zb_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -2 gpurun_out/r05zb_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  DUAL_ONLY=planes timeout -k 10 200 python -u profiles/dual_bench.py 1316000 10 256 2 > gpurun_out/r05zb_clause_def$i.log 2>&1 || exit 4
  DUAL_ONLY=planes MARLSAT_LIB=$SX timeout -k 10 200 python -u profiles/dual_bench.py 1316000 10 256 2 > gpurun_out/r05zb_clause_sx$i.log 2>&1 || exit 5
  DUAL_ONLY=planes timeout -k 10 200 python -u profiles/dual_bench.py 560000 10 128 2 > gpurun_out/r05zb_var_def$i.log 2>&1 || exit 6
  DUAL_ONLY=planes MARLSAT_LIB=$SX timeout -k 10 200 python -u profiles/dual_bench.py 560000 10 128 2 > gpurun_out/r05zb_var_sx$i.log 2>&1 || exit 7
done
grep -H '^{' gpurun_out/r05zb_*_def*.log gpurun_out/r05zb_*_sx*.log | cut -c1-150
