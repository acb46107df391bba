#!/bin/bash
# round 4, call l: dual data gradient with the weights issued two steps ahead (MARLSAT_DGRAD_WD=2)
# vs LDS-DMA (product), alternating, bitwise checksums, both GRU cell shapes; then the dual GEMM tests with it
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for i in 1 2 3; do
  for r in 1 2; do
    MARLSAT_DGRAD_WD=$r DUAL_ONLY=dgrad DUAL_CHECKSUM=1 timeout -k 10 120 python profiles/dual_bench.py 1316000 10 256 > gpurun_out/r04l_c_$r_$i.log 2>&1 || exit $?
    sed "s/^/clause wd$r /" gpurun_out/r04l_c_$r_$i.log | grep -v amdgpu.ids
    MARLSAT_DGRAD_WD=$r DUAL_ONLY=dgrad DUAL_CHECKSUM=1 timeout -k 10 120 python profiles/dual_bench.py 560000 10 128 > gpurun_out/r04l_v_$r_$i.log 2>&1 || exit $?
    sed "s/^/var wd$r /" gpurun_out/r04l_v_$r_$i.log | grep -v amdgpu.ids
  done
done
MARLSAT_DGRAD_WD=2 timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q -k "dual" --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r04l_tests.log 2>&1
echo "dual tests (wd) rc $?"; tail -2 gpurun_out/r04l_tests.log
