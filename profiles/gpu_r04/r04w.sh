#!/bin/bash
# round 4, call w: dual data gradient with 384-row workgroups of 12 waves, one per CU (MARLSAT_DGRAD_WAVES=12)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for i in 1 2 3; do
  for r in 4 12; do
    MARLSAT_DGRAD_WAVES=$r DUAL_ONLY=dgrad DUAL_CHECKSUM=1 timeout -k 10 120 python profiles/dual_bench.py 1316000 10 256 > gpurun_out/r04w_c_${r}_$i.log 2>&1 || exit $?
    sed "s/^/clause w$r /" gpurun_out/r04w_c_${r}_$i.log | grep -v amdgpu.ids
    MARLSAT_DGRAD_WAVES=$r DUAL_ONLY=dgrad DUAL_CHECKSUM=1 timeout -k 10 120 python profiles/dual_bench.py 560000 10 128 > gpurun_out/r04w_v_${r}_$i.log 2>&1 || exit $?
    sed "s/^/var w$r /" gpurun_out/r04w_v_${r}_$i.log | grep -v amdgpu.ids
  done
done
MARLSAT_DGRAD_WAVES=12 timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q -k "dual" --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r04w_tests.log 2>&1
echo "dual tests (w) rc $?"; tail -2 gpurun_out/r04w_tests.log
