#!/bin/bash
# round 4, call c: dual data gradient 256-row tiles (MARLSAT_DGRAD_RT=4) vs 128-row tiles, alternating, bitwise
# output checksums; the dual-launch GEMM tests with the 256-row form forced on
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for i in 1 2 3; do
  for r in 2 4; do
    MARLSAT_DGRAD_RT=$r DUAL_CHECKSUM=1 timeout -k 10 120 python profiles/dual_bench.py > gpurun_out/r04c_rt${r}_$i.log 2>&1 || exit $?
    sed "s/^/rt$r /" gpurun_out/r04c_rt${r}_$i.log | grep -v amdgpu.ids
  done
done
MARLSAT_DGRAD_RT=4 timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q -k "dual or h2" --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r04c_gemm_tests.log 2>&1
echo "gemm tests (rt4) rc $?"; tail -3 gpurun_out/r04c_gemm_tests.log
