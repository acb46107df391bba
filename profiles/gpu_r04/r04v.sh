#!/bin/bash
# round 4, call v: dual data gradient with both operands issued two steps ahead by untracked loads and explicit
# waits (MARLSAT_DGRAD_ASW=1) vs the product kernel, alternating, bitwise checksums; GEMM tests with it
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for i in 1 2 3; do
  for r in 0 1; do
    MARLSAT_DGRAD_ASW=$r DUAL_ONLY=dgrad DUAL_CHECKSUM=1 timeout -k 10 120 python profiles/dual_bench.py 1316000 10 256 > gpurun_out/r04v_c_${r}_$i.log 2>&1 || exit $?
    sed "s/^/clause asw$r /" gpurun_out/r04v_c_${r}_$i.log | grep -v amdgpu.ids
    MARLSAT_DGRAD_ASW=$r DUAL_ONLY=dgrad DUAL_CHECKSUM=1 timeout -k 10 120 python profiles/dual_bench.py 560000 10 128 > gpurun_out/r04v_v_${r}_$i.log 2>&1 || exit $?
    sed "s/^/var asw$r /" gpurun_out/r04v_v_${r}_$i.log | grep -v amdgpu.ids
  done
done
MARLSAT_DGRAD_ASW=1 timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q -k "dual" --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r04v_tests.log 2>&1
echo "dual tests (asw) rc $?"; tail -2 gpurun_out/r04v_tests.log
