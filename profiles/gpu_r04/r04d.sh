#!/bin/bash
# round 4, call d: resident-weight dual data gradient -- bitwise vs the per-tile kernel, fp64 bounds, then
# A/B timing (MARLSAT_DGRAD_RESIDENT=0 per-tile, 3 default prefetch depth, 2 / 4) on both GRU cell shapes
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q -k "dual or h2" --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r04d_gemm_tests.log 2>&1
rc=$?
echo "gemm tests rc $rc"; tail -15 gpurun_out/r04d_gemm_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for r in 0 3 2 4; do
    MARLSAT_DGRAD_RESIDENT=$r DUAL_ONLY=dgrad timeout -k 10 120 python profiles/dual_bench.py 1316000 10 256 > gpurun_out/r04d_c_r${r}_$i.log 2>&1 || exit $?
    sed "s/^/clause r$r /" gpurun_out/r04d_c_r${r}_$i.log | grep -v amdgpu.ids
    MARLSAT_DGRAD_RESIDENT=$r DUAL_ONLY=dgrad timeout -k 10 120 python profiles/dual_bench.py 560000 10 128 > gpurun_out/r04d_v_r${r}_$i.log 2>&1 || exit $?
    sed "s/^/var r$r /" gpurun_out/r04d_v_r${r}_$i.log | grep -v amdgpu.ids
  done
done
timeout -k 10 500 python -u -m pytest tests/test_mappo_gpu.py tests/test_gnn_gpu.py -q -k "every_adam_step or backward" --timeout 350 --timeout-method thread -p no:cacheprovider > gpurun_out/r04d_parity_tests.log 2>&1
echo "parity tests rc $?"; grep -E "passed|failed|Error:" gpurun_out/r04d_parity_tests.log | tail -8
