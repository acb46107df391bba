#!/bin/bash
# round 4, call e: full-width dual data gradient -- bitwise vs the per-tile kernel, fp64 bounds, A/B timing
# (MARLSAT_DGRAD_WIDE=0 per-tile vs 1 full-width) on both GRU cell shapes, then the training parity subset
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q -k "dual or h2" --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r04e_gemm_tests.log 2>&1
rc=$?
echo "gemm tests rc $rc"; tail -15 gpurun_out/r04e_gemm_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for r in 0 1; do
    MARLSAT_DGRAD_WIDE=$r DUAL_ONLY=dgrad DUAL_CHECKSUM=1 timeout -k 10 120 python profiles/dual_bench.py 1316000 10 256 > gpurun_out/r04e_c_w${r}_$i.log 2>&1 || exit $?
    sed "s/^/clause w$r /" gpurun_out/r04e_c_w${r}_$i.log | grep -v amdgpu.ids
    MARLSAT_DGRAD_WIDE=$r DUAL_ONLY=dgrad DUAL_CHECKSUM=1 timeout -k 10 120 python profiles/dual_bench.py 560000 10 128 > gpurun_out/r04e_v_w${r}_$i.log 2>&1 || exit $?
    sed "s/^/var w$r /" gpurun_out/r04e_v_w${r}_$i.log | grep -v amdgpu.ids
  done
done
timeout -k 10 500 python -u -m pytest tests/test_mappo_gpu.py tests/test_gnn_gpu.py -q -k "every_adam_step or backward" --timeout 350 --timeout-method thread -p no:cacheprovider > gpurun_out/r04e_parity_tests.log 2>&1
echo "parity tests rc $?"; grep -E "passed|failed|Error:" gpurun_out/r04e_parity_tests.log | tail -8
