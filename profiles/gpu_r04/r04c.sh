#!/bin/bash
# round 4, call c: (1) dual data gradient 256-row tiles (MARLSAT_DGRAD_RT=4) vs 128-row tiles, alternating,
# bitwise output checksums; (2) GRU forward: per-tile kernel vs the persistent walk without / with prefetch;
# (3) the dual-launch GEMM tests with the 256-row form forced on; (4) train-cycle parity at the round-4 bars
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for i in 1 2 3; do
  for r in 2 4; do
    MARLSAT_DGRAD_RT=$r DUAL_CHECKSUM=1 timeout -k 10 120 python profiles/dual_bench.py > gpurun_out/r04c_rt${r}_$i.log 2>&1 || exit $?
    sed "s/^/rt$r /" gpurun_out/r04c_rt${r}_$i.log | grep -v amdgpu.ids
  done
done
for i in 1 2; do
  for p in 0 2 1; do
    MARLSAT_GRU_PERSIST=$p GRU_KERNELS=h2r GRU_CHECKSUM=1 timeout -k 10 120 python profiles/gru_r_bench.py > gpurun_out/r04c_p${p}_$i.log 2>&1 || exit $?
    sed "s/^/p$p /" gpurun_out/r04c_p${p}_$i.log | grep cell
  done
done
MARLSAT_DGRAD_RT=4 timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q -k "dual or h2" --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r04c_gemm_tests.log 2>&1
echo "gemm tests (rt4) rc $?"; tail -3 gpurun_out/r04c_gemm_tests.log
timeout -k 10 500 python -u -m pytest tests/test_mappo_gpu.py tests/test_gru_bwd_reduction_gpu.py tests/test_gru_fused_gpu.py -q -k "every_adam_step or reduction or backward" --timeout 350 --timeout-method thread -p no:cacheprovider > gpurun_out/r04c_parity_tests.log 2>&1
echo "parity tests rc $?"; grep -E "passed|failed|Error:" gpurun_out/r04c_parity_tests.log | tail -8
