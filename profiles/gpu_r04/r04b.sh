#!/bin/bash
# round 4, call b: persistent GRU forward (MARLSAT_GRU_PERSIST=1) vs the per-tile kernel, alternating, bitwise
# output checksums; then the GRU kernel tests with the persistent form forced on
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for i in 1 2 3; do
  for p in 0 1; do
    MARLSAT_GRU_PERSIST=$p GRU_KERNELS=h2r GRU_CHECKSUM=1 timeout -k 10 120 python profiles/gru_r_bench.py > gpurun_out/r04b_p${p}_$i.log 2>&1 || exit $?
    sed "s/^/p$p /" gpurun_out/r04b_p${p}_$i.log | grep cell
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gru_fused_gpu.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04b_gru_tests.log 2>&1
echo "gru tests rc $?"; tail -3 gpurun_out/r04b_gru_tests.log
timeout -k 10 200 python -u -m pytest tests/test_debug_build.py -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r04b_debug_tests.log 2>&1
echo "debug tests rc $?"; tail -3 gpurun_out/r04b_debug_tests.log
timeout -k 10 400 python -u -m pytest tests/test_gru_bwd_reduction_gpu.py tests/test_mappo_gpu.py -q -k "reduction or every_adam_step" --timeout 350 --timeout-method thread -p no:cacheprovider --durations=5 > gpurun_out/r04b_parity_tests.log 2>&1
echo "parity tests rc $?"; tail -12 gpurun_out/r04b_parity_tests.log
