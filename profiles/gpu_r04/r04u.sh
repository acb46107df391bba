#!/bin/bash
# round 4, call u: the data gradient with its weight planes in k16 column order (activation loads as 64-byte
# row runs): GEMM tests, dual_bench on both cell shapes, then the training parity subset
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q -k "dual or h2" --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r04u_gemm_tests.log 2>&1
rc=$?; echo "gemm tests rc $rc"; tail -3 gpurun_out/r04u_gemm_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  DUAL_ONLY=dgrad timeout -k 10 120 python profiles/dual_bench.py 1316000 10 256 2>&1 | grep -v amdgpu.ids | sed "s/^/clause k16 /"
  DUAL_ONLY=dgrad timeout -k 10 120 python profiles/dual_bench.py 560000 10 128 2>&1 | grep -v amdgpu.ids | sed "s/^/var k16 /"
done
timeout -k 10 500 python -u -m pytest tests/test_mappo_gpu.py tests/test_gnn_gpu.py -q -k "every_adam_step or backward or depth16 or matches_oracle_replay" --timeout 350 --timeout-method thread -p no:cacheprovider > gpurun_out/r04u_parity_tests.log 2>&1
echo "parity tests rc $?"; grep -E "passed|failed|Error:" gpurun_out/r04u_parity_tests.log | tail -6
