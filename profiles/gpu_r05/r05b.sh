#!/bin/bash
# round 5, call b: the stamp test and the dual-launch wbig cases (ADVICE), then the env legs alone with the
# kernel's phase stamps (side file bench_env_stamps_n1.json)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_env_gpu.py tests/test_gemm_gpu.py -m gpu -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "clock_stamps or dual_launches" > gpurun_out/r05b_tests.log 2>&1
rc=$?
echo "tests rc $rc"; tail -3 gpurun_out/r05b_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --mappo '' --cpu-budget 0 > gpurun_out/r05b_bench_env.json 2> gpurun_out/r05b_bench_env.err
rb=$?
echo "bench rc $rb"
exit $rb
