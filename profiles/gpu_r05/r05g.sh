#!/bin/bash
# round 5, call g: env kernel -- timed-out envs prefetch their reset instance before the scan, the unsat load
# retired before the scan's stores; bit-exact env tests, then the env legs with stamps (twice)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T="python -u -m pytest -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T -q tests/test_env_gpu.py tests/test_single_env_gpu.py tests/test_runner_gpu.py > gpurun_out/r05g_env_tests.log 2>&1
rc=$?; echo "env tests rc $rc"; tail -2 gpurun_out/r05g_env_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  timeout -k 10 300 python bench.py --mappo '' --cpu-budget 0 > gpurun_out/r05g_bench_env_$i.json 2> gpurun_out/r05g_bench_env_$i.err || exit 4
  cp gpurun_out/bench_env_stamps_n1.json gpurun_out/r05g_env_stamps_$i.json
done
exit 0
