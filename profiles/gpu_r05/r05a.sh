#!/bin/bash
# round 5, call a: env + C-ABI GPU tests (the step kernel gained diagnostic clock stamps), then the default bench
# (time-based pre-roll, sclk_mhz from the kernel's stamps, 3 MAPPO cycles, CPU baseline on every affinity core)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_env_gpu.py tests/test_capi.py -m gpu -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r05a_env_tests.log 2>&1
rc=$?
echo "tests rc $rc"; tail -3 gpurun_out/r05a_env_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 800 python bench.py > gpurun_out/r05a_bench.json 2> gpurun_out/r05a_bench.err
rb=$?
echo "bench rc $rb"
tail -c 600 gpurun_out/r05a_bench.json
exit $rb
