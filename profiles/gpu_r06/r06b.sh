#!/bin/bash
# round 6, call b: env tests with the reset queue (timed-out resets in workgroups of their own; verdict item 5),
# the config-2 / headline env legs with stamps, then which fp16x2 kernel carries the default path's train-cycle
# error (profiles/parity_switch_probe.py)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py tests/test_capi.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r06b_env_tests.log 2>&1
rc=$?
echo "env tests rc $rc"; tail -4 gpurun_out/r06b_env_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --cpu-budget 0 --mappo= --env-legs uf50-218:1024,uf100-430:4096 \
    > gpurun_out/r06b_bench_env.json 2> gpurun_out/r06b_bench_env.err
rc=$?
echo "bench rc $rc"; tail -c 900 gpurun_out/r06b_bench_env.json
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 python -u profiles/parity_switch_probe.py > gpurun_out/r06b_switch_probe.log 2>&1
rc=$?
echo "probe rc $rc"; grep -E "^===|margins .* step 1" gpurun_out/r06b_switch_probe.log | cut -c1-260
exit $rc
