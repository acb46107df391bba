#!/bin/bash
# round 6, call y: the width rule for the uf100 class (128 lanes from 2048 envs) -- env / single-agent / runner tests,
# then the uf100 x 4096 side leg by the default rule
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_env_gpu.py tests/test_capi.py tests/test_single_env_gpu.py \
    tests/test_runner_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r06y_env_tests.log 2>&1
rc=$?
echo "env tests rc $rc"; tail -2 gpurun_out/r06y_env_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python bench.py --cpu-budget 0 --mappo= --env-legs= --workload uf100-430 --envs 4096 --steps 500 \
    --warmup 20 > gpurun_out/r06y_uf100.json 2> gpurun_out/r06y_uf100.err || { echo "bench failed"; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r06y_uf100.json').read().strip().splitlines()[-1])
print('uf100 x 4096 default rule', d['value'], 'kernel_us %.3f frac %.3f' % (d['roofline']['kernel_ms']*1e3, d['roofline']['frac']), d['roofline'].get('kernel'), d['sclk_mhz'])"
