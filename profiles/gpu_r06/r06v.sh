#!/bin/bash
# round 6, call v: env workgroups of 128 lanes for small instances in batches of <= 1024 envs -- env / single-agent /
# runner tests, then config 2 by the default heuristic (twice) and the headline shape
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_env_gpu.py tests/test_capi.py tests/test_single_env_gpu.py \
    tests/test_runner_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r06v_env_tests.log 2>&1
rc=$?
echo "env tests rc $rc"; tail -3 gpurun_out/r06v_env_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 python bench.py --cpu-budget 0 --mappo= --env-legs= --workload uf50-218 --envs 1024 --steps 2000 \
      --warmup 50 > gpurun_out/r06v_uf50_$i.json 2> gpurun_out/r06v_uf50_$i.err || { echo "bench failed"; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r06v_uf50_$i.json').read().strip().splitlines()[-1])
print('config 2 run $i', d['value'], 'kernel_us %.3f frac %.3f' % (d['roofline']['kernel_ms']*1e3, d['roofline']['frac']), d['config'], d['sclk_mhz'])" | tee -a gpurun_out/r06v_config2.txt
done
