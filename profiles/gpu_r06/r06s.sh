#!/bin/bash
# round 6, call s: the instance cache (msat_env_state.inst_cache) -- env / C-ABI / single-agent tests (the cache is on
# for their small batches) incl. its invisibility test, the GRU small-activation test with its negative control,
# then config 2 (uf50 x 1024) A/B with the cache on / off, alternated, and the headline shape (cache off by size)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py tests/test_capi.py tests/test_single_env_gpu.py -m gpu -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06s_env_tests.log 2>&1
rc=$?
echo "env tests rc $rc"; tail -3 gpurun_out/r06s_env_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 bash profiles/gpu_r06/r06r.sh || exit 1
for i in 1 2; do
  for c in auto 0; do
    MARLSAT_INST_CACHE=$c timeout -k 10 120 python bench.py --cpu-budget 0 --mappo= --env-legs= --workload uf50-218 \
        --envs 1024 --steps 2000 --warmup 50 > gpurun_out/r06s_uf50_c${c}_$i.json 2> gpurun_out/r06s_uf50_c${c}_$i.err \
        || { echo "bench failed"; tail -5 gpurun_out/r06s_uf50_c${c}_$i.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/r06s_uf50_c${c}_$i.json').read().strip().splitlines()[-1]); sp=d['stamp_phases']
print('cache=${c} run $i kernel_us %.3f frac %.3f span' % (d['roofline']['kernel_ms']*1e3, d['roofline']['frac']), sp['launch_span_us'], 'wg_med', sp['workgroup_median_us'], 'wg_max', sp['workgroup_max_us'], 'sclk', d['sclk_mhz'], 'phases', sp['phase_median_us'])" | tee -a gpurun_out/r06s_cache_ab.txt
  done
done
timeout -k 10 200 python bench.py --cpu-budget 0 --mappo= --env-legs= > gpurun_out/r06s_headline.json 2> gpurun_out/r06s_headline.err \
    || { echo "headline bench failed"; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r06s_headline.json').read().strip().splitlines()[-1])
print('headline', d['value'], d['ms_per_step'], d['roofline']['frac'], d['sclk_mhz'])" | tee -a gpurun_out/r06s_cache_ab.txt
