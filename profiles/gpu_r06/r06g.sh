#!/bin/bash
# round 6, call g: the reset queue as a pending-token array (rank scan, no atomics): env tests incl. a whole-batch
# timeout, then per-launch times from a fresh reset (mass timeout at launch 511) with the queue on / off, and
# config 2 A/B
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py tests/test_capi.py tests/test_single_env_gpu.py -m gpu -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06g_env_tests.log 2>&1
rc=$?
echo "env tests rc $rc"; tail -3 gpurun_out/r06g_env_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for q in 1 0; do
  for spec in "uf50-218 1024" "uf200-860 4096"; do
    MARLSAT_RESET_QUEUE=$q timeout -k 10 120 python profiles/env_mass_timeout.py $spec 2>/dev/null | tee -a gpurun_out/r06g_mass_timeout.log \
        || { echo "mass timeout probe failed"; exit 1; }
  done
done
for i in 1 2; do
  for q in 1 0; do
    MARLSAT_RESET_QUEUE=$q timeout -k 10 120 python bench.py --cpu-budget 0 --mappo= --env-legs= --workload uf50-218 \
        --envs 1024 --steps 2000 --warmup 50 > gpurun_out/r06g_uf50_q${q}_$i.json 2> gpurun_out/r06g_uf50_q${q}_$i.err \
        || { echo "bench failed"; tail -5 gpurun_out/r06g_uf50_q${q}_$i.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/r06g_uf50_q${q}_$i.json').read().strip().splitlines()[-1]); sp=d['stamp_phases']
print('q${q} run $i kernel_us %.3f frac %.3f span' % (d['roofline']['kernel_ms']*1e3, d['roofline']['frac']), sp['launch_span_us'], 'wg_med', sp['workgroup_median_us'], 'wg_max', sp['workgroup_max_us'], 'sclk', d['sclk_mhz'])"
  done
done
