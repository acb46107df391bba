#!/bin/bash
# round 6, call t: config 2 (uf50 x 1024) at 64 / 128 / 256 lanes per env workgroup (MARLSAT_ENV_THREADS), alternated
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for i in 1 2; do
  for t in 64 128 256; do
    MARLSAT_ENV_THREADS=$t timeout -k 10 120 python bench.py --cpu-budget 0 --mappo= --env-legs= --workload uf50-218 \
        --envs 1024 --steps 2000 --warmup 50 > gpurun_out/r06t_uf50_t${t}_$i.json 2> gpurun_out/r06t_uf50_t${t}_$i.err \
        || { echo "bench failed"; tail -5 gpurun_out/r06t_uf50_t${t}_$i.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/r06t_uf50_t${t}_$i.json').read().strip().splitlines()[-1]); sp=d['stamp_phases']
print('threads ${t} run $i kernel_us %.3f frac %.3f span' % (d['roofline']['kernel_ms']*1e3, d['roofline']['frac']), sp['launch_span_us'], 'wg_med', sp['workgroup_median_us'], 'wg_max', sp['workgroup_max_us'], 'sclk', d['sclk_mhz'], 'phases', sp['phase_median_us'])" | tee -a gpurun_out/r06t_threads_ab.txt
  done
done
