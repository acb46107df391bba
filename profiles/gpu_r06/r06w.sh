#!/bin/bash
# round 6, call w: env workgroup width at 4096 envs -- uf100 at 128 / 256 lanes, uf200 (the headline) at 256 / 512
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for i in 1 2; do
  for spec in "uf100-430 128" "uf100-430 256" "uf200-860 256" "uf200-860 512"; do
    set -- $spec
    MARLSAT_ENV_THREADS=$2 timeout -k 10 120 python bench.py --cpu-budget 0 --mappo= --env-legs= --workload $1 \
        --envs 4096 --steps 500 --warmup 20 > gpurun_out/r06w.json 2> gpurun_out/r06w.err \
        || { echo "bench failed"; tail -5 gpurun_out/r06w.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/r06w.json').read().strip().splitlines()[-1])
print('$1 x 4096 threads $2 run $i kernel_us %.3f frac %.3f sclk %s' % (d['roofline']['kernel_ms']*1e3, d['roofline']['frac'], d['sclk_mhz']))" | tee -a gpurun_out/r06w_threads_4096.txt
  done
done
