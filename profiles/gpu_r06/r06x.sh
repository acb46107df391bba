#!/bin/bash
# round 6, call x: uf100 env workgroup width at 1024 / 2048 envs (64 / 128 / 256 lanes), alternated twice
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for i in 1 2; do
  for B in 1024 2048; do
    for t in 64 128 256; do
      MARLSAT_ENV_THREADS=$t timeout -k 10 120 python bench.py --cpu-budget 0 --mappo= --env-legs= --workload uf100-430 \
          --envs $B --steps 1000 --warmup 20 > gpurun_out/r06x.json 2> gpurun_out/r06x.err \
          || { echo "bench failed"; tail -5 gpurun_out/r06x.err; exit 1; }
      python -c "
import json; d=json.loads(open('gpurun_out/r06x.json').read().strip().splitlines()[-1])
print('uf100-430 x $B threads $t run $i kernel_us %.3f frac %.3f sclk %s' % (d['roofline']['kernel_ms']*1e3, d['roofline']['frac'], d['sclk_mhz']))" | tee -a gpurun_out/r06x_uf100_threads.txt
    done
  done
done
