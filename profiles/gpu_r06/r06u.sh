#!/bin/bash
# round 6, call u: uf50 at 2048 / 4096 envs with 64 vs 128 lanes per env workgroup (where the width heuristic's batch
# threshold goes), alternated twice
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for i in 1 2; do
  for B in 2048 4096; do
    for t in 64 128; do
      MARLSAT_ENV_THREADS=$t timeout -k 10 120 python bench.py --cpu-budget 0 --mappo= --env-legs= --workload uf50-218 \
          --envs $B --steps 1000 --warmup 50 > gpurun_out/r06u.json 2> gpurun_out/r06u.err \
          || { echo "bench failed"; tail -5 gpurun_out/r06u.err; exit 1; }
      python -c "
import json; d=json.loads(open('gpurun_out/r06u.json').read().strip().splitlines()[-1])
print('B $B threads ${t} run $i kernel_us %.3f frac %.3f sclk %s' % (d['roofline']['kernel_ms']*1e3, d['roofline']['frac'], d['sclk_mhz']))" | tee -a gpurun_out/r06u_threads_ab.txt
    done
  done
done
