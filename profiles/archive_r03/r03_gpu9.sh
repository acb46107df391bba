#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
MARLSAT_DIST_BACKEND=gloo MARLSAT_SHARE_GPU=1 timeout -k 10 600 python bench.py --gpus 2 --steps 20 --warmup 5 \
    --mappo uf200-860:4096:1 --mappo-micro-gb 100 --cpu-budget 0 > gpurun_out/r03i_dist2.json 2> gpurun_out/r03i_dist2.err
python3 -c "
import json
for r in (0, 1):
    d = json.load(open(f'gpurun_out/bench_mappo_uf200-860_n2_rank{r}.json'))
    print(r, d['params_check'])
" > gpurun_out/r03i_check.txt
