#!/bin/bash
# N=2 rehearsal (gloo, both ranks on this GPU) with the filtered bench pool: params finite + identical
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
MARLSAT_DIST_BACKEND=gloo MARLSAT_SHARE_GPU=1 timeout -k 10 700 python bench.py --gpus 2 --steps 20 --warmup 5 \
    --mappo uf200-860:4096:1,uf100-430:4096:1 --mappo-micro-gb 100 --cpu-budget 0 > gpurun_out/r03z_dist2.json 2> gpurun_out/r03z_dist2.err
python3 -c "
import json
l=[x for x in open('gpurun_out/r03z_dist2.json') if x.startswith('{')][-1]; d=json.loads(l)
for leg in d['mappo_other_legs']+[d['mappo']]: print(leg['config']['workload'], leg['params_check'], leg['s_per_update'])
" > gpurun_out/r03z_check.txt
