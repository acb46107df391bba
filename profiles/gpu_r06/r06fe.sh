#!/bin/bash
# round 6, call fe: N = 2 rehearsal of the driver's multi-GPU bench through the --gpus launcher on the final
# tree (gloo, both ranks on one GPU): env legs incl. the side legs, both MAPPO legs at T = 1, two timed cycles
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
MARLSAT_DIST_BACKEND=gloo MARLSAT_SHARE_GPU=1 timeout -k 10 900 python bench.py --gpus 2 --steps 20 --warmup 5 \
    --mappo uf100-430:4096:1,uf200-860:4096:1 --mappo-micro-gb 100 --cpu-budget 2 > gpurun_out/r06fe_dist2.json 2> gpurun_out/r06fe_dist2.err || { tail -30 gpurun_out/r06fe_dist2.err; exit 1; }
python3 -c "
import json
l=[x for x in open('gpurun_out/r06fe_dist2.json') if x.startswith('{')][-1]; d=json.loads(l)
print('n_gpus', d['n_gpus'], 'rccl_ranks', d['rccl_ranks'], d['dist_backend'], 'global_envs', d['config']['global_envs'], 'value', d['value'])
print('side legs', d['env_other_legs'])
for g in [d['mappo']]+d['mappo_other_legs']: print(g.get('config'), g['s_min_med_max'], g['params_check'])
"
