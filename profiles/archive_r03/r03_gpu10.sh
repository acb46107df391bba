#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --mappo uf200-860:4096:1,uf100-430:4096:2 --cpu-budget 0 > gpurun_out/r03j_n1.json 2> gpurun_out/r03j_n1.err
python3 -c "
import json
l=[x for x in open('gpurun_out/r03j_n1.json') if x.startswith('{')][-1]; d=json.loads(l)
for leg in d['mappo_other_legs']+[d['mappo']]: print(leg['config']['workload'], leg['params_check'], leg['s_per_update'])
" > gpurun_out/r03j_check.txt
