#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for gb in 240 300 340; do
  timeout -k 10 300 python3 bench.py --cpu-budget 0 --steps 2 --warmup 1 --mappo uf100-430:4096:8 --mappo-micro-gb $gb > gpurun_out/r03m_micro_$gb.json 2> gpurun_out/r03m_micro_$gb.err || { tail -20 gpurun_out/r03m_micro_$gb.err; exit 1; }
  python3 -c "
import json,sys
l=[x for x in open('gpurun_out/r03m_micro_$gb.json') if x.startswith('{')][-1]; d=json.loads(l)['mappo']
print($gb, d['s_per_update'], d['config'].get('micro_batch'), d.get('peak_hbm_gb'), d['phase_ms'])
"
done
