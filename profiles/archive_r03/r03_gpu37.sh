#!/bin/bash
# MAPPO at SURVEY.md §8(d)'s profile: uf100-430 x 4096 envs, T = 32 (one timed update after the warm-up)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
# heartbeat: the timed update runs ~3 minutes without output
( while true; do date >> gpurun_out/r03f_heartbeat.log; sleep 50; done ) &
HB=$!
timeout -k 10 900 python bench.py --steps 5 --warmup 2 --cpu-budget 0 --mappo uf100-430:4096:32 > gpurun_out/r03f_t32.json 2> gpurun_out/r03f_t32.err
rc=$?
kill $HB
[ $rc -eq 0 ] || { tail -20 gpurun_out/r03f_t32.err; exit 1; }
python3 -c "
import json
l=[x for x in open('gpurun_out/r03f_t32.json') if x.startswith('{')][-1]; d=json.loads(l)
g=d['mappo']; print(g['config'], g['s_per_update'], g['samples_per_s'], g['adam_steps_per_s'], g['phase_ms'], g['params_check'])
"
