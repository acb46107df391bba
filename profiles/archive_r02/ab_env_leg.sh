#!/bin/bash
# A/B of two library builds on the env leg only (uf200 x 4096): bench.py --mappo=, alternating.
# usage: bash profiles/ab_env_leg.sh <other.so> [extra bench args]
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OTHER=$1; shift || true
for lib in "$OTHER" "" "$OTHER" ""; do
  env ${lib:+MARLSAT_LIB=$lib} timeout -k 10 200 python $R/bench.py --steps 200 --warmup 20 --cpu-budget 0 --mappo= "$@" > $R/gpurun_out/ab_env.json 2>/dev/null
  python -c "import json; d=json.loads(open('$R/gpurun_out/ab_env.json').read().strip().splitlines()[-1]); print('$(basename ${lib:-current})', round(d['value'] / 1e6, 2), 'M/s', round(d['roofline']['kernel_ms'] * 1e3, 1), 'us', round(d['roofline']['frac'], 3))"
done
