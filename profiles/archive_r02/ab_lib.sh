#!/bin/bash
# A/B of two builds of libmarlsat.so on one box (MARLSAT_LIB override): probe + GRU bench, alternating.
# usage: bash profiles/ab_lib.sh <other.so> [workload S_roll S_train]
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OTHER=$1; WL=${2:-uf50}; SR=${3:-1024}; ST=${4:-1366}
for lib in "$OTHER" "" "$OTHER" ""; do
  tag=${lib:-current}
  env ${lib:+MARLSAT_LIB=$lib} timeout -k 10 200 python $R/profiles/mappo_probe.py $WL $SR $ST > $R/gpurun_out/ab_probe.json 2>/dev/null
  python -c "import json; d=json.load(open('$R/gpurun_out/ab_probe.json')); print('$(basename $tag)', {k: round(v['samples_per_s'], 1) for k, v in d.items() if isinstance(v, dict)})"
done
