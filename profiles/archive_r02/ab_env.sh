#!/bin/bash
# A/B of an env switch on one box: probe (train + rollout) alternating "VAR=a" / "VAR=b".
# usage: bash profiles/ab_env.sh "VAR=a" "VAR=b" [workload S_roll S_train]
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
A=$1; B=$2; WL=${3:-uf50}; SR=${4:-1024}; ST=${5:-1366}
for cfg in "$A" "$B" "$A" "$B"; do
  env $cfg timeout -k 10 200 python $R/profiles/mappo_probe.py $WL $SR $ST > $R/gpurun_out/ab_probe.json 2>/dev/null
  python -c "import json; d=json.load(open('$R/gpurun_out/ab_probe.json')); print('$cfg', {k: round(v['samples_per_s'], 1) for k, v in d.items() if isinstance(v, dict)})"
done
