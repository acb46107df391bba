#!/bin/bash
# A/B of encoder variants on one box: probe uf200 / uf50 train+rollout under env switches.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ab
mkdir -p $OUT
for wl in uf200:256:32 uf50:1024:1366; do
  IFS=: read w r t <<< "$wl"
  for cfg in "MARLSAT_FUSE_PHI=1" "MARLSAT_FUSE_PHI=0" "MARLSAT_FUSE_PHI=0 MARLSAT_WGRAD_SKINNY=0" "MARLSAT_FUSE_PHI=1"; do
    tag=$(echo $cfg | tr ' =' '__')
    env $cfg timeout -k 10 200 python $R/profiles/mappo_probe.py $w $r $t > $OUT/${w}_$tag.json 2>>$OUT/err.log
    python -c "import json; d=json.load(open('$OUT/${w}_$tag.json')); print('$w', '$cfg', {k: round(v['samples_per_s'], 1) for k, v in d.items() if isinstance(v, dict)})"
  done
done
