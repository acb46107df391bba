#!/bin/bash
# A/B of the x3 weight gradient: base library vs current build, and workgroup budgets.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for lib in "$R/ab/base.so" ""; do
  for wg in 512 768 1024; do
    echo "== ${lib:-current} wg=$wg"
    env ${lib:+MARLSAT_LIB=$lib} MARLSAT_WGRAD_WG=$wg timeout -k 10 120 python $R/profiles/wgrad_x3_only.py 20
  done
done
