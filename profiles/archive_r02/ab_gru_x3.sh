#!/bin/bash
# A/B of the x3 fused GRU forward: base library (ab/base.so) vs the current build, alternating.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for lib in "$R/ab/base.so" "" "$R/ab/base.so" ""; do
  echo "== ${lib:-current}"
  env ${lib:+MARLSAT_LIB=$lib} timeout -k 10 120 python $R/profiles/gru_x3_only.py 20
done
