#!/bin/bash
# A/B of the data gradient: base library (ab/base.so) vs current build, alternating.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for lib in "$R/ab/base.so" "" "$R/ab/base.so" ""; do
  echo "== ${lib:-current}"
  env ${lib:+MARLSAT_LIB=$lib} timeout -k 10 120 python $R/profiles/dgrad_h2_bench.py 10
done
