#!/bin/bash
# A/B: base library (ab/base.so) vs current build on the GRU forward and data-gradient microbenchmarks.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for lib in "$R/ab/base.so" "" "$R/ab/base.so" ""; do
  echo "== ${lib:-current}"
  env ${lib:+MARLSAT_LIB=$lib} GRU_KERNELS=h2r,x3r timeout -k 10 120 python $R/profiles/gru_r_bench.py 1400000 560000
  env ${lib:+MARLSAT_LIB=$lib} timeout -k 10 120 python $R/profiles/dgrad_h2_bench.py 10
done
