#!/bin/bash
# A/B of the GRU forward: base library (ab/base.so) vs current build, alternating on one box.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for lib in "$R/ab/base.so" "" "$R/ab/base.so" ""; do
  echo "== ${lib:-current}"
  env ${lib:+MARLSAT_LIB=$lib} GRU_KERNELS=h2r timeout -k 10 120 python $R/profiles/gru_r_bench.py 1400000 560000
done
