#!/bin/bash
# GRU forward tape stores non-temporal (ab/nt.so, built with a since-removed MSAT_GRU_NT=1 switch) against plain stores (current),
# alternating, tape on.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for lib in "$R/ab/nt.so" "" "$R/ab/nt.so" "" "$R/ab/nt.so" ""; do
  echo "== ${lib:-current} tape=True"
  env ${lib:+MARLSAT_LIB=$lib} GRU_KERNELS=h2r GRU_TAPE=True timeout -k 10 120 python $R/profiles/gru_r_bench.py 1400000 560000
done
