#!/bin/bash
# GRU backward (profiles/gru_bwd_only.py, uf50 training shapes): var-cell form compiled for 5 waves per
# SIMD (ab/occ5: __launch_bounds__(256, 5), spills), with a 1,280-block grid (occ5b), the grid alone
# (b1280), against the current build (4 waves per SIMD, 1,024 blocks); alternating.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for rep in 1 2; do
  for lib in "" "$R/ab/occ5.so" "$R/ab/occ5b.so" "$R/ab/b1280.so"; do
    echo "== ${lib:-current}"
    env ${lib:+MARLSAT_LIB=$lib} timeout -k 10 120 python $R/profiles/gru_bwd_only.py 10
  done
done
