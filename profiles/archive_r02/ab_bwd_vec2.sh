#!/bin/bash
# GRU backward (profiles/gru_bwd_only.py, uf50 training shapes): the current build (vector column layout
# for the var cell only) against ab/bwdvecall.so (vector layout for the clause cell too) and
# ab/bwdvec0.so (scalar layout everywhere); alternating.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for rep in 1 2 3; do
  for lib in "" "$R/ab/bwdvecall.so" "$R/ab/bwdvec0.so"; do
    echo "== ${lib:-current}"
    env ${lib:+MARLSAT_LIB=$lib} timeout -k 10 120 python $R/profiles/gru_bwd_only.py 20
  done
done
