#!/bin/bash
# GRU backward (profiles/gru_bwd_only.py, uf50 training shapes): vector column layout (MSAT_BWD_VEC=1,
# the current build: a lane owns PER adjacent columns, dwordx2 accesses at H = 128) against the
# scalar layout (ab/bwdvec0.so: columns lane + 64 u, dword accesses); alternating.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for rep in 1 2 3; do
  for lib in "" "$R/ab/bwdvec0.so"; do
    echo "== ${lib:-current}"
    env ${lib:+MARLSAT_LIB=$lib} timeout -k 10 120 python $R/profiles/gru_bwd_only.py 20
  done
done
