#!/bin/bash
# GRU forward epilogue in packed fp32 with DPP row sums (current, MSAT_GRU_PKE=1) against the scalar
# epilogue with shuffle sums (ab/pke0.so), alternating, tape off and on.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for tape in False True; do
  for lib in "$R/ab/pke0.so" "" "$R/ab/pke0.so" "" "$R/ab/pke0.so" ""; do
    echo "== ${lib:-current} tape=$tape"
    env ${lib:+MARLSAT_LIB=$lib} GRU_KERNELS=h2r GRU_TAPE=$tape timeout -k 10 120 python $R/profiles/gru_r_bench.py 1400000 560000
  done
done
