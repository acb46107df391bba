#!/bin/bash
# A/B of the GRU forward's epilogue h fetch: LDS-DMA in the last step (current, MSAT_GRU_HVE=1) vs
# global loads at the epilogue (ab/hve0.so), alternating on one box, without and with the tape.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for tape in False True; do
  for lib in "$R/ab/hve0.so" "" "$R/ab/hve0.so" ""; do
    echo "== ${lib:-current} tape=$tape"
    env ${lib:+MARLSAT_LIB=$lib} GRU_KERNELS=h2r GRU_TAPE=$tape timeout -k 10 120 python $R/profiles/gru_r_bench.py 1400000 560000
  done
done
