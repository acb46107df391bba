#!/bin/bash
# GRU forward: where waves 0..3 / 4..7 issue a step's weight + activation DMA (block index; "-1" = step
# start): current (-1 / -1) against d8 (-1 / 8), d4, d6, d10 and d8s (d8 + waves 4..7 split at block 19);
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for rep in 1 2 3; do
  for lib in "" "$R/ab/d8.so" "$R/ab/d4.so" "$R/ab/d6.so" "$R/ab/d10.so" "$R/ab/d8s.so"; do
    echo "== ${lib:-current}"
    env ${lib:+MARLSAT_LIB=$lib} GRU_KERNELS=h2r GRU_TAPE=True timeout -k 10 120 python $R/profiles/gru_r_bench.py 1400000 560000
  done
done
