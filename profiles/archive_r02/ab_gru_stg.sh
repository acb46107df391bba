#!/bin/bash
# GRU forward stagger of SIMD partners (MSAT_GRU_STG bits 1 split, 2 DMA issue of waves 4..7),
# against the current build, alternating on one box, tape on.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for rep in 1 2; do
  for lib in "" "$R/ab/stg1.so" "$R/ab/stg2.so" "$R/ab/stg3.so"; do
    echo "== ${lib:-current}"
    env ${lib:+MARLSAT_LIB=$lib} GRU_KERNELS=h2r GRU_TAPE=True timeout -k 10 120 python $R/profiles/gru_r_bench.py 1400000 560000
  done
done
