#!/bin/bash
# (The split-halves switch MSAT_GRU_SPLH was removed after this measurement: profiles/r02_ab_gru_la.log.)
# GRU forward (LDS-staged fp16x2) variants, alternating on one box, tape on: fragment lookahead 3 / 4
# blocks (ab/la3, la4; current 2) and the activation split in two halves (ab/splh, splhla3).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for rep in 1 2; do
  for lib in "" "$R/ab/la3.so" "$R/ab/la4.so" "$R/ab/splh.so" "$R/ab/splhla3.so"; do
    echo "== ${lib:-current}"
    env ${lib:+MARLSAT_LIB=$lib} GRU_KERNELS=h2r GRU_TAPE=True timeout -k 10 120 python $R/profiles/gru_r_bench.py 1400000 560000
  done
done
