#!/bin/bash
# (The 16-wave kernel was removed after these measurements: profiles/r02_ab_gru_h4*.log)
# GRU forward: 16-wave form (MARLSAT_GRU_H4=1: two waves per 16-row group, 64 accumulator registers,
# four waves per SIMD) against the 8-wave LDS-staged kernel, alternating on one box, tape off and on.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for tape in False True; do
  for h4 in 0 1 0 1; do
    echo "== h4=$h4 tape=$tape"
    MARLSAT_GRU_H4=$h4 GRU_KERNELS=h2r GRU_TAPE=$tape timeout -k 10 120 python $R/profiles/gru_r_bench.py 1400000 560000
  done
done
