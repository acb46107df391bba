#!/bin/bash
# A/B of the fp16x2 GRU forward: activations to registers (MARLSAT_GRU_H2S=0) vs LDS-staged (default)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in 0 1 0 1; do
  echo "== MARLSAT_GRU_H2S=$v"
  MARLSAT_GRU_H2S=$v GRU_KERNELS=h2r timeout -k 10 120 python $R/profiles/gru_r_bench.py 1400000 560000
done
