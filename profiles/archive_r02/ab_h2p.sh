#!/bin/bash
# A/B of the fp16x2 GRU forward: 128-row tiles, one workgroup per CU (default) vs 64-row ping-pong
# tiles, two workgroups per CU (MARLSAT_GRU_H2P=1), alternating on one box.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in 0 1 0 1; do
  echo "== MARLSAT_GRU_H2P=$v"
  MARLSAT_GRU_H2P=$v GRU_KERNELS=h2r timeout -k 10 120 python $R/profiles/gru_r_bench.py 1400000 560000
done
