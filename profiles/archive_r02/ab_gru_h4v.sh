#!/bin/bash
# (The 16-wave kernel was removed after these measurements: profiles/r02_ab_gru_h4*.log)
# 16-wave GRU forward variants (MARLSAT_GRU_H4=1): DMA of waves 8..15 before block 4 / 6 (ab/h4d4,
# h4d6), fragment lookahead 2 (h4la2), against the 8-wave kernel; tape on, alternating.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for rep in 1 2; do
  for v in "0:" "1:" "1:$R/ab/h4d4.so" "1:$R/ab/h4d6.so" "1:$R/ab/h4la2.so"; do
    h4=${v%%:*}; lib=${v#*:}
    echo "== h4=$h4 ${lib:-current}"
    env ${lib:+MARLSAT_LIB=$lib} MARLSAT_GRU_H4=$h4 GRU_KERNELS=h2r GRU_TAPE=True timeout -k 10 120 python $R/profiles/gru_r_bench.py 1400000 560000
  done
done
