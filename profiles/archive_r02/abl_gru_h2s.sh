#!/bin/bash
# Ablations of the LDS-staged fp16x2 GRU forward (ab/gabl<N>.so built by profiles/build_abl.sh with
# -DMSAT_GRU_ABL=N): timing only.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for lib in "" $R/ab/gabl1.so $R/ab/gabl2.so $R/ab/gabl3.so $R/ab/gabl4.so $R/ab/gabl8.so $R/ab/gabl16.so ""; do
  echo "== ${lib:-current}"
  env ${lib:+MARLSAT_LIB=$lib} GRU_KERNELS=h2r GRU_TAPE=False timeout -k 10 120 python $R/profiles/gru_r_bench.py 1400000 560000
done
