#!/bin/bash
# GRU forward (LDS-staged fp16x2) time split: no epilogue (ab/gabl128), one k step (gabl256: prologue +
# epilogue), one k step and no epilogue (gabl384), against the current build; tape on and off.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for tape in False True; do
  for lib in "" "$R/ab/gabl128.so" "$R/ab/gabl256.so" "$R/ab/gabl384.so"; do
    echo "== ${lib:-current} tape=$tape"
    env ${lib:+MARLSAT_LIB=$lib} GRU_KERNELS=h2r GRU_TAPE=$tape timeout -k 10 120 python $R/profiles/gru_r_bench.py 1400000 560000
  done
done
