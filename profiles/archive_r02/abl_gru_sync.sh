#!/bin/bash
# Synchronisation ablations of the staged GRU forward (ab/gabl32: no step-end barrier, gabl64: no step-end
# vmcnt wait, gabl96: neither; timing only) + SQ counters of the product kernel.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for lib in "" $R/ab/gabl32.so $R/ab/gabl64.so $R/ab/gabl96.so ""; do
  echo "== ${lib:-current}"
  env ${lib:+MARLSAT_LIB=$lib} GRU_KERNELS=h2r GRU_TAPE=False timeout -k 10 120 python $R/profiles/gru_r_bench.py 1400000 560000
done
GRU_KERNELS=h2r GRU_TAPE=False GRU_REPS=3 bash $R/profiles/pmc_sq.sh h2s $R/profiles/gru_r_bench.py 1400000 560000
