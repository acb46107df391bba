#!/bin/bash
# round 4, call n: unit counters of the dual data gradient and the GRU forward (clause training shape)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
DUAL_ONLY=dgrad timeout -k 10 500 bash profiles/pmc_units.sh dgrad profiles/dual_bench.py 1316000 3 256 > gpurun_out/r04n_units_dgrad.json 2>&1
echo "dgrad rc $?"
GRU_KERNELS=h2r GRU_TAPE=True GRU_REPS=3 timeout -k 10 500 bash profiles/pmc_units.sh gru profiles/gru_r_bench.py 1400000 560000 > gpurun_out/r04n_units_gru.json 2>&1
echo "gru rc $?"
