#!/bin/bash
# HBM traffic of the training GRU forward (gru_ln_fused_fwd_h2s_kernel, clause cell, 1.4 M rows, with the
# tape): FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes over profiles/gru_r_bench.py, and the
# kernel trace of the same command for the launch duration.  Summary: profiles/pmc_gru_summary.py.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_gru_traffic
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export GRU_KERNELS=h2r GRU_TAPE=True GRU_REPS=5
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/profiles/gru_r_bench.py 1400000 560000 > $OUT/trace.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $R/profiles/gru_r_bench.py 1400000 560000 > $OUT/fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $R/profiles/gru_r_bench.py 1400000 560000 > $OUT/write.log 2>&1
python3 $R/profiles/pmc_gru_summary.py $OUT > $R/gpurun_out/pmc_gru_traffic.json
