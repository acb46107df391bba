#!/bin/bash
# rocprofv3 evidence for the bench workload (run on the GPU box from the repo root):
#   pass 1: --kernel-trace --stats         (per-kernel durations, the full default bench command)
#   pass 2: --pmc FETCH_SIZE               (HBM read side; gfx950 reports 1/2 of wide reads)
#   pass 3: --pmc WRITE_SIZE               (HBM write side)
# Counters are collected in their own passes (no sys/runtime trace domains).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
TAG=${1:-r01}
shift || true
ARGS=${@:-"--steps 200 --warmup 20 --cpu-budget 0 --mappo="}  # the default bench's env leg
FULL=${MARLSAT_TRACE_ARGS:-"--steps 20 --warmup 5"}  # the driver's bench command (env + MAPPO legs)
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/bench.py $FULL > $OUT/trace_bench.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $R/bench.py $ARGS > $OUT/fetch_bench.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $R/bench.py $ARGS > $OUT/write_bench.log 2>&1
echo "profiles collected under $OUT"
