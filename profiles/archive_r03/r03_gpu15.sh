#!/bin/bash
# determinism under contention: two processes run the forward + backward repetition probe at once
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u tests/probe_determinism.py 200 64 10 > gpurun_out/r03o_det_a.log 2>&1 &
A=$!
timeout -k 10 400 python -u tests/probe_determinism.py 200 64 10 > gpurun_out/r03o_det_b.log 2>&1 &
B=$!
wait $A; ra=$?
wait $B; rb=$?
echo "rc $ra $rb"
