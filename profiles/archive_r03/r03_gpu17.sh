#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for sy in 0 1; do
PROBE_SYNC=$sy timeout -k 10 300 python -u tests/probe_row257.py > gpurun_out/r03r_a$sy.log 2>&1 &
A=$!
PROBE_SYNC=$sy timeout -k 10 300 python -u tests/probe_row257.py > gpurun_out/r03r_b$sy.log 2>&1 &
B=$!
wait $A; wait $B
done
