#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u tests/probe_determinism.py 200 64 10 > gpurun_out/r03q_alone.log 2>&1
timeout -k 10 300 python -u tests/probe_determinism.py 200 64 10 > gpurun_out/r03q_a.log 2>&1 &
A=$!
timeout -k 10 300 python -u tests/probe_determinism.py 200 64 10 > gpurun_out/r03q_b.log 2>&1 &
B=$!
wait $A; wait $B
