#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u tests/probe_bwd_replay.py > gpurun_out/r03s_a.log 2>&1 &
A=$!
timeout -k 10 300 python -u tests/probe_bwd_replay.py > gpurun_out/r03s_b.log 2>&1 &
B=$!
wait $A; wait $B
