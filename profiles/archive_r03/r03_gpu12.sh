#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u tests/probe_determinism.py 200 64 6 > gpurun_out/r03l_det200.log 2>&1
timeout -k 10 300 python -u tests/probe_determinism.py 100 256 6 > gpurun_out/r03l_det100.log 2>&1
