#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u tests/probe_flow_determinism.py uf200-860 1024 1 > gpurun_out/r03m_flowdet.log 2>&1
