#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u tests/probe_mappo_finite.py uf200-860 4096 1 100 > gpurun_out/r03g_finite_uf200.log 2>&1
timeout -k 10 400 python -u tests/probe_mappo_finite.py uf100-430 4096 2 240 > gpurun_out/r03g_finite_uf100.log 2>&1
