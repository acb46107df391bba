#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dist_learner_gpu.py -k replicas -v --timeout 300 --timeout-method thread > gpurun_out/r03e_replicas.log 2>&1
