#!/bin/bash
# bisect rank 1's first uf200 minibatch to the sample(s) with a non-finite gradient; fp64 oracle on it
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
PROBE_BISECT=1 timeout -k 10 500 python -u tests/probe_nan_grad.py > gpurun_out/r03y_bisect.log 2>&1
