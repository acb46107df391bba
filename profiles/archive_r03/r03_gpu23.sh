#!/bin/bash
# rank 1's first uf200 minibatch: non-finite gradients per precision path
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
PROBE_CALLS=1 timeout -k 10 300 python -u tests/probe_nan_grad.py > gpurun_out/r03x_default.log 2>&1 &&
MARLSAT_PRECISION=bf16x3 timeout -k 10 300 python -u tests/probe_nan_grad.py > gpurun_out/r03x_bf16x3.log 2>&1 &&
MARLSAT_PRECISION=fp32 timeout -k 10 300 python -u tests/probe_nan_grad.py > gpurun_out/r03x_fp32.log 2>&1
