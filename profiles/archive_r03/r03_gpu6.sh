#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 200 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 tests/probe_replica_check.py > gpurun_out/r03f_rc.log 2>&1
