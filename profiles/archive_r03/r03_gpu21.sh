#!/bin/bash
# N=2 replica run on bench.py's env/pool with per-step finiteness hooks
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
REPLICA_DEBUG=1 REPLICA_BENCH_ENV=1 REPLICA_BENCH_FLOW=1 MARLSAT_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29581 tests/dist_replica_worker.py /tmp/rep2 128 uf200-860 4096 1 16 100 1 > gpurun_out/r03v_rep_n2.log 2>&1
