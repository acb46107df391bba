#!/bin/bash
# rank 1's shard of the N=2 run, alone (world 1): is the non-finite first gradient data-dependent?
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
REPLICA_SEED_OFFSET=1 REPLICA_DEBUG=1 REPLICA_BENCH_ENV=1 REPLICA_BENCH_FLOW=1 MARLSAT_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29582 tests/dist_replica_worker.py /tmp/rep1 128 uf200-860 4096 1 16 100 1 > gpurun_out/r03w_seed1_n1.log 2>&1
