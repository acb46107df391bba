#!/bin/bash
# N=2 replica run on bench.py's env/pool (512-step episodes, 1024 instances): which Adam step goes non-finite
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for n in 2 1; do
REPLICA_BENCH_ENV=1 REPLICA_BENCH_FLOW=1 REPLICA_KTIMER=1 MARLSAT_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nproc-per-node $n --master-addr 127.0.0.1 \
  --master-port 2957$n tests/dist_replica_worker.py /tmp/rep$n 128 uf200-860 4096 1 16 100 1 > gpurun_out/r03u_rep_n$n.log 2>&1 || exit 1
python - <<PY >> gpurun_out/r03u_rep_n$n.log
import torch, math
for k in range($n):
    r = torch.load(f"/tmp/rep$n/rank{k}.pt", weights_only=True)
    print("rank", k, "final finite", bool(torch.isfinite(r["final"]).all()), "bufs", r["bufs"])
    for s, t in enumerate(r["trace"]):
        print(" step", s, "p", t["params"][0].item(), "g", t["grads"][0].item())
PY
done
