#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out /tmp/rep1 /tmp/rep2
for i in 1 2; do
REPLICA_BENCH_FLOW=1 REPLICA_KTIMER=0 MARLSAT_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 2956$i tests/dist_replica_worker.py /tmp/rep$i 128 uf200-860 1024 1 16 100 1 > gpurun_out/r03n_rep_$i.log 2>&1 || exit 1
done
python - <<PY
import torch
for k in range(2):
    a = torch.load(f"/tmp/rep1/rank{k}.pt", weights_only=True); b = torch.load(f"/tmp/rep2/rank{k}.pt", weights_only=True)
    print("rank", k, "final equal across runs", torch.equal(a["final"], b["final"]))
    for key in a["bufs"]:
        if a["bufs"][key] != b["bufs"][key]: print("  buf differs", key, a["bufs"][key], b["bufs"][key])
    for s, (x, y) in enumerate(zip(a["trace"], b["trace"])):
        if not torch.equal(x["grads"], y["grads"]): print("  first differing grad step", s, x["grads"][0].item(), y["grads"][0].item()); break
PY
