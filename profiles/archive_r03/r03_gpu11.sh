#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out /tmp/rep
cmp() {
python - <<PY
import torch
r = [torch.load(f"/tmp/rep/rank{k}.pt", weights_only=True) for k in range(2)]
print("final finite", bool(torch.isfinite(r[0]["final"]).all()), bool(torch.isfinite(r[1]["final"]).all()), "equal", torch.equal(r[0]["final"], r[1]["final"]))
for s, (a, b) in enumerate(zip(r[0]["trace"], r[1]["trace"])):
    print(s, "p", a["params"][0].item(), b["params"][0].item(), "g", a["grads"][0].item(), b["grads"][0].item())
bad = (~torch.isfinite(r[0]["final"])).nonzero().flatten()
print("non-finite idx", bad[:10].tolist(), "count", bad.numel())
PY
}
for kt in 1 0; do
echo "=== bench flow, ktimer=$kt"
REPLICA_BENCH_FLOW=1 REPLICA_KTIMER=$kt MARLSAT_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 2955$kt tests/dist_replica_worker.py /tmp/rep 128 uf200-860 4096 1 16 100 1 > gpurun_out/r03k_rep_$kt.log 2>&1 || exit 1
cmp
done
