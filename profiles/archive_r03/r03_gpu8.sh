#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p /tmp/rep
MARLSAT_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29544 tests/dist_replica_worker.py /tmp/rep 128 uf200-860 4096 1 16 100 1 > gpurun_out/r03h_rep.log 2>&1
python - <<PY >> gpurun_out/r03h_rep.log
import torch
r = [torch.load(f"/tmp/rep/rank{k}.pt", weights_only=True) for k in range(2)]
print("init equal", torch.equal(r[0]["init"], r[1]["init"]), "final equal", torch.equal(r[0]["final"], r[1]["final"]),
      "final finite", bool(torch.isfinite(r[0]["final"]).all()), bool(torch.isfinite(r[1]["final"]).all()))
for s, (a, b) in enumerate(zip(r[0]["trace"], r[1]["trace"])):
    print(s, "params eq", torch.equal(a["params"], b["params"]), "grads eq", torch.equal(a["grads"], b["grads"]),
          a["grads"][:3].tolist(), b["grads"][:3].tolist())
d = (r[0]["final"] - r[1]["final"]).abs()
print("final max diff", float(d.max()), "n diff", int((d > 0).sum()), "first idx", (d > 0).nonzero()[:5].flatten().tolist())
PY
