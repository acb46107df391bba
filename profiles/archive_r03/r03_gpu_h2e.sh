#!/bin/bash
# GRU forward with the per-row features in the epilogue (msat_gru_ln_fused_fwd_h2e): its tests, the network
# oracle tests that run it, the kernel timing against h2r, then the default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gru_fused_gpu.py tests/test_gnn_gpu.py tests/test_mappo_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03p_tests.log 2>&1 || { tail -40 gpurun_out/r03p_tests.log; exit 1; }
tail -2 gpurun_out/r03p_tests.log
for i in 1 2 3; do GRU_KERNELS=h2r,h2e timeout -k 10 200 python3 profiles/gru_r_bench.py >> gpurun_out/r03p_gru_h2e.log 2>&1 || exit 1; done
grep '^{' gpurun_out/r03p_gru_h2e.log | python3 -c "
import sys,json,collections
d=collections.defaultdict(list)
for l in sys.stdin:
    r=json.loads(l); d[(r['cell'],r['tape'],r['kernel'])].append(r['ms'])
for k,v in sorted(d.items()): print(k, sorted(v))
"
