#!/bin/bash
# round 3: full GPU suite + smoke + default bench after the round-3 pruning
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03b_gpu_tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03b_smoke.log 2>&1 &&
timeout -k 10 900 python bench.py > gpurun_out/r03b_bench.json 2> gpurun_out/r03b_bench.err
