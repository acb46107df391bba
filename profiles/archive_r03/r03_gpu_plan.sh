#!/bin/bash
# learner tests touched by the per-minibatch size plan, then the MAPPO leg's trace and idle gaps
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_learner_glue_gpu.py tests/test_mappo_gpu.py tests/test_dist_learner_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03n_tests.log 2>&1 || { tail -30 gpurun_out/r03n_tests.log; exit 1; }
tail -2 gpurun_out/r03n_tests.log
bash profiles/collect_mappo.sh r03n > /dev/null 2>&1 || { echo trace failed; exit 1; }
head -3 gpurun_out/keep/r03n_mappo_uf100-430_gaps.txt
grep -o '"s_per_update": [0-9.]*' gpurun_out/keep/r03n_mappo_uf100-430_bench.json | head -1
