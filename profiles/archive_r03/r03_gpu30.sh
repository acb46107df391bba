#!/bin/bash
# rocprofv3 kernel traces of the two MAPPO legs alone (uf200 x 4096 T=2, uf100 x 4096 T=8): slices + stats
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash profiles/collect_mappo.sh r03 uf200-860:4096:2 > gpurun_out/r03_collect_uf200.log 2>&1 || { tail -20 gpurun_out/r03_collect_uf200.log; exit 1; }
bash profiles/collect_mappo.sh r03 uf100-430:4096:8 > gpurun_out/r03_collect_uf100.log 2>&1 || { tail -20 gpurun_out/r03_collect_uf100.log; exit 1; }
ls gpurun_out/keep
