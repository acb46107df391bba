#!/bin/bash
# data gradient with whole-row activation loads + row_ror:8 exchange: GEMM / network / MAPPO tests, then
# the dual launches A/B against the previous build (bit checksums must agree)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gemm_gpu.py tests/test_gnn_gpu.py tests/test_mappo_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03aa_tests.log 2>&1 || { tail -40 gpurun_out/r03aa_tests.log; exit 1; }
tail -1 gpurun_out/r03aa_tests.log
DUAL_CHECKSUM=1 LIBS="base" bash profiles/r03_ab_multi.sh 3 profiles/dual_bench.py > gpurun_out/r03aa_ab_dgrad_rows.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03aa_ab_dgrad_rows.log
