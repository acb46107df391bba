set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -k "dual" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03c_tests.log 2>&1 &&
bash profiles/r03_ab.sh 3 profiles/dual_bench.py 1316000 20 > gpurun_out/r03c_ab_dual.log 2>&1 &&
bash profiles/pmc_dual.sh > gpurun_out/r03c_pmc_dual.log 2>&1
