#!/bin/bash
# round 5, call w: rocprofv3 kernel trace of the headline MAPPO leg on the planes path (collect_mappo.sh): how long
# the planes weight gradient and its bf16x3 fixup take per launch in the real workload
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 bash profiles/collect_mappo.sh r05w > gpurun_out/r05w_collect.log 2>&1
rc=$?; echo "collect rc $rc"; tail -3 gpurun_out/r05w_collect.log
grep -E "wgrad|gemm_h2r16|gru_ln" gpurun_out/keep/r05w_mappo_uf100-430_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
exit $rc
