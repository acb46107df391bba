#!/bin/bash
# round 5, call x: the same MAPPO kernel trace with the packed rows in fp32 (MARLSAT_PLANES=0): the fp32-row
# weight gradient in the real workload, beside call w (planes)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
MARLSAT_PLANES=0 timeout -k 10 900 bash profiles/collect_mappo.sh r05x > gpurun_out/r05x_collect.log 2>&1
rc=$?; echo "collect rc $rc"; tail -3 gpurun_out/r05x_collect.log
grep -E "wgrad|gemm_h2r16|gru_ln" gpurun_out/keep/r05x_mappo_uf100-430_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
exit $rc
