#!/bin/bash
# round 6, call q: rocprofv3 kernel trace of the headline MAPPO leg on the final tree (profiles/collect_mappo.sh)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 bash profiles/collect_mappo.sh r06q > gpurun_out/r06q_collect.log 2>&1
rc=$?; echo "collect rc $rc"; tail -3 gpurun_out/r06q_collect.log; ls gpurun_out/keep | grep r06q
exit $rc
