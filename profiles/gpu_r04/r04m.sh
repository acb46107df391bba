#!/bin/bash
# round 4, call m: SQ counters of the dual data gradient (where its wave cycles go), and the counter list
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export DUAL_ONLY=dgrad
timeout -k 10 200 bash profiles/pmc_sq.sh dgrad profiles/dual_bench.py 1316000 3 256 > gpurun_out/r04m_sq.txt 2>&1
echo "sq rc $?"; cat gpurun_out/r04m_sq.txt | tail -5
cd /tmp && timeout -s KILL 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/r04m_counters.txt 2>&1; echo "list rc $?"
