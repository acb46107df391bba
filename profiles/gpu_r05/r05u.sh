#!/bin/bash
# round 5, call u: the default bench on the final tree, then rocprofv3 evidence for its env leg (kernel trace +
# stats, FETCH_SIZE and WRITE_SIZE passes, profiles/collect.sh with the env leg's own arguments)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 800 python bench.py > gpurun_out/r05u_bench.json 2> gpurun_out/r05u_bench.err
rb=$?
echo "bench rc $rb"; tail -c 400 gpurun_out/r05u_bench.json
[ $rb -eq 0 ] || exit $rb
MARLSAT_TRACE_ARGS="--steps 200 --warmup 20 --cpu-budget 0 --mappo=" timeout -k 10 900 bash profiles/collect.sh r05 > gpurun_out/r05u_collect.log 2>&1
rc=$?; echo "collect rc $rc"; tail -2 gpurun_out/r05u_collect.log
exit $rc
