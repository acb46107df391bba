#!/bin/bash
# round 6, call fb: the final tree's default bench (env legs, MAPPO legs + the fp32-path cycle), then rocprofv3
# evidence for the env leg (kernel trace + stats, FETCH_SIZE and WRITE_SIZE passes) summarised per kernel
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python bench.py > gpurun_out/r06fb_bench.json 2> gpurun_out/r06fb_bench.err
rb=$?
echo "bench rc $rb"; tail -c 1200 gpurun_out/r06fb_bench.json
[ $rb -eq 0 ] || exit $rb
rm -rf gpurun_out/prof
MARLSAT_TRACE_ARGS="--steps 200 --warmup 20 --cpu-budget 0 --mappo=" timeout -k 10 900 bash profiles/collect.sh r06 > gpurun_out/r06fb_collect.log 2>&1
rc=$?; echo "collect rc $rc"; tail -2 gpurun_out/r06fb_collect.log
[ $rc -eq 0 ] || exit $rc
python profiles/pmc_env_summary.py gpurun_out/prof gpurun_out/r06fb_env_pmc_traffic.json
