#!/bin/bash
# round-3 rocprofv3 evidence for the default bench: kernel trace of the full command + FETCH / WRITE passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash profiles/collect.sh r03 > gpurun_out/r03g_collect.log 2>&1 || { tail -20 gpurun_out/r03g_collect.log; exit 1; }
python3 profiles/summarize.py r03 > gpurun_out/r03g_summary.txt 2>&1 || { cat gpurun_out/r03g_summary.txt; exit 1; }
cp profiles/r03_kernel_stats.csv profiles/r03_pmc.json gpurun_out/ 
cat gpurun_out/r03g_summary.txt

cp gpurun_out/prof/trace_bench.log gpurun_out/r03g_trace_bench.log
rm -rf gpurun_out/prof gpurun_out/bench_mappo_*.json
