#!/bin/bash
# Round evidence on the GPU box: collect.sh (trace of the full bench command + PMC passes of the env
# leg), summarize.py, then keep only the summaries under gpurun_out/keep/ (the raw kernel trace of
# the MAPPO legs is >64 MiB; gpurun merges back at most that).   bash profiles/collect_r.sh r02
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02}
bash $R/profiles/collect.sh $TAG
cd $R
python3 profiles/summarize.py $TAG uf200-860/B4096/int32
mkdir -p gpurun_out/keep
cp profiles/${TAG}_kernel_stats.csv profiles/${TAG}_pmc.json gpurun_out/keep/
cp gpurun_out/prof/trace_bench.log gpurun_out/keep/${TAG}_trace_bench.log
rm -rf gpurun_out/prof
