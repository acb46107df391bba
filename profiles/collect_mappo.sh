#!/bin/bash
# rocprofv3 kernel trace of the bench's headline MAPPO leg alone (uf100-430 x 4096 envs, T = 8) and
# the per-kernel slice of its timed cycle (profiles/mappo_slice.py).   bash profiles/collect_mappo.sh r02
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02}
LEG=${2:-uf100-430:4096:8}
OUT=$R/gpurun_out/profm
mkdir -p $OUT $R/gpurun_out/keep
trap 'rm -rf $OUT' EXIT  # the raw trace is far larger than what gpurun copies back
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o m -- python3 $R/bench.py --steps 20 --warmup 5 --cpu-budget 0 --mappo $LEG > $OUT/bench.log 2>&1
W=${LEG%%:*}
python3 $R/profiles/mappo_slice.py $OUT/m_kernel_trace.csv $OUT/bench.log $R/gpurun_out/keep/${TAG}_mappo_${W}_slice.json
python3 $R/profiles/gaps.py $OUT/m_kernel_trace.csv ${GAP_WINDOW_S:-36} ${GAP_MIN_US:-3} > $R/gpurun_out/keep/${TAG}_mappo_${W}_gaps.txt || true
cp $OUT/m_kernel_stats.csv $R/gpurun_out/keep/${TAG}_mappo_${W}_kernel_stats.csv
grep '^{' $OUT/bench.log > $R/gpurun_out/keep/${TAG}_mappo_${W}_bench.json
rm -rf $OUT
