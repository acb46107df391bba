#!/bin/bash
# round 4, call h: rocprofv3 evidence for the round-4 tree -- env leg kernel trace + FETCH/WRITE passes,
# the MAPPO uf100 leg's kernel trace slice, and the GRU forward's PMC traffic
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
MARLSAT_TRACE_ARGS="--steps 20 --warmup 5 --mappo=" timeout -k 10 700 bash profiles/collect.sh r04 || exit $?
echo "env profiles rc 0"
timeout -k 10 400 bash profiles/pmc_gru_traffic.sh || exit $?
echo "gru pmc rc 0"; cat gpurun_out/pmc_gru_traffic.json
timeout -k 10 700 bash profiles/collect_mappo.sh r04 || exit $?
echo "mappo trace rc 0"; cat gpurun_out/keep/r04_mappo_uf100-430_bench.json | head -c 600
