#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for lib in ab/libmarlsat_probesync.so marl-sat_amd/marlsat/lib/libmarlsat.so; do
tag=$(basename $lib .so)
MARLSAT_LIB=$PWD/$lib PROBE_SYNC=1 timeout -k 10 300 python -u tests/probe_row257.py > gpurun_out/r03t_${tag}_a.log 2>&1 &
A=$!
MARLSAT_LIB=$PWD/$lib PROBE_SYNC=1 timeout -k 10 300 python -u tests/probe_row257.py > gpurun_out/r03t_${tag}_b.log 2>&1 &
B=$!
wait $A; wait $B
done
