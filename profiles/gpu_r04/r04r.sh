#!/bin/bash
# round 4, call r: the default bench on the final tree (config-2 side leg added)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 800 python bench.py > gpurun_out/r04r_bench.json 2> gpurun_out/r04r_bench.err
rb=$?; echo "bench rc $rb"; tail -c 2000 gpurun_out/r04r_bench.json; exit $rb
