#!/bin/bash
# round 4, call p: unit counters of the dual weight gradient (clause training shape)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
DUAL_ONLY=wgrad timeout -k 10 500 bash profiles/pmc_units.sh wgrad profiles/dual_bench.py 1316000 3 256 > gpurun_out/r04p_units_wgrad.json 2>&1
echo "wgrad rc $?"
