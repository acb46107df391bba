#!/bin/bash
# round 4, call s: texture-path probe -- L2-resident read rates and TA / TD busy, loads vs LDS-DMA
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 120 python profiles/l2_probe.py 2048 5 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04s_l2_probe.log
timeout -k 10 400 bash profiles/pmc_units.sh l2 profiles/l2_probe.py 2048 2 > gpurun_out/r04s_units_l2.json 2>&1
echo "units rc $?"
