#!/bin/bash
# round 4, call f: HBM read rate of the data gradient's activation pattern (strips vs rows)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 180 python profiles/strip_probe.py 1316000 10 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04f_strip_probe.log
