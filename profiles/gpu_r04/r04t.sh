#!/bin/bash
# round 4, call t: texture-path probe over row strides (register-A and weight-piece patterns)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 200 python profiles/l2_probe.py 2048 5 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04t_l2_strides.log
