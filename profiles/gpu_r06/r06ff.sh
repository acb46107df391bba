#!/bin/bash
# round 6, call ff: fixed-parameter gradients of the uf50 L = 16 (step 3) and uf200 A = 25 L = 8 (step 1) train cycles
# on the default, bf16x3 and fp32 paths (profiles/parity_attrib.py), for the CPU comparison with the oracle
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/pdump4
MARLSAT_PARITY_DUMP=gpurun_out/pdump4 timeout -k 10 400 python -u -m pytest tests/test_mappo_gpu.py \
    -k "every_adam_step and fp16x2 and (50-218 or 200-860)" -s -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r06ff_dump.log 2>&1
rc=$?; echo "dump rc $rc"; ls gpurun_out/pdump4
[ $rc -eq 0 ] || exit $rc
export ATTRIB_CASES=default,bf16x3,fp32
timeout -k 10 300 python -u profiles/parity_attrib.py gpurun_out/pdump4/fp16x2_V50_L16_s4.npz 3 gpurun_out/pdump4/attrib_uf50_s3.npz \
    > gpurun_out/r06ff_attrib.log 2>&1 && \
timeout -k 10 300 python -u profiles/parity_attrib.py gpurun_out/pdump4/fp16x2_V200_L8_s4.npz 1 gpurun_out/pdump4/attrib_uf200_s1.npz \
    >> gpurun_out/r06ff_attrib.log 2>&1
rc=$?; echo "attrib rc $rc"; grep -v amdgpu gpurun_out/r06ff_attrib.log | tail -8; du -sh gpurun_out/pdump4
exit $rc
