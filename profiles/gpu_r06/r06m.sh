#!/bin/bash
# round 6, call m: the headline-shape train cycle's step-1 gradient at FIXED parameters under each kernel family's
# alternative form (profiles/parity_attrib.py), for the CPU attribution of the default path's error
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/pdump2
MARLSAT_PARITY_DUMP=gpurun_out/pdump2 timeout -k 10 300 python -u -m pytest tests/test_mappo_gpu.py \
    -k "every_adam_step and 100-430 and fp16x2" -s -q --timeout 280 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r06m_dump.log 2>&1
rc=$?; echo "dump rc $rc"; grep "^margins" gpurun_out/r06m_dump.log | sed 's/loss err.*grad worst/grad worst/'
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u profiles/parity_attrib.py gpurun_out/pdump2/fp16x2_V100_L16_s4.npz 1 \
    gpurun_out/pdump2/attrib_s1.npz > gpurun_out/r06m_attrib.log 2>&1
rc=$?; echo "attrib rc $rc"; tail -12 gpurun_out/r06m_attrib.log; ls -la gpurun_out/pdump2
exit $rc
