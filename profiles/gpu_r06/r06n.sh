#!/bin/bash
# round 6, call n: the GRU forward with its activations scaled by 2^7 before the fp16x2 split -- GRU / network
# tests, the step-1 gradient at the round's fixed parameters (scratch/: the call-m dump) for the attribution,
# and the teacher-forced train cycle's margins on all cases and paths
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/pdump3
timeout -k 10 400 python -u -m pytest tests/test_gru_fused_gpu.py tests/test_gnn_gpu.py -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r06n_gru_tests.log 2>&1
rc=$?; echo "gru/gnn tests rc $rc"; tail -2 gpurun_out/r06n_gru_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u profiles/parity_attrib.py scratch/fp16x2_V100_L16_s4.npz 1 gpurun_out/pdump3/attrib_s1.npz \
    > gpurun_out/r06n_attrib.log 2>&1
rc=$?; echo "attrib rc $rc"; tail -3 gpurun_out/r06n_attrib.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_mappo_gpu.py -k every_adam_step -s -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r06n_margins.log 2>&1
rc=$?; echo "margins rc $rc"; grep "^margins" gpurun_out/r06n_margins.log | sed 's/loss err.*grad worst/grad worst/'
exit $rc
