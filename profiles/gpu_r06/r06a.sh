#!/bin/bash
# round 6, call a: the full GPU suite on the tree without the h2u GRU form (ABI version 2, stamp-buffer checks),
# then the teacher-forced train cycle on all three precision paths with its margins printed (verdict item 1)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r06a_gpu_tests.log 2>&1
rc=$?
echo "suite rc $rc"; tail -4 gpurun_out/r06a_gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests/test_mappo_gpu.py -k every_adam_step -s -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r06a_margins.log 2>&1
rc=$?
echo "margins rc $rc"; grep -c "^margins" gpurun_out/r06a_margins.log; tail -3 gpurun_out/r06a_margins.log
exit $rc
