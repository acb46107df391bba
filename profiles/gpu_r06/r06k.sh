#!/bin/bash
# round 6, call k: final tree -- the full GPU suite, smoke(), and the teacher-forced train cycle on all three
# precision paths with per-step margins printed (verdict item 1)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r06k_gpu_tests.log 2>&1
rc=$?
echo "suite rc $rc"; tail -4 gpurun_out/r06k_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06k_smoke.log 2>&1
rc=$?
echo "smoke rc $rc"; tail -2 gpurun_out/r06k_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_mappo_gpu.py -k every_adam_step -s -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r06k_margins.log 2>&1
rc=$?
echo "margins rc $rc"; grep -c "^margins" gpurun_out/r06k_margins.log; tail -3 gpurun_out/r06k_margins.log
exit $rc
