#!/bin/bash
# round 6, call fg: the final tree after the header-doc rebuild -- the full GPU suite and smoke()
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r06fg_gpu_tests.log 2>&1
rc=$?
echo "suite rc $rc"; tail -3 gpurun_out/r06fg_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06fg_smoke.log 2>&1
rc=$?
echo "smoke rc $rc"; tail -1 gpurun_out/r06fg_smoke.log
[ $rc -eq 0 ] || exit $rc
rc=$?
exit $rc
