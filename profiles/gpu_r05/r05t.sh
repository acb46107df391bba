#!/bin/bash
# round 5, call t (and tb): final validation -- the whole GPU test suite and smoke() on the committed tree
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T="python -u -m pytest -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T -q tests > gpurun_out/r05t_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc $rc"; tail -3 gpurun_out/r05t_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05t_smoke.log 2>&1
rc=$?; echo "smoke rc $rc"; tail -2 gpurun_out/r05t_smoke.log
exit $rc
