#!/bin/bash
# round 4, call g: full GPU suite + default bench on the round-4 tree
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04g_gpu_tests.log 2>&1
rc=$?
echo "tests rc $rc"
tail -5 gpurun_out/r04g_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 800 python bench.py > gpurun_out/r04g_bench.json 2> gpurun_out/r04g_bench.err
rb=$?
echo "bench rc $rb"
exit $rb
