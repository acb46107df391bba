#!/bin/bash
# round 4, call a: full GPU suite + default bench on the first round-4 tree
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04a_gpu_tests.log 2>&1
rc=$?
echo "tests rc $rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 700 python bench.py > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err
rb=$?
echo "bench rc $rb"
tail -3 gpurun_out/r04a_gpu_tests.log
exit $rb
