#!/bin/bash
# round 4, call y: final tree -- smoke(), the full GPU suite, the default bench
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04y_smoke.log 2>&1
rc=$?; echo "smoke rc $rc"; tail -1 gpurun_out/r04y_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04y_gpu_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -2 gpurun_out/r04y_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python bench.py > gpurun_out/r04y_bench.json 2> gpurun_out/r04y_bench.err
rb=$?; echo "bench rc $rb"; exit $rb
