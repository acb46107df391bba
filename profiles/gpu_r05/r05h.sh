#!/bin/bash
# round 5, call h: the unit-half GRU forward (MARLSAT_GRU_FORM=h2u: 256-row tiles, two passes over the hidden
# units) -- GRU forward tests on both forms, then the microbenchmark alternating h2s / h2u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T="python -u -m pytest -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T -q tests/test_gru_fused_gpu.py -k "h2u or h2s" > gpurun_out/r05h_gru_tests.log 2>&1
rc=$?; echo "gru tests rc $rc"; tail -4 gpurun_out/r05h_gru_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2 3; do
  for f in h2s h2u; do
    MARLSAT_GRU_FORM=$f timeout -k 10 120 python profiles/gru_r_bench.py > gpurun_out/r05h_gru_bench_${f}_$i.log 2>&1 || exit 3
    echo "$f $i"; grep -h "h2r" gpurun_out/r05h_gru_bench_${f}_$i.log | head -4
  done
done
exit 0
