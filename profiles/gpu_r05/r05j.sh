#!/bin/bash
# round 5, call j: the packed rows as fp16x2 planes (verdict item 5: G split once per row) -- the planes tests,
# the dual-product / GRU-backward tests they sit beside, then the dual products timed in both forms
# (clause shape 1.316 M rows x K1 256, var shape 560 K x 128), alternated three times on one box
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T="python -u -m pytest -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T -v tests/test_planes_gpu.py > gpurun_out/r05j_planes_tests.log 2>&1
rc=$?; echo "planes tests rc $rc"; tail -3 gpurun_out/r05j_planes_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 $T -q tests/test_gemm_gpu.py tests/test_gru_bwd_reduction_gpu.py > gpurun_out/r05j_gemm_tests.log 2>&1
rc=$?; echo "gemm tests rc $rc"; tail -3 gpurun_out/r05j_gemm_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u profiles/dual_bench.py 1316000 10 256 3 > gpurun_out/r05j_dual_clause.log 2>&1 || exit 4
timeout -k 10 300 python -u profiles/dual_bench.py 560000 10 128 3 > gpurun_out/r05j_dual_var.log 2>&1 || exit 5
cat gpurun_out/r05j_dual_clause.log gpurun_out/r05j_dual_var.log
timeout -k 10 400 $T -q tests/test_mappo_gpu.py > gpurun_out/r05j_mappo_tests.log 2>&1
rc=$?; echo "mappo tests rc $rc"; tail -3 gpurun_out/r05j_mappo_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for p in 0 1; do
    MARLSAT_PLANES=$p timeout -k 10 200 python -u profiles/mappo_probe.py uf100 256 512 train > gpurun_out/r05j_probe_p${p}_$i.json 2>&1 || exit 6
    echo "planes=$p run $i: $(grep -o '"s": [0-9.e-]*' gpurun_out/r05j_probe_p${p}_$i.json)"
  done
done
