#!/bin/bash
# round 5, call s: the committed planes path end to end -- planes / gemm / GRU-backward / MAPPO tests, both dual
# product forms on the clause and var shapes (three alternations), and the training micro-batch with the packed rows
# in fp32 (MARLSAT_PLANES=0) and as planes (1), three alternations
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T="python -u -m pytest -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T -q tests/test_planes_gpu.py tests/test_gemm_gpu.py tests/test_gru_bwd_reduction_gpu.py tests/test_mappo_gpu.py > gpurun_out/r05s_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -2 gpurun_out/r05s_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u profiles/dual_bench.py 1316000 10 256 3 > gpurun_out/r05s_dual_clause.log 2>&1 || exit 4
timeout -k 10 300 python -u profiles/dual_bench.py 560000 10 128 3 > gpurun_out/r05s_dual_var.log 2>&1 || exit 5
cat gpurun_out/r05s_dual_clause.log gpurun_out/r05s_dual_var.log | grep '^{'
for i in 1 2 3; do
  for p in 0 1; do
    MARLSAT_PLANES=$p timeout -k 10 200 python -u profiles/mappo_probe.py uf100 256 512 train > gpurun_out/r05s_probe_p${p}_$i.json 2>&1 || exit 6
    echo "planes=$p run $i: $(grep -o '"s": [0-9.e-]*' gpurun_out/r05s_probe_p${p}_$i.json)"
  done
done
L=marl-sat_amd/marlsat/lib
for i in 1 2 3; do
  for v in cur prio; do
    lib=$L/libmarlsat.so; [ $v != cur ] && lib=$L/libmarlsat_$v.so
    echo -n "$v $i clause: "
    MARLSAT_LIB=$(readlink -f $lib) DUAL_ONLY="wgrad planes" timeout -k 10 120 python -u profiles/dual_bench.py 1316000 10 256 1 2>/dev/null | tail -1 || exit 7
  done
done 2>&1 | tee gpurun_out/r05s_wgrad_prio.log
