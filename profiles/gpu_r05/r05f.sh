#!/bin/bash
# round 5, call f: accurate tanh in the register-A GRU epilogues -- GRU tests, the network depth tests, the
# teacher-forced train-cycle tests (margins), then the GRU forward microbenchmark alternating the previous
# build (libmarlsat_abA.so: 2 sigma(2x) - 1) and this one
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T="python -u -m pytest -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $T -q tests/test_gru_fused_gpu.py tests/test_gnn_gpu.py > gpurun_out/r05f_gru_gnn_tests.log 2>&1
rc=$?; echo "gru/gnn tests rc $rc"; tail -3 gpurun_out/r05f_gru_gnn_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for P in fp16x2 bf16x3; do
  MARLSAT_PRECISION=$P timeout -k 10 400 $T -s -v tests/test_mappo_gpu.py -k every_adam_step > gpurun_out/r05f_margins_$P.log 2>&1
  r=$?; echo "$P margins rc $r"; grep -E "rollout: |PASSED|FAILED" gpurun_out/r05f_margins_$P.log | head -12
  if [ $r -ne 0 ] && [ $r -ne 1 ]; then exit $r; fi
done
L=$GRAFT_REPO_ROOT/marl-sat_amd/marlsat/lib
for i in 1 2 3; do
  for v in abA cur; do
    lib=$L/libmarlsat.so; [ $v = abA ] && lib=$L/libmarlsat_abA.so
    MARLSAT_LIB=$lib timeout -k 10 120 python profiles/gru_r_bench.py > gpurun_out/r05f_gru_bench_${v}_$i.log 2>&1 || exit 3
    echo "$v $i"; grep -h "h2r" gpurun_out/r05f_gru_bench_${v}_$i.log | head -4
  done
done
exit 0
