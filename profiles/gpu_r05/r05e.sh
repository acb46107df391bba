#!/bin/bash
# round 5, call e: env kernel with problem_idx-independent loads in the first round trip (bit-exact env tests,
# stamps), env legs with tail statistics; then the uf100 L = 16 rollout-value outlier: phi folding off, and the
# register-A GRU kernels with IEEE gate functions (libmarlsat_ieee.so, -DMSAT_GRU_IEEE_GATES)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T="python -u -m pytest -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T -q tests/test_env_gpu.py > gpurun_out/r05e_env_tests.log 2>&1
rc=$?; echo "env tests rc $rc"; tail -2 gpurun_out/r05e_env_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --mappo '' --cpu-budget 0 > gpurun_out/r05e_bench_env.json 2> gpurun_out/r05e_bench_env.err
rb=$?; echo "bench rc $rb"; cp gpurun_out/bench_env_stamps_n1.json gpurun_out/r05e_env_stamps.json
if [ $rb -ne 0 ]; then exit $rb; fi
K="every_adam_step and 100-430"
for cfg in "fp16x2 0 std" "fp32 0 std" "fp16x2 1 ieee" "bf16x3 1 ieee"; do
  set -- $cfg
  LIB=$GRAFT_REPO_ROOT/marl-sat_amd/marlsat/lib/libmarlsat.so
  [ $3 = ieee ] && LIB=$GRAFT_REPO_ROOT/marl-sat_amd/marlsat/lib/libmarlsat_ieee.so
  MARLSAT_PRECISION=$1 MARLSAT_FUSE_PHI=$2 MARLSAT_LIB=$LIB timeout -k 10 300 $T -s -v tests/test_mappo_gpu.py -k "$K" \
      > gpurun_out/r05e_uf100_$1_phi$2_$3.log 2>&1
  r=$?; echo "$cfg rc $r"; grep -E "rollout V|worst ratio" gpurun_out/r05e_uf100_$1_phi$2_$3.log | head -3
  if [ $r -ne 0 ] && [ $r -ne 1 ]; then exit $r; fi
done
exit 0
