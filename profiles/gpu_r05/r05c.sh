#!/bin/bash
# round 5, call c: stamp test + dual-launch wbig cases + debug-build tests; the teacher-forced train-cycle tests
# with their printed margins (-s); the env legs with phase stamps; then ONE run of the uf50 L = 16 teacher-forced
# case on libmarlsat_debug.so with MARLSAT_DEBUG=1 (single process)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T="python -u -m pytest -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T -q tests/test_env_gpu.py tests/test_gemm_gpu.py tests/test_debug_build.py \
    -k "clock_stamps or dual_launches or debug" > gpurun_out/r05c_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -3 gpurun_out/r05c_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 $T -s -v tests/test_mappo_gpu.py -k every_adam_step > gpurun_out/r05c_parity_margins.log 2>&1
rm_=$?; echo "margins rc $rm_"; tail -6 gpurun_out/r05c_parity_margins.log
if [ $rm_ -ne 0 ] && [ $rm_ -ne 1 ]; then exit $rm_; fi
timeout -k 10 300 python bench.py --mappo '' --cpu-budget 0 > gpurun_out/r05c_bench_env.json 2> gpurun_out/r05c_bench_env.err
rb=$?; echo "bench rc $rb"
if [ $rb -ne 0 ]; then exit $rb; fi
MARLSAT_LIB=$GRAFT_REPO_ROOT/marl-sat_amd/marlsat/lib/libmarlsat_debug.so MARLSAT_DEBUG=1 timeout -k 10 600 $T -s -v \
    tests/test_mappo_gpu.py -k "every_adam_step and 50-218" > gpurun_out/r05c_debug_train_cycle.log 2>&1
rd=$?; echo "debug run rc $rd"; tail -4 gpurun_out/r05c_debug_train_cycle.log
exit $(( rc | rm_ | rd ))
