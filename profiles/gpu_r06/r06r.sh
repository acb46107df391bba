#!/bin/bash
# round 6, call r: the small-activation regression test on the product library (2^7 pre-scale) and, as the
# negative control, on a build of the same source with the scale set to 1 (libmarlsat_noasc.so: must fail)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gru_fused_gpu.py -k "small_activations or out_of_range" -v -s \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06r_small_act.log 2>&1
rc=$?; echo "product rc $rc"; grep -E "PASS|FAIL|passed|failed|small activations" gpurun_out/r06r_small_act.log | tail -12
[ $rc -eq 0 ] || exit $rc
MARLSAT_LIB=$PWD/marl-sat_amd/marlsat/lib/libmarlsat_noasc.so timeout -k 10 200 python -u -m pytest \
    tests/test_gru_fused_gpu.py -k small_activations -v -s --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r06r_small_act_noasc.log 2>&1
rc=$?; echo "unscaled build rc $rc (expected 1)"; grep -E "small activations|AssertionError|passed|failed" gpurun_out/r06r_small_act_noasc.log | tail -6
[ $rc -eq 1 ] && exit 0 || exit 3
