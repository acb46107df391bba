#!/bin/bash
# round 6, call h: the planes weight gradient's small-column fixup: the planes tests with tiny A
# columns, first on the kernel WITHOUT the check (the previous commit's build, libmarlsat_nosmall.so: expected to
# miss the 4e-6 bar), then with it, then the dual-product timing (profiles/dual_bench.py) of both
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=$PWD/marl-sat_amd/marlsat/lib
MARLSAT_LIB=$L/libmarlsat_nosmall.so timeout -k 10 300 python -u -m pytest tests/test_planes_gpu.py -m gpu -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider -k "wgrad" > gpurun_out/r06h_planes_nosmall.log 2>&1
echo "without the check rc $?"; grep -E "passed|failed|^FAILED" gpurun_out/r06h_planes_nosmall.log | head -5
timeout -k 10 300 python -u -m pytest tests/test_planes_gpu.py tests/test_gemm_gpu.py -m gpu -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r06h_planes.log 2>&1
rc=$?
echo "with the check rc $rc"; tail -2 gpurun_out/r06h_planes.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for lib in libmarlsat libmarlsat_nosmall; do
    echo "== $lib $i" >> gpurun_out/r06h_dual_bench.log
    MARLSAT_LIB=$L/$lib.so timeout -k 10 120 python profiles/dual_bench.py >> gpurun_out/r06h_dual_bench.log 2>&1 || exit 1
  done
done
grep -E "==|wgrad" gpurun_out/r06h_dual_bench.log | cut -c1-200
