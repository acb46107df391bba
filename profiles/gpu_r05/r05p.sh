#!/bin/bash
# round 5, call p: the planes weight gradient with the A split's LDS reads issued ahead of the fragment reads (cur)
# vs the committed order (prev); MFMA + split ablations of both (abl6c / abl6); planes tests; clause shape, three
# alternations
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T="python -u -m pytest -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T -q tests/test_planes_gpu.py > gpurun_out/r05p_planes_tests.log 2>&1
rc=$?; echo "planes tests rc $rc"; tail -2 gpurun_out/r05p_planes_tests.log
[ $rc -eq 0 ] || exit $rc
L=marl-sat_amd/marlsat/lib
for i in 1 2 3; do
  for v in cur prev abl6c abl6; do
    lib=$L/libmarlsat.so; [ $v != cur ] && lib=$L/libmarlsat_$v.so
    echo -n "$v $i: "
    MARLSAT_LIB=$(readlink -f $lib) DUAL_ONLY="wgrad planes" timeout -k 10 120 python -u profiles/dual_bench.py 1316000 10 256 1 2>/dev/null | tail -1 || exit 3
  done
done 2>&1 | tee gpurun_out/r05p_wgrad_split_first.log
