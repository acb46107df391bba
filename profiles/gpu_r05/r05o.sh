#!/bin/bash
# round 5, call o: the planes weight gradient with pass-major MFMA order (cur) vs the accumulator-major order
# (prev), and the MFMA + split ablation in both orders (abl6b / abl6), clause shape, three alternations
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=marl-sat_amd/marlsat/lib
for i in 1 2 3; do
  for v in cur prev abl6b abl6; do
    lib=$L/libmarlsat.so; [ $v != cur ] && lib=$L/libmarlsat_$v.so
    echo -n "$v $i: "
    MARLSAT_LIB=$(readlink -f $lib) DUAL_ONLY="wgrad planes" timeout -k 10 120 python -u profiles/dual_bench.py 1316000 10 256 1 2>/dev/null | tail -1 || exit 3
  done
done 2>&1 | tee gpurun_out/r05o_wgrad_order.log
