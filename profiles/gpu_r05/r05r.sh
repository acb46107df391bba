#!/bin/bash
# round 5, call r: planes weight gradient with the split's vector work held back to the 7th MFMA (cur) vs call q's
# build (q) vs the round's first committed pipelined build (prev); clause and var shapes, three alternations
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=marl-sat_amd/marlsat/lib
for i in 1 2 3; do
  for v in cur q prev; do
    lib=$L/libmarlsat.so; [ $v != cur ] && lib=$L/libmarlsat_$v.so
    echo -n "$v $i clause: "
    MARLSAT_LIB=$(readlink -f $lib) DUAL_ONLY="wgrad planes" timeout -k 10 120 python -u profiles/dual_bench.py 1316000 10 256 1 2>/dev/null | tail -1 || exit 3
  done
done 2>&1 | tee gpurun_out/r05r_wgrad.log
for v in cur q; do
  lib=$L/libmarlsat.so; [ $v != cur ] && lib=$L/libmarlsat_$v.so
  echo -n "$v var: "
  MARLSAT_LIB=$(readlink -f $lib) DUAL_ONLY="wgrad" timeout -k 10 120 python -u profiles/dual_bench.py 560000 10 128 2 2>/dev/null | tail -2 | tr '\n' ' ' || exit 4
  echo
done 2>&1 | tee -a gpurun_out/r05r_wgrad.log
