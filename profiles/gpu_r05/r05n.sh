#!/bin/bash
# round 5, call n: the planes weight gradient -- product build vs the SIMD-partner staggered split (stg) and more
# ablations (MSAT_WGRAD_ABL 14: MFMAs + barriers only, 30: MFMAs only, 12: MFMAs + fragment reads, 6: MFMAs + split),
# clause shape, two alternations
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=marl-sat_amd/marlsat/lib
for i in 1 2; do
  for v in cur stg abl14 abl30 abl12 abl6; do
    lib=$L/libmarlsat.so; [ $v != cur ] && lib=$L/libmarlsat_$v.so
    echo -n "$v $i: "
    MARLSAT_LIB=$(readlink -f $lib) DUAL_ONLY="wgrad planes" timeout -k 10 120 python -u profiles/dual_bench.py 1316000 10 256 1 2>/dev/null | tail -1 || exit 3
  done
done 2>&1 | tee gpurun_out/r05n_wgrad_ablate.log
