#!/bin/bash
# round 5, call m: ablations of the planes weight gradient (libmarlsat_ablN.so, MSAT_WGRAD_ABL bits: 1 no MFMAs,
# 2 no fragment reads, 4 no DMAs, 8 no A split; 6 = only MFMAs + split) against the product build, clause shape,
# two alternations -- what bounds the kernel
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=marl-sat_amd/marlsat/lib
for i in 1 2; do
  for v in cur abl1 abl2 abl4 abl8 abl6; do
    lib=$L/libmarlsat.so; [ $v != cur ] && lib=$L/libmarlsat_$v.so
    echo -n "$v $i: "
    MARLSAT_LIB=$(readlink -f $lib) DUAL_ONLY="wgrad planes" timeout -k 10 120 python -u profiles/dual_bench.py 1316000 10 256 1 2>/dev/null | tail -1 || exit 3
  done
done 2>&1 | tee gpurun_out/r05m_wgrad_ablate.log
