#!/bin/bash
# round 5, call v: (1) the planes weight gradient with the row-exponent table (libmarlsat_dlt.so, 4 DMA pieces per
# wave and slab) vs the product build (5 pieces), clause and var shapes, three alternations; (2) the headline MAPPO
# leg (uf100-430 x 4096, T = 8, three timed cycles) with the packed rows in fp32 (MARLSAT_PLANES=0) and as planes
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=marl-sat_amd/marlsat/lib
for i in 1 2 3; do
  for v in cur dlt; do
    lib=$L/libmarlsat.so; [ $v != cur ] && lib=$L/libmarlsat_$v.so
    echo -n "$v $i clause: "
    MARLSAT_LIB=$(readlink -f $lib) timeout -k 10 120 python -u profiles/dual_bench.py 1316000 10 256 1 2>/dev/null | grep "wgrad planes" || exit 3
    echo -n "$v $i var: "
    MARLSAT_LIB=$(readlink -f $lib) timeout -k 10 120 python -u profiles/dual_bench.py 560000 10 128 1 2>/dev/null | grep "wgrad planes" || exit 3
  done
done 2>&1 | tee gpurun_out/r05v_wgrad_dlt.log
for p in 0 1; do
  MARLSAT_PLANES=$p timeout -k 10 420 python bench.py --steps 20 --warmup 5 --cpu-budget 0 --env-legs "" \
      --mappo uf100-430:4096:8 > gpurun_out/r05v_mappo_planes$p.json 2> gpurun_out/r05v_mappo_planes$p.err || exit 4
  echo "planes=$p: $(grep -o '"s_min_med_max": \[[^]]*\]' gpurun_out/r05v_mappo_planes$p.json)"
  cp gpurun_out/bench_mappo_uf100-430_n1_rank0.json gpurun_out/r05v_mappo_planes${p}_kernels.json
done
