#!/bin/bash
# round 6, call fh: GRU forward writing h' straight from the registers (16 lanes x 4 B per row segment, as the tape) instead of an LDS stage and float4 rows
# (libmarlsat_ghd.so) vs the product, alternated three times, checksums (outputs and tapes must be bitwise equal)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=$PWD/marl-sat_amd/marlsat/lib
O=gpurun_out/r06fh_gru_hdirect.log
for i in 1 2 3; do
  for lib in libmarlsat libmarlsat_ghd; do
    echo "== $lib $i" >> $O
    GRU_KERNELS=h2r GRU_CHECKSUM=1 MARLSAT_LIB=$L/$lib.so timeout -k 10 120 python profiles/gru_r_bench.py >> $O 2>&1 || { echo "$lib failed"; tail -3 $O; exit 1; }
  done
done
python - <<'PY'
import json, collections
cur=None; res=collections.defaultdict(list); bits={}
for line in open("gpurun_out/r06fh_gru_hdirect.log"):
    if line.startswith("=="): cur=line.split()[1]; continue
    if line.startswith("{"):
        d=json.loads(line); k=(cur,d['cell'],d['tape']); res[k].append(d['ms'])
        bits.setdefault((d['cell'],d['tape']),set()).add((d.get('out_bits'),d.get('g4_bits')))
for k,v in sorted(res.items()): print(k, ' '.join('%.4f'%x for x in v))
print('bitwise equal across builds:', all(len(s)==1 for s in bits.values()))
PY
