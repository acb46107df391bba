#!/bin/bash
# round 6, call j: GRU forward (h2s) -- epilogue / prologue ablations (e1 transcendentals replaced by one VALU op,
# e2 no gate math, e3 no h' flush, e4 no prologue wait; timing only, wrong results) and two DMA-spread forms that
# must be bitwise equal to the product (d1: weight pairs and activations at blocks +0/+3/+6/+9, d2: +0/+2/+4/+6)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=$PWD/marl-sat_amd/marlsat/lib
O=gpurun_out/r06j_gru_epi.log
for lib in libmarlsat libmarlsat_gepi_d1 libmarlsat_gepi_d2 libmarlsat_gepi_e1 libmarlsat_gepi_e2 libmarlsat_gepi_e3 libmarlsat_gepi_e4 libmarlsat libmarlsat_gepi_d1 libmarlsat_gepi_d2; do
  echo "== $lib" >> $O
  GRU_KERNELS=h2r GRU_CHECKSUM=1 MARLSAT_LIB=$L/$lib.so timeout -k 10 120 python profiles/gru_r_bench.py >> $O 2>&1 || { echo "$lib failed"; tail -3 $O; exit 1; }
done
python - <<'PY'
import json
cur = None
for line in open("gpurun_out/r06j_gru_epi.log"):
    if line.startswith("=="):
        cur = line.split()[1]; continue
    if line.startswith("{"):
        d = json.loads(line)
        print(f"{cur:22s} {d['cell']:6s} tape {str(d['tape']):5s} {d['ms']:.4f} ms  out {d.get('out_bits')} g4 {d.get('g4_bits')}")
PY
