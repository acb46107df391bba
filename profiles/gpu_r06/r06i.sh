#!/bin/bash
# round 6, call i: GRU forward (h2s) ablations -- what bounds a k step: no weight DMA after step 1 (1), no
# activation DMA (2), neither (3), no step-end vmcnt wait (4), none of the three (7), no MFMAs (8), no step-end
# barrier (16); wrong results, timing only (profiles/gru_r_bench.py, clause / var shapes, tape on and off)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=$PWD/marl-sat_amd/marlsat/lib
for lib in libmarlsat libmarlsat_gabl1 libmarlsat_gabl2 libmarlsat_gabl3 libmarlsat_gabl4 libmarlsat_gabl7 libmarlsat_gabl8 libmarlsat_gabl16 libmarlsat; do
  echo "== $lib" >> gpurun_out/r06i_gru_ablate.log
  MARLSAT_LIB=$L/$lib.so timeout -k 10 120 python profiles/gru_r_bench.py >> gpurun_out/r06i_gru_ablate.log 2>&1 || { echo "$lib failed"; tail -3 gpurun_out/r06i_gru_ablate.log; exit 1; }
done
python - <<'PY'
import json
cur = None
for line in open("gpurun_out/r06i_gru_ablate.log"):
    if line.startswith("=="):
        cur = line.split()[1]; continue
    if line.startswith("{"):
        d = json.loads(line)
        if d["kernel"] == "h2r":
            print(f"{cur:20s} {d['cell']:6s} tape {str(d['tape']):5s} {d['ms']:.4f} ms")
PY
