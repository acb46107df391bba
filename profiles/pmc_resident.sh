#!/bin/bash
# PMC of the dual data gradient, per-tile (MARLSAT_DGRAD_RESIDENT=0) vs resident-weight kernel: HBM fetch
# (FETCH_SIZE, gfx950 wide-read correction x2) and L2 hit rate (TCC_HIT_sum / TCC_MISS_sum), clause shape.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_res
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for r in 0 3; do
  MARLSAT_DGRAD_RESIDENT=$r DUAL_ONLY=dgrad timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/f$r -o f -- python3 $R/profiles/dual_bench.py 1316000 3 256 > $OUT/f$r.log 2>&1
  MARLSAT_DGRAD_RESIDENT=$r DUAL_ONLY=dgrad timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/h$r -o h -- python3 $R/profiles/dual_bench.py 1316000 3 256 > $OUT/h$r.log 2>&1
  MARLSAT_DGRAD_RESIDENT=$r DUAL_ONLY=dgrad timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/w$r -o w -- python3 $R/profiles/dual_bench.py 1316000 3 256 > $OUT/w$r.log 2>&1
done
python3 - <<PY
import csv, glob, collections, json
acc = collections.defaultdict(list)
for r in ("0", "3"):
    for f in glob.glob("$OUT/[fhw]" + r + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0][-44:]
            if "dual" in k:
                acc[(r, k, row["Counter_Name"])].append(float(row["Counter_Value"]))
out = {}
for (r, k, c), v in sorted(acc.items()):
    x = sum(v) / len(v)
    if c in ("FETCH_SIZE", "WRITE_SIZE"):
        x *= 1024 * (2 if c == "FETCH_SIZE" else 1)
    out.setdefault(r + " " + k, {})[c] = x
for k, d in out.items():
    if "TCC_HIT_sum" in d:
        d["l2_hit"] = d["TCC_HIT_sum"] / max(1.0, d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
print(json.dumps(out, indent=1))
PY
