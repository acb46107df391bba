#!/bin/bash
# SQ counter passes over one python microbenchmark; prints per-kernel averages.
# usage: bash profiles/pmc_sq.sh <tag> <script.py> [args...]
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_SALU"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o p$i -- python3 "$@" > $OUT/p$i.log 2>&1
done
python3 - <<PY
import csv, glob, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob("$OUT/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if "msat::" in r["Kernel_Name"]:
            acc[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
ks = sorted({k for k, _ in acc})
for k in ks:
    d = {c: sum(v) / len(v) for (kk, c), v in acc.items() if kk == k}
    wc = d.get("SQ_WAVE_CYCLES", 1)
    waves = d.get("SQ_WAVES", 1)
    print(k, {c: round(v / wc, 3) if c.startswith("SQ_WAIT") or c == "SQ_ACTIVE_INST_ANY" else round(v / waves, 1)
              for c, v in sorted(d.items())})
PY
