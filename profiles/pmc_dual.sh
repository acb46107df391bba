#!/bin/bash
# PMC HBM traffic of the dual data / weight gradients (profiles/dual_bench.py): FETCH_SIZE and WRITE_SIZE
# passes + kernel trace.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_dual
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/profiles/dual_bench.py 1316000 10 > $OUT/timing.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/profiles/dual_bench.py 1316000 3 > $OUT/trace.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $R/profiles/dual_bench.py 1316000 3 > $OUT/fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $R/profiles/dual_bench.py 1316000 3 > $OUT/write.log 2>&1
python3 - <<PY
import csv, glob, collections, json
acc = collections.defaultdict(list)
for f in glob.glob("$OUT/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"].split("(")[0][-40:], r["Counter_Name"])].append(float(r["Counter_Value"]))
out = {}
for (k, c), v in sorted(acc.items()):
    if "msat" in k or "wgrad" in k or "gemm" in k:
        out.setdefault(k, {})[c] = sum(v) / len(v) * 1024 * (2 if c == "FETCH_SIZE" else 1)
print(json.dumps(out, indent=1))
PY
cat $OUT/timing.txt
