#!/bin/bash
# round 5, call l: where the weight gradient's cycles go, both forms (fp32 rows: wgrad_w_dual_kernel<2>, planes:
# wgrad_w_dual_pl_kernel) on the clause shape -- unit counters (pmc_units.sh) and PMC HBM fetch per launch
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export DUAL_ONLY=wgrad
timeout -k 10 500 bash profiles/pmc_units.sh wgrad profiles/dual_bench.py 1316000 3 256 1 > gpurun_out/r05l_units_wgrad.json 2> gpurun_out/r05l_units_wgrad.err || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05l_fetch -o fetch -- python3 $GRAFT_REPO_ROOT/profiles/dual_bench.py 1316000 3 256 1 > $GRAFT_REPO_ROOT/gpurun_out/r05l_fetch.log 2>&1 || exit 4
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05l_trace -o trace -- python3 $GRAFT_REPO_ROOT/profiles/dual_bench.py 1316000 3 256 1 > $GRAFT_REPO_ROOT/gpurun_out/r05l_trace.log 2>&1 || exit 5
cd $GRAFT_REPO_ROOT && python3 - <<'PY'
import csv, glob, collections, json
acc = collections.defaultdict(list)
for f in glob.glob("gpurun_out/r05l_fetch/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"].split("(")[0][-40:]].append(float(r["Counter_Value"]) * 1024 * 2)
print(json.dumps({k: sum(v) / len(v) for k, v in acc.items() if "wgrad" in k}, indent=1))
PY
python3 - <<'PY'
import csv, glob, json
for f in glob.glob("gpurun_out/r05l_trace/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wgrad" in r["Name"]:
            print(r["Name"][:60], r["Calls"], r["AverageNs"])
PY
cat gpurun_out/r05l_units_wgrad.json | python3 -c "import json,sys; d=json.load(sys.stdin); [print(k, {c: round(v,3) for c,v in x.items() if 'frac' in c or c in ('SQ_INSTS_VALU','SQ_INSTS_MFMA','SQ_INSTS_LDS','SQ_WAVE_CYCLES','SQ_BUSY_CYCLES','SQ_VALU_MFMA_BUSY_CYCLES','SQ_LDS_BANK_CONFLICT','GRBM_GUI_ACTIVE')}) for k,x in d.items()]"
