#!/bin/bash
# Where a kernel's cycles go, by unit: SQ wave states and instruction mix, texture address / data units
# (TA / TD busy and stall cycles), L1 (TCP) stalls, GPU-active cycles -- one rocprofv3 --pmc pass per
# group, within each block's slot limit.  usage: bash profiles/pmc_units.sh <tag> <script.py> [args...]
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
SCRIPT=$(readlink -f "$1"); shift
OUT=$R/gpurun_out/pmcu_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE" \
         "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o p$i -- python3 $SCRIPT "$@" > $OUT/p$i.log 2>&1 || echo "pass $i failed"
done
python3 - <<PY
import csv, glob, collections, json
acc = collections.defaultdict(list)
for f in sorted(glob.glob("$OUT/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if "msat::" in r["Kernel_Name"]:
            acc[(r["Kernel_Name"].split("(")[0][-50:], r["Counter_Name"])].append(float(r["Counter_Value"]))
out = {}
for (k, c), v in sorted(acc.items()):
    out.setdefault(k, {})[c] = sum(v) / len(v)
for k, d in out.items():
    wc = d.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if c in d:
                d[c + "_frac"] = d[c] / wc
    ga = d.get("GRBM_GUI_ACTIVE")
    if ga:
        for c in ("TA_TA_BUSY_sum", "TD_TD_BUSY_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TCP_TCP_TA_DATA_STALL_CYCLES_sum",
                  "TCP_PENDING_STALL_CYCLES_sum", "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"):
            if c in d:
                d[c + "_per_unit_frac"] = d[c] / ga / 256.0  # per CU-instance, vs the GPU-active cycles
print(json.dumps(out, indent=1))
PY
