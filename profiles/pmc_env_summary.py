"""Per-launch HBM bytes of the env kernels from a profiles/collect.sh run (rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE
passes, each its own run): per kernel instantiation, the mean FETCH_SIZE / WRITE_SIZE (KiB) per launch, FETCH x 2
per the gfx950 correction (MI355X_MICROARCH.md, HBM section: FETCH_SIZE reports half of a wide streaming read) and
their sum.  The headline env leg's record also carries "workload" (bench.py load_pmc_traffic reads it).

    python profiles/pmc_env_summary.py gpurun_out/prof OUT.json [workload]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def counters(root, name):
    per = defaultdict(list)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != name:
                    continue
                k = row["Kernel_Name"]
                k = k[5:] if k.startswith("void ") else k
                per[k.split("(")[0].replace("msat::", "")].append(float(row["Counter_Value"]))
    return per


if __name__ == "__main__":
    root, out = sys.argv[1], sys.argv[2]
    workload = sys.argv[3] if len(sys.argv) > 3 else "uf200-860/B4096/int32"
    fetch, write = counters(os.path.join(root, "fetch"), "FETCH_SIZE"), counters(os.path.join(root, "write"), "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) & set(write)):
        if not k.startswith("env_"):
            continue
        f, w = sum(fetch[k]) / len(fetch[k]), sum(write[k]) / len(write[k])
        res[k] = {"FETCH_SIZE": {"launches": len(fetch[k]), "mean_raw_KiB": f},
                  "WRITE_SIZE": {"launches": len(write[k]), "mean_raw_KiB": w},
                  "per_launch_bytes": {"fetch_x2_gfx950": 2 * f * 1024, "write": w * 1024, "total": (2 * f + w) * 1024}}
    head = "env_kernel<2, int, 512>"
    if head in res:
        res["headline"] = dict(res[head], kernel=head)
        res["workload"] = workload
        res["hbm_bytes_per_launch"] = res[head]["per_launch_bytes"]["total"]
    res["_note"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (profiles/collect.sh) of bench.py's env legs; FETCH x 2 "
                    "per the gfx950 correction; per kernel instantiation (the headline uf200 x 4096 leg is "
                    "env_kernel<2, int, 512>)")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v.get("per_launch_bytes", v) if isinstance(v, dict) else v for k, v in res.items()}, indent=0)[:2000])
