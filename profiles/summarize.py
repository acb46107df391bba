"""Summarise a profiles/collect.sh run (gpurun_out/prof) into committed files under profiles/:
  <tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied as is)
  <tag>_pmc.json           per-launch FETCH_SIZE / WRITE_SIZE of the env step kernel, and the HBM
                           bytes per launch bench.py reports as roofline.traffic.

Counter handling (MI355X_MICROARCH.md §HBM): FETCH_SIZE/WRITE_SIZE are in KiB; WRITE_SIZE is exact
for 16 B-per-lane streaming stores (the obs pass, >97 % of this kernel's traffic); FETCH_SIZE reads
1/2 of WIDE (16 B/lane) coalesced reads, but this kernel's reads are 1-8 B per lane (pool words,
table words, assignment bytes), an uncalibrated width, so the read side is reported raw."""
import csv, json, os, shutil, statistics, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
workload = sys.argv[2] if len(sys.argv) > 2 else "uf200-860/B4096/int32"
prof = os.path.join(ROOT, "gpurun_out", "prof")
KERNEL = sys.argv[3] if len(sys.argv) > 3 else "env_kernel<2, int, 512>"  # the uf200 x 4096 instantiation

def counter(path, name):
    rows = [r for r in csv.DictReader(open(path)) if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == name]
    return [float(r["Counter_Value"]) for r in rows], rows

stats_src = os.path.join(prof, "trace", "trace_kernel_stats.csv")
shutil.copy(stats_src, os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
avg_ns = None
for r in csv.DictReader(open(stats_src)):
    if KERNEL in r["Name"]:
        avg_ns = float(r["AverageNs"])
fetch, frows = counter(os.path.join(prof, "fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
write, _ = counter(os.path.join(prof, "write", "write_counter_collection.csv"), "WRITE_SIZE")
f_kib, w_kib = statistics.mean(fetch), statistics.mean(write)
out = {
    "workload": workload,
    "kernel": frows[0]["Kernel_Name"],
    "launches_profiled": len(write),
    "avg_duration_ns_kernel_trace": avg_ns,
    "fetch_size_kib_per_launch": f_kib,
    "write_size_kib_per_launch": w_kib,
    "hbm_bytes_per_launch": (f_kib + w_kib) * 1024,
    "vgpr": int(frows[0]["VGPR_Count"]), "sgpr": int(frows[0]["SGPR_Count"]),
    "lds_bytes": int(frows[0]["LDS_Block_Size"]),
    "note": "FETCH raw (narrow reads, uncalibrated width); WRITE exact for the 16 B obs stores",
}
json.dump(out, open(os.path.join(ROOT, "profiles", f"{tag}_pmc.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
