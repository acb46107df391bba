"""Summarise profiles/pmc_gru_traffic.sh: per launch of gru_ln_fused_fwd_h2s_kernel (clause 1.4 M rows and
var 560 K rows, tape on) the PMC HBM bytes (FETCH_SIZE x 2: gfx950 tallies half of 16-B-per-lane reads,
MI355X_MICROARCH.md HBM section; WRITE_SIZE exact for the 16-B and dword stores) against the algorithmic
bytes (x, h in; h', 4H tape out) and the kernel-trace duration."""
import csv, glob, json, statistics, sys

out = sys.argv[1]
K = "gru_ln_fused_fwd_h2s_kernel"
H = 128
cells = {"clause": (1400000, 2 * H + 4), "var": (560000, H + 8)}  # rows, Kx (gru_r_bench.py shapes)


def rows_of(pattern, counter=None):
    f = glob.glob(f"{out}/{pattern}", recursive=True)[0]
    r = [x for x in csv.DictReader(open(f)) if K in x["Kernel_Name"]]
    return [x for x in r if counter is None or x["Counter_Name"] == counter]


trace = rows_of("trace/**/*kernel_trace.csv")
fetch = rows_of("fetch/**/*counter_collection.csv", "FETCH_SIZE")
write = rows_of("write/**/*counter_collection.csv", "WRITE_SIZE")
grid = lambda r: int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
res = {}
for cell, (R, Kx) in cells.items():
    tiles = (R + 127) // 128
    sel = lambda rs: [x for x in rs if grid(x) == tiles * 512]
    dur = statistics.mean((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) for x in sel(trace))
    f = statistics.mean(float(x["Counter_Value"]) for x in sel(fetch)) * 1024 * 2
    w = statistics.mean(float(x["Counter_Value"]) for x in sel(write)) * 1024
    alg = 4.0 * R * (Kx + 2 * H + 4 * H)
    res[cell] = {"rows": R, "launch_us": dur / 1e3, "pmc_read_bytes": f, "pmc_write_bytes": w,
                 "pmc_bytes": f + w, "algorithmic_bytes": alg, "pmc_over_algorithmic": (f + w) / alg,
                 "algorithmic_GBps": alg / dur, "pmc_GBps": (f + w) / dur}
print(json.dumps(res, indent=1))
