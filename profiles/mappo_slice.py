"""Per-kernel durations of the bench's TIMED MAPPO cycle from a rocprofv3 kernel trace, to set beside
the bench's own HIP-event numbers (bench.py "mappo" -> "kernels").

The timed cycle (rollout, GAE, PPO epochs, metrics) is the last GPU work of a bench run with one
MAPPO leg and --cpu-budget 0, so its launches of a kernel are that kernel's LAST n launches in the
trace, n = the launch count the bench reports.  Writes a JSON summary (run on the GPU box):
    python3 profiles/mappo_slice.py <kernel_trace.csv> <bench stdout> <out.json>"""
import csv
import json
import sys

trace, bench_log, out = sys.argv[1:4]
line = next(l for l in open(bench_log) if l.startswith("{") and '"mappo"' in l)
bench = json.loads(line)["mappo"]
if "kernels" not in bench:  # compact leg (round 3): the per-kernel table is in its side file
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    det = bench["detail"]  # the side file; since round 4 its name only: gpurun_out/bench_<detail>.json
    bench = json.load(open(os.path.join(root, det if os.sep in det else os.path.join("gpurun_out", f"bench_{det}.json"))))
ROCPROF_NAMES = {  # bench label -> rocprof kernel names whose launches the bench's event pair brackets
    "gru_ln_fused_fwd_x3r_kernel (bf16x3)": ["gru_ln_fused_fwd_x3r_kernel"],
    "gru_ln_fused_fwd_h2r_kernel (fp16x2, + x3r fixup launch)": ["gru_ln_fused_fwd_h2r_kernel", "gru_ln_fused_fwd_x3r_kernel"],
    "gru_ln_fused_fwd_h2s_kernel (fp16x2, + x3r fixup launch)": ["gru_ln_fused_fwd_h2s_kernel", "gru_ln_fused_fwd_x3r_fix_kernel"],
    "gemm_x3r16_kernel (dgrad, bf16x3)": ["gemm_x3r16_kernel"],
    "wgrad_x3_kernel + reduce (bf16x3)": ["wgrad_x3_kernel", "wgrad_reduce4_kernel"],
    "wgrad_w_kernel<3> + reduce (bf16x3)": ["wgrad_w_kernel<3", "wgrad_reduce4_kernel"],
    "wgrad_w_kernel<2> + fixup + reduce (fp16x2)": ["wgrad_w_dual_kernel<2", "wgrad_w_dual_kernel<3",
                                                    "wgrad_reduce4_kernel"],
    "gemm_h2r16_kernel (dgrad, fp16x2)": ["gemm_h2r16_dual_kernel"],
    "gemm_h2r16_kernel (dgrad, fp16x2 planes)": ["gemm_h2r16_dual_kernel"],
    "wgrad_w_dual_pl_kernel + fixup + reduce (fp16x2 planes)": ["wgrad_w_dual_pl_kernel", "wgrad_w_dual_kernel<3",
                                                                 "wgrad_reduce4_kernel"],
}
launches = {}
for r in csv.DictReader(open(trace)):
    launches.setdefault(r["Kernel_Name"], []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
res = {"bench_config": bench["config"], "kernels": []}
for k in bench["kernels"]:
    names = ROCPROF_NAMES.get(k["kernel"])
    if not names:
        continue
    n, tot = k["launches"], 0.0
    for nm in names:
        rows = sorted(v for key, vals in launches.items() if nm in key for v in vals)
        last = rows[-n:]
        if last:
            tot += sum(e - s for s, e in last) / len(last) / 1e6
    res["kernels"].append({"kernel": k["kernel"], "launches": n, "bench_event_ms_avg": k["ms_avg"],
                           "rocprof_ms_avg_last_n": tot, "ratio": k["ms_avg"] / tot,
                           "bench_tflops_fp32_equiv": k["tflops_fp32_equiv"], "bench_frac": k["frac"]})
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
