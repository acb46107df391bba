#!/bin/bash
# round 6, call c: config 2 (uf50 x 1024) with and without the reset queue, alternated on one box; then the
# train-cycle margins of the default path and of each fp16x2 kernel family in bf16x3, over four seeds each
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for i in 1 2 3; do
  for q in 1 0; do
    MARLSAT_RESET_QUEUE=$q timeout -k 10 120 python bench.py --cpu-budget 0 --mappo= --env-legs= --workload uf50-218 \
        --envs 1024 --steps 2000 --warmup 50 > gpurun_out/r06c_uf50_q${q}_$i.json 2> gpurun_out/r06c_uf50_q${q}_$i.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "bench q$q rc $rc"; tail -5 gpurun_out/r06c_uf50_q${q}_$i.err; exit $rc; fi
    python - gpurun_out/r06c_uf50_q${q}_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sp = d["stamp_phases"]
print(sys.argv[1].split("/")[-1], "kernel_us %.3f" % (d["roofline"]["kernel_ms"] * 1e3), "frac %.3f" % d["roofline"]["frac"],
      "span", sp["launch_span_us"], "wg_med", sp["workgroup_median_us"], "wg_max", sp["workgroup_max_us"],
      "reset_wg", sp["reset_workgroup_median_us"], "sclk", d["sclk_mhz"], sp["phase_median_us"])
PY
  done
done
timeout -k 10 900 python -u profiles/parity_switch_probe.py --seeds 4,5,6,7 default gru dgrad bf16x3 \
    > gpurun_out/r06c_switch_probe.log 2>&1
rc=$?
echo "probe rc $rc"; grep -E "^=== .*(passed|FAILED)|margins .* step" gpurun_out/r06c_switch_probe.log | grep -o "^=== .*\|margins [^ ]* .*step [0-9]\|grad worst ratio [0-9.e-]* ([^)]*)" | paste - - - | head -60
exit $rc
