#!/bin/bash
# round 6, call e: env tests on the step kernel with its first round trip kept whole (branch-free prefetch, the
# queue entry in the action load, step / unsat with problem_idx), then config 2 with / without the reset queue
# (alternated) and the default env legs
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py tests/test_capi.py tests/test_single_env_gpu.py -m gpu -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06e_env_tests.log 2>&1
rc=$?
echo "env tests rc $rc"; tail -3 gpurun_out/r06e_env_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  for q in 1 0; do
    MARLSAT_RESET_QUEUE=$q timeout -k 10 120 python bench.py --cpu-budget 0 --mappo= --env-legs= --workload uf50-218 \
        --envs 1024 --steps 2000 --warmup 50 > gpurun_out/r06e_uf50_q${q}_$i.json 2> gpurun_out/r06e_uf50_q${q}_$i.err \
        || { echo "bench failed"; tail -5 gpurun_out/r06e_uf50_q${q}_$i.err; exit 1; }
    python - gpurun_out/r06e_uf50_q${q}_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sp = d["stamp_phases"]
print(sys.argv[1].split("/")[-1], "kernel_us %.3f" % (d["roofline"]["kernel_ms"] * 1e3), "frac %.3f" % d["roofline"]["frac"],
      "span", sp["launch_span_us"], "wg_med", sp["workgroup_median_us"], "wg_max", sp["workgroup_max_us"],
      "reset_wg", sp["reset_workgroup_median_us"], "sclk", d["sclk_mhz"], sp["phase_median_us"])
PY
  done
done
timeout -k 10 300 python bench.py --cpu-budget 0 --mappo= > gpurun_out/r06e_bench_env.json 2> gpurun_out/r06e_bench_env.err
rc=$?
echo "bench rc $rc"; python -c "
import json;d=json.loads(open('gpurun_out/r06e_bench_env.json').read().strip().splitlines()[-1])
print('headline', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['sclk_mhz']); print(d['env_other_legs'])"
exit $rc
