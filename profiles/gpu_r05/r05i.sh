#!/bin/bash
# round 5, call i: unit counters (profiles/pmc_units.sh) of the GRU forward in both forms (h2s: 128 x 128 tiles,
# h2u: 256-row tiles in two unit halves), clause and var shapes without the tape, fp16x2 kernel only; then the
# env tests on the reverted env kernel (the reset prefetch measured no gain)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export GRU_KERNELS=h2r GRU_TAPE=False GRU_REPS=5
for f in h2s h2u; do
  MARLSAT_GRU_FORM=$f timeout -k 10 400 bash profiles/pmc_units.sh gru_$f profiles/gru_r_bench.py > gpurun_out/r05i_units_$f.json 2> gpurun_out/r05i_units_$f.err || exit 3
  echo "$f done"
done
T="python -u -m pytest -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T -q tests/test_env_gpu.py > gpurun_out/r05i_env_tests.log 2>&1
rc=$?; echo "env tests rc $rc"; tail -2 gpurun_out/r05i_env_tests.log
exit $rc
