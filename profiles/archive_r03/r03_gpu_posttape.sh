#!/bin/bash
# gate tape after activation: GRU / network / MAPPO oracle tests, then backward kernel and MAPPO-leg A/B
# against the previous build (ab/libmarlsat_base.so, pre-activation tape)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gru_fused_gpu.py tests/test_gnn_gpu.py tests/test_mappo_gpu.py tests/test_dist_learner_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03r_tests.log 2>&1 || { tail -40 gpurun_out/r03r_tests.log; exit 1; }
tail -1 gpurun_out/r03r_tests.log
LIBS="base" bash profiles/r03_ab_multi.sh 3 profiles/gru_bwd_only.py > gpurun_out/r03r_ab_bwd.log 2>&1 || { tail gpurun_out/r03r_ab_bwd.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03r_ab_bwd.log
for lib in base new base new; do
  if [ $lib = base ]; then L=$PWD/ab/libmarlsat_base.so; else L=$PWD/marl-sat_amd/marlsat/lib/libmarlsat.so; fi
  MARLSAT_LIB=$L timeout -k 10 400 python3 bench.py --cpu-budget 0 --steps 2 --warmup 1 --mappo uf100-430:4096:8 > gpurun_out/r03r_mappo_$lib.json 2>/dev/null || exit 1
  python3 -c "
import json
l=[x for x in open('gpurun_out/r03r_mappo_$lib.json') if x.startswith('{')][-1]; d=json.loads(l)['mappo']
print('$lib', d['s_per_update'], d['phase_ms'])
" | tee -a gpurun_out/r03r_ab_mappo.log
done
