#!/bin/bash
# var gather, two rows per wave (MSAT_VG_HW=1) vs one (0): network + gather tests, then the 4-gather step
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gnn_gpu.py > gpurun_out/r03w_vg_tests.log 2>&1 || { tail -30 gpurun_out/r03w_vg_tests.log; exit 1; }
tail -1 gpurun_out/r03w_vg_tests.log
for i in 1 2 3; do for hw in 0 1; do
echo "== hw $hw" >> gpurun_out/r03w_vg_ab.log
MSAT_VG_HW=$hw timeout -k 10 120 python -u profiles/gather_xcd.py >> gpurun_out/r03w_vg_ab.log 2>&1 || exit 1
done; done
grep -v amdgpu.ids gpurun_out/r03w_vg_ab.log
