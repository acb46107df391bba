#!/bin/bash
# round 5, call d: the headline-shape teacher-forced case (uf100 A10 m10 H128 L16) on each arithmetic path, with
# per-sample rollout value errors printed (device vs fp64 oracle, and the fp32 CPU oracle's own)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T="python -u -m pytest -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider -s -v"
rc=0
for P in fp16x2 bf16x3 fp32; do
  MARLSAT_PRECISION=$P timeout -k 10 300 $T tests/test_mappo_gpu.py -k "every_adam_step and 100-430" \
      > gpurun_out/r05d_uf100_$P.log 2>&1
  r=$?; echo "$P rc $r"; grep -E "rollout V|margins|worst ratio" gpurun_out/r05d_uf100_$P.log | head -8
  if [ $r -ne 0 ] && [ $r -ne 1 ]; then exit $r; fi
done
exit 0
