#!/bin/bash
# A/B of the dual gradient kernels (profiles/dual_bench.py): ab/base.so, current build, and optional
# further libraries, alternating on one box.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
LIBS=("$R/ab/base.so" "" "$@")
for round in 1 2; do
  for lib in "${LIBS[@]}"; do
    echo "== $(basename ${lib:-current})"
    env ${lib:+MARLSAT_LIB=$lib} timeout -k 10 120 python $R/profiles/dual_bench.py 1316000 10
  done
done
