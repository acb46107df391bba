#!/bin/bash
# A/B of two library builds on one box: alternate MARLSAT_LIB between ab/libmarlsat_base.so and the in-tree
# build, N rounds, running the given python script (args after --).  usage: r03_ab.sh N script.py [args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
N=$1; shift
for i in $(seq 1 $N); do
  for lib in ab/libmarlsat_base.so marl-sat_amd/marlsat/lib/libmarlsat.so; do
    echo "== round $i lib $lib"
    MARLSAT_LIB=$PWD/$lib timeout -k 10 300 python3 "$@" || exit 1
  done
done
