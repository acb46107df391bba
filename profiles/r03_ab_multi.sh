#!/bin/bash
# A/B of several library builds on one box: for N rounds, run the given python script once per library
# (the in-tree build first, then each ab/libmarlsat_*.so named in LIBS).  usage: LIBS="s1 s2" r03_ab_multi.sh N script.py [args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
N=$1; shift
for i in $(seq 1 $N); do
  for v in base $LIBS; do
    if [ "$v" = base ]; then lib=marl-sat_amd/marlsat/lib/libmarlsat.so; else lib=ab/libmarlsat_$v.so; fi
    echo "== round $i lib $v"
    MARLSAT_LIB=$PWD/$lib timeout -k 10 300 python3 "$@" || exit 1
  done
done
