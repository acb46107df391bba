#!/bin/bash
# Gathers on the uf100 training graph shape (profiles/gather_xcd.py) with an exploration build (ab/gx.so:
# MARLSAT_GATHER_XCD = XCD-contiguous row walk, MARLSAT_GATHER_GRID = grid cap): timing sweep, then
# FETCH_SIZE per variant (L2 fabric reads; gfx950 reports half of 16-B-per-lane reads).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/gather_walk
mkdir -p $OUT
for rep in 1 2; do
  for x in 0 1; do
    for g in 8192 2048 1024; do
      echo "== xcd=$x grid=$g"
      MARLSAT_LIB=$R/ab/gx.so MARLSAT_GATHER_XCD=$x MARLSAT_GATHER_GRID=$g timeout -k 10 120 python $R/profiles/gather_xcd.py 820 10
    done
  done
done > $OUT/time.log 2>&1
cd /tmp && export TMPDIR=/tmp
for v in "0 8192" "1 8192" "1 2048"; do
  set -- $v
  MARLSAT_LIB=$R/ab/gx.so MARLSAT_GATHER_XCD=$1 MARLSAT_GATHER_GRID=$2 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_$1_$2 -o fetch -- python3 $R/profiles/gather_xcd.py 820 3 > $OUT/fetch_$1_$2.log 2>&1
done
echo done
