#!/bin/bash
# HBM-side traffic of the four gathers on the uf100 training graph shape (profiles/gather_xcd.py):
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes (no trace domains).  FETCH_SIZE counts the
# L2's fabric reads (Infinity-Cache hits included); gfx950 reports half the bytes of 16-B-per-lane reads.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_gather
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $R/profiles/gather_xcd.py 820 3 > $OUT/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $R/profiles/gather_xcd.py 820 3 > $OUT/write.log 2>&1
echo done
