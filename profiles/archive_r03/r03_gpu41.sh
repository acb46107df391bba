#!/bin/bash
# GRU forward HBM traffic (PMC) with the padding DMA pointed at one line, against the previous build
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
MARLSAT_LIB=$PWD/ab/libmarlsat_base.so bash profiles/pmc_gru_traffic.sh > gpurun_out/r03j_pmc_base.log 2>&1 || { tail -20 gpurun_out/r03j_pmc_base.log; exit 1; }
cp gpurun_out/pmc_gru_traffic.json gpurun_out/r03j_pmc_gru_base.json
bash profiles/pmc_gru_traffic.sh > gpurun_out/r03j_pmc_new.log 2>&1 || { tail -20 gpurun_out/r03j_pmc_new.log; exit 1; }
cp gpurun_out/pmc_gru_traffic.json gpurun_out/r03j_pmc_gru_new.json
rm -rf gpurun_out/pmc_gru_traffic
cat gpurun_out/r03j_pmc_gru_base.json gpurun_out/r03j_pmc_gru_new.json
