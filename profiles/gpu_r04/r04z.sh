#!/bin/bash
# round 4, call z: the MAPPO headline leg's kernel trace slice on the final tree (384-row data-gradient blocks)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 700 bash profiles/collect_mappo.sh r04z || exit $?
echo "mappo trace rc 0"
