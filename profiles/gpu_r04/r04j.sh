#!/bin/bash
# round 4, call j: the untethered train-cycle replay at the tightened bars
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mappo_gpu.py -q -s -k "matches_oracle_replay" --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r04j_replay.log 2>&1
rc=$?
echo "rc $rc"; grep -E "replay mode|passed|failed|Error" gpurun_out/r04j_replay.log | head
