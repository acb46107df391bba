#!/bin/bash
# round 4, call i: the small-network parity test with the elementwise fp32-yardstick bar added, and the
# untethered train-cycle replay's measured loss / update errors (printed)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gnn_gpu.py tests/test_mappo_gpu.py -q -s -k "forward_backward_match_oracle or matches_oracle_replay" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04i_parity.log 2>&1
rc=$?
echo "rc $rc"; grep -E "^small|^replay|passed|failed|Error" gpurun_out/r04i_parity.log | head -60
