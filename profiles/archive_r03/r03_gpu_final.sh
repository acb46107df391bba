#!/bin/bash
# full GPU suite + smoke + default bench on the current tree (tag as $1)
set -o pipefail
T=${1:-r03q}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 700 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python3 -c "
import json
l=[x for x in open('gpurun_out/${T}_bench.json') if x.startswith('{')][-1]; d=json.loads(l)
print('env', d['value'], d['roofline']['frac'], 'line chars', len(l))
for g in d['mappo_other_legs']+[d['mappo']]: print(g['config']['workload'], g['s_per_update'], g['roofline']['kernel_ms'], g['roofline']['frac'], g['params_check'])
"
