#!/bin/bash
# round 6, call fc: the headline-shape train cycle's margins over four seeds on the bf16x3 and fp32 paths (the default
# path's are r06o_seeds.log), for the distribution of the worst ratio per path
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u profiles/parity_switch_probe.py --seeds 4,5,6,7 bf16x3 fp32 > gpurun_out/r06fc_seeds.log 2>&1
rc=$?
echo "seeds rc $rc"; grep "^margins\|FAILED" gpurun_out/r06fc_seeds.log | grep -v rollout | sed 's/loss err.*grad worst/grad worst/'
exit $rc
