#!/bin/bash
# round 6, call o: final tree (GRU activations pre-scaled) -- the full GPU suite, smoke(), and the headline-shape
# train cycle's margins over four seeds on the default path (profiles/parity_switch_probe.py)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r06o_gpu_tests.log 2>&1
rc=$?
echo "suite rc $rc"; tail -3 gpurun_out/r06o_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06o_smoke.log 2>&1
rc=$?
echo "smoke rc $rc"; tail -1 gpurun_out/r06o_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u profiles/parity_switch_probe.py --seeds 4,5,6,7 default > gpurun_out/r06o_seeds.log 2>&1
rc=$?
echo "seeds rc $rc"; grep "^margins\|^===" gpurun_out/r06o_seeds.log | grep -v "rollout" | sed 's/loss err.*grad worst/grad worst/'
exit $rc
