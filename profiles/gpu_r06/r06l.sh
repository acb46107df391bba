#!/bin/bash
# round 6, call l: dump the inputs of the headline-shape teacher-forced train cycle (uf100 A = 10 L = 16, seed 4)
# on the three precision paths (device parameters and gradients of every Adam step, the minibatch) for the CPU
# study of fp32's own noise at the worst elements (profiles/parity_orderings.py)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
MARLSAT_PARITY_DUMP=gpurun_out/pdump timeout -k 10 500 python -u -m pytest tests/test_mappo_gpu.py \
    -k "every_adam_step and 100-430" -s -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r06l_dump.log 2>&1
rc=$?
echo "rc $rc"; grep "^margins" gpurun_out/r06l_dump.log | sed 's/loss err.*grad worst/grad worst/'; ls -la gpurun_out/pdump
exit $rc
