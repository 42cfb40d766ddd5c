#!/bin/bash
# GPU job (round 3): k_cnn_train tests + A/B + stamps, config-5 conv kernel tests and update
# timing with a kernel trace, env sync experiment.
set -o pipefail
O=gpurun_out/r03b; mkdir -p $O
export TMPDIR=/tmp
bash tools/gpurun/train_ab.sh build/lib_train_head.so \
&& timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dqn_gpu.py > $O/pytest_dqn.txt 2>&1; tail -3 $O/pytest_dqn.txt
timeout -k 10 200 python -u tools/prof_dqn.py > $O/dqn_update.txt 2>&1 && cat $O/dqn_update.txt \
&& cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_dqn -o dqn --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/tools/prof_dqn.py > $GRAFT_REPO_ROOT/$O/prof_dqn.log 2>&1; cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/exp_sync.py 20 > $O/sync.txt 2>&1 && cat $O/sync.txt \
&& timeout -k 10 120 python -u tools/exp_sync.py --spin 20 > $O/sync_spin.txt 2>&1 && cat $O/sync_spin.txt
