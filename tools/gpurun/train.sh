#!/bin/bash
# GPU job: fused A3C update (k_cnn_train) parity tests, timing and kernel trace.
# usage (from the repo root, through gpurun): bash tools/gpurun/train.sh [out dir]
set -o pipefail
O=${1:-gpurun_out/train}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_a3c_gpu.py \
    -k "update or trainer" > $O/pytest.txt 2>&1 && tail -3 $O/pytest.txt \
&& timeout -k 10 300 python -u tools/exp_train.py 16777216 rein48_amd/lib/librein48.so rein48_amd/lib/librein48.so > $O/train.txt 2>&1 \
&& cat $O/train.txt \
&& cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o train --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/tools/prof_train.py 16777216 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 \
&& cd $GRAFT_REPO_ROOT && find $O/prof -name "*stats*" | head
