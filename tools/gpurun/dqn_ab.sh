#!/bin/bash
# Config-5 DQN timings (act + update at 2^21 boards, 64K minibatch) across library builds, alternated
# over two rounds, after the DQN GPU tests on the first library.
# usage: bash tools/gpurun/dqn_ab.sh OUTDIR lib.so [lib.so ...]   (libraries from tools/build_variant.sh)
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
R48_LIB=$1 timeout -k 10 600 python -u -m pytest tests/test_dqn_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for L in "$@"; do
R48_LIB=$L timeout -k 10 300 python -u -c "
import os, torch, bench
r = bench.dqn_config5(torch.device('cuda', 0), 0x20485EED, 1 << 21)
print(os.path.basename(os.environ['R48_LIB']), 'act %.2f ms update %.2f ms' % (r['act_ms'], r['update_ms']), flush=True)
" 2>&1 | grep -v amdgpu.ids >> $O/timing.txt || exit 1
done; done
cat $O/timing.txt
