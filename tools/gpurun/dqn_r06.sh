#!/bin/bash
# Round-6 config-5 update work: DQN GPU tests on the current tree, then the update timing of the
# current tree vs an older tree (tools/gpurun/tree_ab.sh, one process per arm), then library variants
# of the current tree with an A/A control (one process per library, alternated).
# usage: bash tools/gpurun/dqn_r06.sh OUT OLD_DIR [lib.so ...]
set -o pipefail
NAME=$1; O=gpurun_out/$1; OLD=$2; shift 2; mkdir -p $O
export TMPDIR=/tmp
T="import os, torch, bench; r = bench.dqn_config5(torch.device('cuda', 0), 0x20485EED, 1 << 21); print(os.path.basename(os.environ.get('R48_LIB', 'tree')), 'act %.2f ms update %.2f ms' % (r['act_ms'], r['update_ms']), flush=True)"
timeout -k 10 600 python -u -m pytest tests/test_dqn_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
N=${N:-3} bash tools/gpurun/tree_ab.sh $NAME/tree $OLD "python -u -c \"$T\"" || exit 1
if [ $# -gt 0 ]; then
for i in 1 2 3; do for L in "$@"; do
R48_LIB=$L timeout -k 10 300 python -u -c "$T" 2>&1 | grep -v amdgpu.ids >> $O/libs.txt || exit 1
done; done
cat $O/libs.txt
fi
[ -z "$PROF" ] || bash tools/gpurun/dqn_prof.sh $O/prof
