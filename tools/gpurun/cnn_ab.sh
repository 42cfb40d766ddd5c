#!/bin/bash
# The CNN A3C path (config-3 size, both loss modes) across library builds, alternated over two rounds,
# after the CNN rollout / update GPU tests on the first library.
# usage: bash tools/gpurun/cnn_ab.sh OUTDIR lib.so [lib.so ...]   (libraries from tools/build_variant.sh)
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
R48_LIB=$1 timeout -k 10 600 python -u -m pytest tests/test_a3c_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "rollout or fused_cnn or trainer_fused_update" > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in $(seq ${N:-2}); do for L in "$@"; do
R48_LIB=$L timeout -k 10 300 python -u -c "
import os, torch, bench
d = torch.device('cuda', 0)
for mode, feat in (('textbook', 'exponents'), ('reference', 'values')):
    r = bench.a3c_config3(d, 0x20485EED, 1 << 20, mode=mode, features=feat, net='cnn', bf16=True)
    print(os.path.basename(os.environ['R48_LIB']), mode, 'rollout %.2f ms update %.2f ms' % (r['rollout_ms'], r['update_ms']), flush=True)
" 2>&1 | grep -v amdgpu.ids >> $O/timing.txt || exit 1
done; done
cat $O/timing.txt
