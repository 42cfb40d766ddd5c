#!/bin/bash
# A/B of the reference-MLP A3C path across library builds: the MLP GPU tests on the first library, then
# config-3 train-step timings (bench.a3c_config3, net='mlp': reference loss on raw values, textbook on
# exponents) of every library, alternated over N rounds in separate processes.
# usage: N=4 bash tools/gpurun/mlp_rollout_ab.sh OUT lib.so [lib.so ...]
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
R48_LIB=$1 timeout -k 10 600 python -u -m pytest tests/test_a3c_gpu.py tests/test_checkpoint_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "mlp or MLP" > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in $(seq ${N:-2}); do for L in "$@"; do
R48_LIB=$L timeout -k 10 300 python -u -c "
import os, torch, bench
d = torch.device('cuda', 0)
for name, kw in (('mlp reference', dict(mode='reference', features='values', net='mlp', bf16=False)),
                 ('mlp textbook', dict(mode='textbook', features='exponents', net='mlp', bf16=False))):
    r = bench.a3c_config3(d, 0x20485EED, 1 << 20, **kw)
    print(os.path.basename(os.environ['R48_LIB']), name, 'rollout %.2f ms update %.2f ms' % (r['rollout_ms'], r['update_ms']), flush=True)
" 2>&1 | grep -v amdgpu.ids >> $O/timing.txt || exit 1
done; done
cat $O/timing.txt
