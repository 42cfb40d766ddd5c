#!/bin/bash
# Config-3-size A3C timings (2^20 boards x 100 steps) of the CNN (bf16) and the reference MLP (fp32)
# in both loss modes, after the A3C GPU tests of the MLP and the rollout megakernels.
set -o pipefail
O=gpurun_out/${1:-a3c_timings}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_a3c_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "mlp or rollout" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -c "
import json, torch, bench
d = torch.device('cuda', 0)
for net, bf16, mode, feat in (('mlp', False, 'reference', 'values'), ('mlp', False, 'textbook', 'exponents'),
                              ('cnn', True, 'textbook', 'exponents'), ('cnn', True, 'reference', 'values')):
    r = bench.a3c_config3(d, 0x20485EED, 1 << 20, mode=mode, features=feat, net=net, bf16=bf16)
    print(json.dumps(r), flush=True)
" > $O/a3c.json 2> $O/a3c.err; rc=$?; python -c "
import json
for l in open('$O/a3c.json'):
    r = json.loads(l); print(r['net'][:3], r['mode'], 'rollout %.2f ms update %.2f ms train %.2f G/s' % (r['rollout_ms'], r['update_ms'], r['train_env_steps_per_s'] / 1e9))"; tail -3 $O/a3c.err; exit $rc
