#!/bin/bash
# MLP fused path after the 4-chain FMA split: its GPU tests and the config-3-size timings.
set -o pipefail
O=gpurun_out/r04_mlp2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_a3c_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "mlp" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -c "
import json, torch, bench
d = torch.device('cuda', 0)
for net, bf16, mode, feat in (('mlp', False, 'reference', 'values'), ('mlp', False, 'textbook', 'exponents')):
    r = bench.a3c_config3(d, 0x20485EED, 1 << 20, mode=mode, features=feat, net=net, bf16=bf16)
    print(json.dumps(r), flush=True)
" > $O/a3c.json 2> $O/a3c.err; rc=$?; python -c "
import json
for l in open('$O/a3c.json'):
    r = json.loads(l); print(r['net'][:3], r['mode'], 'rollout %.2f ms update %.2f ms train %.2f G/s' % (r['rollout_ms'], r['update_ms'], r['train_env_steps_per_s'] / 1e9))"; tail -3 $O/a3c.err; exit $rc
