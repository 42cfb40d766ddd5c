#!/bin/bash
# MLP update: gradient diagnostic across tiles-per-wave, its GPU tests, the learning experiment and
# tests, then the A3C timings (CNN + reference MLP).
set -o pipefail
O=gpurun_out/r04_mlp; mkdir -p $O gpurun_out/r04_learn
timeout -k 10 300 python -u tools/exp_mlp_grad_debug.py > $O/grad_debug.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/grad_debug.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_a3c_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "mlp or rollout" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/exp_learning.py gpurun_out/r04_learn/learning.json --a3c-updates 2000 --dqn-steps 3000 > gpurun_out/r04_learn/learning.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r04_learn/learning.log | tail -15; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -c "
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
