#!/bin/bash
# Round-4 config-5 session: the DQN GPU tests (BN fold bit-identity, steady-state convs, train step),
# the fold A/B, then the config-5 bench extra.
set -o pipefail
O=gpurun_out/r04_dqn; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_dqn_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/exp_bnfold.py > $O/bnfold.txt 2>&1; rc=$?; cat $O/bnfold.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -c "
import json, torch, bench
r = bench.dqn_config5(torch.device('cuda', 0), 0x20485EED, 1 << 21)
print(json.dumps(r), flush=True)
" > $O/dqn.json 2> $O/dqn.err; rc=$?; cat $O/dqn.json; tail -2 $O/dqn.err; exit $rc
