#!/bin/bash
# Round-5 config-5 session: the DQN GPU tests (incl. the per-GPU-slice trainer test), a kernel trace
# and per-kernel breakdown of the update, the FETCH_SIZE / WRITE_SIZE traffic passes, a kernel trace
# of acting at 2^21 boards, and the config-5 bench extra three times (box spread).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05_dqn}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_dqn_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpurun/dqn_prof.sh $O/update || exit 1
bash tools/gpurun/dqn_traffic.sh $O/traffic || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/act -o act -- python3 tools/prof_dqn.py 5 act > $O/act.log 2>&1 || exit 1
grep "ms" $O/act.log
for i in 1 2 3; do
timeout -k 10 600 python -u -c "
import json, torch, bench
r = bench.dqn_config5(torch.device('cuda', 0), 0x20485EED, 1 << 21)
print(json.dumps(r), flush=True)
" >> $O/dqn_extra.jsonl 2>> $O/dqn.err || exit 1
done
python3 -c "
import json
for l in open('$O/dqn_extra.jsonl'):
    r = json.loads(l); print({k: r[k] for k in r if k.endswith('_ms') or 'frac' in k})"
