#!/bin/bash
# Round-4 session: the fused reference-MLP tests, its config-3-size A3C timings (bench.a3c_config3 with
# net mlp, both loss modes), then the k_step_n fairness A/B.
set -o pipefail
O=gpurun_out/r04_mlp; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_a3c_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "mlp" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -c "
import json, torch, bench
d = torch.device('cuda', 0)
for mode, feat in (('reference', 'values'), ('textbook', 'exponents')):
    r = bench.a3c_config3(d, 0x20485EED, 1 << 20, mode=mode, features=feat, net='mlp', bf16=False)
    print(json.dumps(r), flush=True)
" > $O/a3c_mlp.json 2> $O/a3c_mlp.err; rc=$?; cat $O/a3c_mlp.json; tail -3 $O/a3c_mlp.err; [ $rc -eq 0 ] || exit $rc
TEST_VAL=2 bash tools/gpurun/stepn_env_ab.sh R48_STEPN_FAIR r04_fair2 0 4 2 3 0 4 2 3
bash tools/gpurun/kstep_nt_ab.sh r04_nt
bash tools/gpurun/stepn_env_ab.sh HIP_FORCE_DEV_KERNARG r04_kernarg 0 1 0 1
