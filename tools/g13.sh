set -o pipefail
O=gpurun_out/g13; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_env.txt 2>&1 \
&& timeout -k 10 300 python tools/exp_dropin_latency.py 3000 > $O/dropin_latency.txt 2>&1
echo rc=$?
