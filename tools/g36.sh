set -o pipefail
O=gpurun_out/g36; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_a3c_gpu.py > $O/pytest_a3c.txt 2>&1 \
&& timeout -k 10 300 python tools/exp_rollout.py build/lib_roll_old.so rein48_amd/lib/librein48.so build/lib_roll_old.so rein48_amd/lib/librein48.so build/lib_roll_old.so rein48_amd/lib/librein48.so > $O/rollout.txt 2>&1
echo rc=$?
