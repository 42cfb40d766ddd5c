set -o pipefail
O=gpurun_out/g41; mkdir -p $O
R48_LIB=build/lib_roll_sync.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_a3c_gpu.py -k "rollout" > $O/pytest_sync.txt 2>&1 \
&& timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_a3c_gpu.py -k "rollout" > $O/pytest_product.txt 2>&1 \
&& timeout -k 10 300 python tools/exp_rollout.py build/lib_roll_head.so rein48_amd/lib/librein48.so build/lib_roll_sync.so build/lib_roll_head.so rein48_amd/lib/librein48.so build/lib_roll_sync.so > $O/rollout.txt 2>&1
echo rc=$?
