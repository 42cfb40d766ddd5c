set -o pipefail
O=gpurun_out/g8; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_env.txt 2>&1 \
&& timeout -k 10 200 python tools/exp_stepn.py pair > $O/exp.txt 2>&1 \
&& R48_LIB=build/librein48_stamp.so timeout -k 10 120 python tools/exp_stamps.py 1048576 20 > $O/stamps_2p20_k20.txt 2>&1
echo rc=$?
