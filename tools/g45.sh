set -o pipefail
O=gpurun_out/g45; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_a3c_gpu.py > $O/pytest_a3c.txt 2>&1 \
&& timeout -k 10 200 python tools/exp_policy.py 1048576 build/lib_stage_plain.so rein48_amd/lib/librein48.so build/lib_stage_plain.so rein48_amd/lib/librein48.so build/lib_stage_plain.so rein48_amd/lib/librein48.so > $O/policy.txt 2>&1 \
&& timeout -k 10 200 python tools/exp_policy.py 100003 build/lib_stage_plain.so rein48_amd/lib/librein48.so build/lib_stage_plain.so rein48_amd/lib/librein48.so >> $O/policy.txt 2>&1 \
&& timeout -k 10 200 python tools/exp_policy.py 8388608 build/lib_stage_plain.so rein48_amd/lib/librein48.so build/lib_stage_plain.so rein48_amd/lib/librein48.so >> $O/policy.txt 2>&1
echo rc=$?
