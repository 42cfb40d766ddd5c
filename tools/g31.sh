set -o pipefail
O=gpurun_out/g31; mkdir -p $O
R48_LIB=build/lib_slide3.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_a3c_gpu.py > $O/pytest_a3c_slide3.txt 2>&1 \
&& timeout -k 10 200 python tools/exp_policy.py 1048576 rein48_amd/lib/librein48.so build/lib_slide3.so build/lib_slide2.so rein48_amd/lib/librein48.so build/lib_slide3.so build/lib_slide2.so > $O/policy.txt 2>&1 \
&& timeout -k 10 300 python tools/exp_rollout.py rein48_amd/lib/librein48.so build/lib_slide3.so build/lib_slide3r2.so rein48_amd/lib/librein48.so build/lib_slide3.so build/lib_slide3r2.so > $O/rollout.txt 2>&1
echo rc=$?
