set -o pipefail
O=gpurun_out/g19; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_env.txt 2>&1 \
&& R48_LIB=build/lib_kstep_old.so timeout -k 10 200 python tools/exp_stepn.py old > $O/exp_old.txt 2>&1 \
&& R48_LIB=build/lib_kstep_lds.so timeout -k 10 200 python tools/exp_stepn.py lds > $O/exp_lds.txt 2>&1
echo rc=$?
