set -o pipefail
O=gpurun_out/g43; mkdir -p $O
R48_LIB=build/lib_train_grouped.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_a3c_gpu.py -k "update" > $O/pytest_grouped.txt 2>&1 \
&& timeout -k 10 300 python tools/exp_train_ablate.py 16777216 rein48_amd/lib/librein48.so build/lib_train_grouped.so rein48_amd/lib/librein48.so build/lib_train_grouped.so rein48_amd/lib/librein48.so build/lib_train_grouped.so > $O/train.txt 2>&1
echo rc=$?
