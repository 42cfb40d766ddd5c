set -o pipefail
O=gpurun_out/g18; mkdir -p $O
R48_LIB=build/lib_np2.so timeout -k 10 200 python tools/exp_stepn.py np2 > $O/exp_np2.txt 2>&1 \
&& timeout -k 10 200 python tools/exp_stepn.py np1 > $O/exp_np1.txt 2>&1
echo rc=$?
