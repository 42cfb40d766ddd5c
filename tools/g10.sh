set -o pipefail
O=gpurun_out/g10; mkdir -p $O
timeout -k 10 200 python tools/exp_stepn.py quarters > $O/exp_q.txt 2>&1 \
&& R48_LIB=build/lib_geo.so timeout -k 10 200 python tools/exp_stepn.py geo > $O/exp_geo.txt 2>&1 \
&& R48_LIB=build/lib_noprio.so timeout -k 10 200 python tools/exp_stepn.py noprio > $O/exp_noprio.txt 2>&1 \
&& timeout -k 10 200 python tools/exp_stepn.py quarters2 > $O/exp_q2.txt 2>&1
echo rc=$?
