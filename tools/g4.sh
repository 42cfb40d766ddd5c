set -o pipefail
O=gpurun_out/g4; mkdir -p $O
timeout -k 10 120 build/bank_rate > $O/bank_rate.txt 2>&1 \
&& R48_LIB=build/librein48_stamp.so timeout -k 10 120 python tools/exp_stamps.py 1048576 20 > $O/stamps_2p20_k20.txt 2>&1 \
&& R48_LIB=build/librein48_stamp.so timeout -k 10 120 python tools/exp_stamps.py 1048576 1000 > $O/stamps_2p20_k1000.txt 2>&1 \
&& R48_LIB=build/librein48_stamp.so timeout -k 10 120 python tools/exp_stamps.py 4194304 100 > $O/stamps_2p22_k100.txt 2>&1
echo rc=$?
