set -o pipefail
O=gpurun_out/g5; mkdir -p $O
R48_LIB=build/librein48_stamp.so timeout -k 10 120 python tools/exp_stamps.py 1048576 20 > $O/stamps_2p20_k20.txt 2>&1 \
&& R48_LIB=build/librein48_stamp.so timeout -k 10 120 python tools/exp_stamps.py 1048576 1000 > $O/stamps_2p20_k1000.txt 2>&1
echo rc=$?
