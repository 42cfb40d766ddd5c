set -o pipefail
O=gpurun_out/g22; mkdir -p $O
timeout -k 10 300 python tools/exp_policy.py 8388608 build/lib_wd2.so build/lib_wd3.so build/lib_wd4.so build/lib_wd6.so build/lib_wd2.so build/lib_wd4.so build/lib_wd6.so > $O/wdepth.txt 2>&1
echo rc=$?
