set -o pipefail
O=gpurun_out/g32; mkdir -p $O
timeout -k 10 200 python tools/exp_policy.py 1048576 rein48_amd/lib/librein48.so build/lib_desync1.so build/lib_desync2.so build/lib_desync2s3.so rein48_amd/lib/librein48.so build/lib_desync1.so build/lib_desync2.so build/lib_desync2s3.so > $O/policy.txt 2>&1 \
&& timeout -k 10 200 python tools/exp_policy.py 8388608 rein48_amd/lib/librein48.so build/lib_desync2.so rein48_amd/lib/librein48.so build/lib_desync2.so >> $O/policy.txt 2>&1 \
&& timeout -k 10 300 python tools/exp_rollout.py rein48_amd/lib/librein48.so build/lib_desync1.so build/lib_desync2.so rein48_amd/lib/librein48.so build/lib_desync1.so build/lib_desync2.so > $O/rollout.txt 2>&1
echo rc=$?
