set -o pipefail
O=gpurun_out/g20; mkdir -p $O
timeout -k 10 200 python tools/exp_policy.py 1048576 rein48_amd/lib/librein48.so build/lib_pairs.so rein48_amd/lib/librein48.so build/lib_pairs.so > $O/policy_pairs.txt 2>&1 \
&& timeout -k 10 200 python tools/exp_policy.py 8388608 rein48_amd/lib/librein48.so build/lib_pairs.so >> $O/policy_pairs.txt 2>&1
echo rc=$?
