set -o pipefail
O=gpurun_out/g30; mkdir -p $O
timeout -k 10 200 python tools/exp_policy.py 1048576 rein48_amd/lib/librein48.so build/lib_split.so build/lib_chain.so rein48_amd/lib/librein48.so build/lib_split.so > $O/policy.txt 2>&1 \
&& timeout -k 10 300 python tools/exp_rollout.py rein48_amd/lib/librein48.so build/lib_split.so rein48_amd/lib/librein48.so build/lib_split.so > $O/rollout.txt 2>&1
echo rc=$?
