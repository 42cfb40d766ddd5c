set -o pipefail
O=gpurun_out/g16; mkdir -p $O
timeout -k 10 200 python tools/exp_policy_reg.py 1048576 rein48_amd/lib/librein48.so build/lib_fwdreg.so build/lib_fwdreg_agpr.so > $O/policy_reg.txt 2>&1 \
&& timeout -k 10 200 python tools/exp_policy_reg.py 8388608 rein48_amd/lib/librein48.so build/lib_fwdreg.so build/lib_fwdreg_agpr.so >> $O/policy_reg.txt 2>&1
echo rc=$?
