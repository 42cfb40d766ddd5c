set -o pipefail
O=gpurun_out/g46; mkdir -p $O
A=rein48_amd/lib/librein48.so; B=build/lib_stage_plain.so
timeout -k 10 300 python tools/exp_policy.py 1048576 $A $B $A $B $A $B $B $A $B $A $B $A > $O/policy.txt 2>&1
echo rc=$?
