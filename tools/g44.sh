set -o pipefail
O=gpurun_out/g44; mkdir -p $O
timeout -k 10 400 python tools/exp_train_ablate.py 16777216 rein48_amd/lib/librein48.so build/lib_train_nobar.so build/ablate_train/librein48_skip1.so build/ablate_train/librein48_skip2.so build/ablate_train/librein48_skip4.so build/ablate_train/librein48_skip7.so rein48_amd/lib/librein48.so build/lib_train_nobar.so > $O/train_ablate.txt 2>&1
echo rc=$?
