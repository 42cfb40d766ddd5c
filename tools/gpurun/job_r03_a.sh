set -o pipefail
bash tools/gpurun/train_ab.sh build/lib_train_head.so \
&& timeout -k 10 120 python -u tools/exp_sync.py 20 > gpurun_out/sync.txt 2>&1 && cat gpurun_out/sync.txt \
&& timeout -k 10 120 python -u tools/exp_sync.py --spin 20 > gpurun_out/sync_spin.txt 2>&1 && cat gpurun_out/sync_spin.txt
