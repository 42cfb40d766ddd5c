set -o pipefail
O=gpurun_out/g23; mkdir -p $O
timeout -k 10 120 build/mfma_chain > $O/mfma_chain.txt 2>&1
echo rc=$?
