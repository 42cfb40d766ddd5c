set -o pipefail
O=gpurun_out/g15; mkdir -p $O
timeout -k 10 120 build/mfma_chain > $O/mfma_chain.txt 2>&1 \
&& R48_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_2rank_gloo.json 2> $O/bench_2rank_gloo.err
echo rc=$?
