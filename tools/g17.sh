set -o pipefail
O=gpurun_out/g17; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
&& timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo rc=$?
