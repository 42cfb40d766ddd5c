# final check of the shipped env build: GPU suite, bench (driver command, poll and block sync), profiles
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/g11; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
&& timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err \
&& timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline --sync block > $O/bench_block.json 2> $O/bench_block.err \
&& timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline --sync poll > $O/bench_poll.json 2> $O/bench_poll.err \
&& bash tools/prof_r02.sh > $O/prof.txt 2>&1
echo rc=$?
