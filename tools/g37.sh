set -o pipefail
O=gpurun_out/g37; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras >> $O/block.jsonl 2>>$O/err.txt || exit 1
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras --sync poll >> $O/poll.jsonl 2>>$O/err.txt || exit 1
  R48_BENCH_PIN=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras >> $O/pin.jsonl 2>>$O/err.txt || exit 1
done
echo rc=$?
