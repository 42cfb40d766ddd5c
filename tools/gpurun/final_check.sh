#!/bin/bash
# Round-end session: k_step_n per-wave stamps at K = 20 / 1000 (diagnostic build from
# tools/stamp_env.py), the standard check (smoke, GPU tests, bench + --steps 20 repeats), then a
# two-rank gloo rehearsal of the multi-GPU bench path (both ranks on the one GPU).
# usage: bash tools/gpurun/final_check.sh r03
set -o pipefail
R=${1:-r03}
O=gpurun_out/check_$R; mkdir -p $O
R48_LIB=build/librein48_stamp.so timeout -k 10 120 python tools/exp_stamps.py 1048576 20 > $O/stamps_k20.txt 2>&1 \
&& R48_LIB=build/librein48_stamp.so timeout -k 10 120 python tools/exp_stamps.py 1048576 1000 > $O/stamps_k1000.txt 2>&1 \
&& cat $O/stamps_k20.txt $O/stamps_k1000.txt \
&& bash tools/gpurun/check.sh $R noprof \
&& echo "== 2-rank gloo rehearsal" && R48_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_2rank_gloo.json 2> $O/bench_2rank_gloo.err && cat $O/bench_2rank_gloo.json
