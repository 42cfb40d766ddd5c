#!/bin/bash
# The driver's bench commands only: the default bench line (with extras) and three --steps 20 repeats.
# usage: bash tools/gpurun/bench_only.sh [out-dir name]
set -o pipefail
OUT=gpurun_out/${1:-bench_only}
mkdir -p $OUT
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err \
&& for i in 1 2 3; do timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $OUT/bench20_$i.json 2>> $OUT/bench.err || exit 1; done \
&& python -c "import json; v=[json.load(open('$OUT/bench20_%d.json'%i))['value'] for i in (1,2,3)]; print('steps20', [round(x/1e9,1) for x in v])"
