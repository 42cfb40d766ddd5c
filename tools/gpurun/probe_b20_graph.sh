#!/bin/bash
# GPU job: three driver-shaped bench runs at --steps 20 (value vs repeats) and the training-step
# HIP-graph probe.  usage: bash tools/gpurun/probe_b20_graph.sh
set -o pipefail
mkdir -p gpurun_out/b20
for i in 1 2 3; do
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/b20/b20_$i.json 2>/dev/null || exit 1
done
python tools/show_bench20.py gpurun_out/b20/b20_1.json gpurun_out/b20/b20_2.json gpurun_out/b20/b20_3.json \
&& timeout -k 10 300 python tools/probe_graph.py > gpurun_out/b20/graph.txt 2>&1; cat gpurun_out/b20/graph.txt
