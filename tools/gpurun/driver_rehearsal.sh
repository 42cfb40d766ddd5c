#!/bin/bash
# The driver's round-end sequence on one box: smoke, the GPU suite, then its exact bench command.
set -o pipefail
OUT=gpurun_out/driver_rehearsal
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log \
&& timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -1 $OUT/pytest_gpu.log; [ $rc -eq 0 ] \
&& timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && python tools/show_extras.py $OUT/bench.json
