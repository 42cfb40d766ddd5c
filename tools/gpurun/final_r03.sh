#!/bin/bash
# Round-end check of the shipped tree: smoke, the whole GPU suite, the bench line (with extras) and
# three runs of the driver's --steps 20 command.  usage: bash tools/gpurun/final_r03.sh
set -o pipefail
OUT=gpurun_out/final_r03
mkdir -p $OUT
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log \
&& echo "== pytest -m gpu" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] \
&& bash tools/gpurun/bench_only.sh final_r03 && python tools/show_extras.py $OUT/bench.json
