#!/bin/bash
# GPU job: A3C GPU tests, config-3 train-step traces (a3c_prof.sh) and the bench line with extras.
set -o pipefail
mkdir -p gpurun_out && timeout -k 10 400 python -u -m pytest tests/test_a3c_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_a3c.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_a3c.log; [ $rc -eq 0 ] && bash tools/gpurun/a3c_prof.sh && timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_a3c.json 2> gpurun_out/bench_a3c.err && python tools/show_extras.py gpurun_out/bench_a3c.json
