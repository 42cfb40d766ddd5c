#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, bench, kernel-trace profile.
# Every GPU step has its own time limit; steps are chained so a failure stops the run.
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -2 $OUT/smoke.log \
&& echo "== pytest -m gpu" && timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -15 $OUT/pytest_gpu.log; [ $rc -eq 0 ] \
&& echo "== bench" && timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err && cat $OUT/bench.json \
&& echo "== chunks" && timeout -k 10 300 python tools/exp_chunks.py > $OUT/exp_chunks.txt 2>&1 && cat $OUT/exp_chunks.txt \
&& echo "== rocprof" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-extras --steps 1000 --warmup 2000 > $OUT/prof.log 2>&1 && ls -R $OUT/prof | head -20
[ $? -eq 0 ] && echo "== rocprof resnet" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_resnet -o run --output-format csv -- python tools/exp_resnet_fused.py > $OUT/prof_resnet.log 2>&1 && tail -1 $OUT/prof_resnet.log
[ $? -eq 0 ] && echo "== rocprof a3c" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_a3c -o a3c --output-format csv -- python tools/prof_a3c.py 2 > $OUT/prof_a3c.log 2>&1 && tail -1 $OUT/prof_a3c.log
