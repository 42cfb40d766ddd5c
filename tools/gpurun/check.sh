#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, the driver's bench command (3 repeats at --steps 20
# for the spread), the per-kernel clocks of the CNN / MLP / ResNet kernels (clocks.sh), then the env
# profiles (prof_env.sh). Every GPU step has its own time limit;
# steps are chained so a failure stops the run.  usage: bash tools/gpurun/check.sh [round] [noprof]
set -o pipefail
R=${1:-r03}
OUT=gpurun_out/check_$R
mkdir -p $OUT
export TMPDIR=/tmp
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -2 $OUT/smoke.log \
&& echo "== pytest -m gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -5 $OUT/pytest_gpu.log; [ $rc -eq 0 ] \
&& echo "== bench" && timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err && cat $OUT/bench.json \
&& for i in 1 2 3; do timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $OUT/bench20_$i.json 2>> $OUT/bench.err || exit 1; done \
&& python -c "import json,sys; v=[json.load(open('$OUT/bench20_%d.json'%i))['value'] for i in (1,2,3)]; print('steps20', [round(x/1e9,1) for x in v], 'spread %.2f%%'%(100*(max(v)-min(v))/min(v)))" \
&& echo "== kernel clocks" && bash tools/gpurun/clocks.sh check_$R/clocks > /dev/null && python3 -c "import json; k=json.load(open('$OUT/clocks/kernel_clocks.json'))['kernels']; [print('%-40s %7.2f ms %5.2f GHz' % (n[:40], v['mean_dispatch_ms'], v['clock_ghz'])) for n, v in list(k.items())[:8]]" \
&& if [ "$2" != noprof ]; then echo "== prof_env" && bash tools/gpurun/prof_env.sh $R; fi
