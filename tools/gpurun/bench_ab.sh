#!/bin/bash
# A/B of bench.py options at the driver's region (--gpus 1 --steps 20 --warmup 5, no CPU baseline,
# no extras), processes alternated, 4 rounds; prints value, wall / device time and repeat_5 per run.
# usage: bash tools/gpurun/bench_ab.sh OUTDIR "label:flags" "label:flags" ...
#   e.g. bash tools/gpurun/bench_ab.sh close_ab "event:--close event" "device:--close device"
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
for i in 1 2 3 4; do for v in "$@"; do
  m=${v%%:*}; F=${v#*:}
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extras $F > $O/b_${m}_$i.json 2>> $O/err.txt || exit 1
  python -c "import json; r=json.load(open('$O/b_${m}_$i.json')); print('$m', '%.1f G' % (r['value']/1e9), 'wall %.1f us dev %.1f us' % (r['roofline']['wall_ms_timed']*1e3, r['roofline']['device_ms_timed']*1e3), 'repeat_5', [round(v/1e9) for v in r['repeat_5']['values']])" | tee -a $O/ab.txt
done; done
