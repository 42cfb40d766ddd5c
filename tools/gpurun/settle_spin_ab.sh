#!/bin/bash
# bench.py --steps 20: settle loop sleeping in the blocking wait (default) vs spinning on its last
# event (--settle-spin), processes alternated; prints value, wall / device time and repeat_5.
set -o pipefail
O=gpurun_out/settle_spin_ab; mkdir -p $O
for i in 1 2 3 4; do for m in block spin; do
  F=""; [ $m = spin ] && F="--settle-spin"
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extras $F > $O/b_${m}_$i.json 2>> $O/err.txt || exit 1
  python -c "import json; r=json.load(open('$O/b_${m}_$i.json')); print('$m', '%.1f G' % (r['value']/1e9), 'wall %.1f us dev %.1f us' % (r['roofline']['wall_ms_timed']*1e3, r['roofline']['device_ms_timed']*1e3), 'repeat_5', [round(v/1e9) for v in r['repeat_5']['values']])" | tee -a $O/ab.txt
done; done
