#!/bin/bash
# bench.py --steps 20 end-of-region wait A/B: the region's last event (event) vs torch.cuda.synchronize
# (device), processes alternated; prints value and repeat_5 of each run.
set -o pipefail
O=gpurun_out/close_ab; mkdir -p $O
for i in 1 2 3 4; do for m in event device; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extras --close $m > $O/b_${m}_$i.json 2>> $O/err.txt || exit 1
  python -c "import json; r=json.load(open('$O/b_${m}_$i.json')); print('$m', '%.1f G' % (r['value']/1e9), 'wall %.1f us dev %.1f us' % (r['roofline']['wall_ms_timed']*1e3, r['roofline']['device_ms_timed']*1e3), 'repeat_5', [round(v/1e9) for v in r['repeat_5']['values']])" | tee -a $O/ab.txt
done; done
