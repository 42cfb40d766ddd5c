#!/bin/bash
# A/B of the untimed settling before the timed region at the driver's --steps 20 (GPU clock ramp
# after start-up): --settle 0.3 / 1.0 / 2.0 s, interleaved, 3 runs each.
set -o pipefail
OUT=gpurun_out/settle_ab
mkdir -p $OUT
for i in 1 2 3; do
  for s in 0.3 1.0 2.0; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extras --settle $s > $OUT/s${s}_$i.json 2>> $OUT/err.log || exit 1
  done
done
python - <<'PY'
import json
for s in ("0.3", "1.0", "2.0"):
    for i in (1, 2, 3):
        d = json.load(open("gpurun_out/settle_ab/s%s_%d.json" % (s, i)))
        r = d["repeat_5"]
        print("settle %s  %.1f G  repeat_5 %s  spread %.3f" % (s, d["value"] / 1e9, " ".join("%.0f" % (v / 1e9) for v in r["values"]), r["spread"]))
PY
