#!/bin/bash
# A/B of the bench's end-of-region synchronisation at the driver's --steps 20: block (default) vs
# spin (hipDeviceScheduleSpin), interleaved, 3 runs each.  usage: bash tools/gpurun/sync_ab.sh
set -o pipefail
OUT=gpurun_out/sync_ab
mkdir -p $OUT
for i in 1 2 3; do
  for m in block spin; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extras --sync $m > $OUT/$m$i.json 2>> $OUT/err.log || exit 1
  done
done
python - <<'PY'
import json
for m in ("block", "spin"):
    for i in (1, 2, 3):
        d = json.load(open("gpurun_out/sync_ab/%s%d.json" % (m, i)))
        r = d["repeat_5"]
        print("%-5s %.1f G  repeat_5 %s  spread %.3f" % (m, d["value"] / 1e9, " ".join("%.0f" % (v / 1e9) for v in r["values"]), r["spread"]))
PY
