"""Print value, repeat_5 values and the region's wall / device ms of bench.py JSON lines."""
import json
import sys

for p in sys.argv[1:]:
    d = json.load(open(p))
    r = d.get("repeat_5", {})
    print("%-28s value %.1f G  repeats %s  wall %.4f ms  device %.4f ms" % (
        p, d["value"] / 1e9, [round(v / 1e9, 1) for v in r.get("values", [])],
        d["roofline"]["wall_ms_timed"], d["roofline"]["device_ms_timed"]))
