"""Average clock of every kernel in one rocprofv3 --pmc GRBM_GUI_ACTIVE pass (tools/prof_clocks.py):
per dispatch GRBM_GUI_ACTIVE (summed over the 8 XCDs) / 8 / (End - Start), averaged per kernel name
weighted by time, for kernels of at least `min_us` per dispatch (the quotient reads high on
dispatches shorter than ~0.3 ms: /opt/skills/guides/MI355X_MICROARCH.md, DVFS give-back).
usage: python tools/kernel_clocks.py <pmc dir> [min_us=100]  -> JSON on stdout"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def clocks(d, min_us=100.0):
    per = defaultdict(lambda: [0, 0.0, 0.0])      # dispatches, summed ns, summed cycles
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
                continue
            ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            if ns < min_us * 1e3:
                continue
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "")
            k = (k[5:] if k.startswith("void ") else k).split("(")[0][:80]
            e = per[k]
            e[0] += 1
            e[1] += ns
            e[2] += float(r["Counter_Value"]) / 8.0
    out = {k: {"dispatches": v[0], "mean_dispatch_ms": v[1] / v[0] / 1e6, "clock_ghz": v[2] / v[1]}
           for k, v in sorted(per.items(), key=lambda kv: -kv[1][1])}
    return out


if __name__ == "__main__":
    res = clocks(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 100.0)
    print(json.dumps({"source": "rocprofv3 --pmc GRBM_GUI_ACTIVE of tools/prof_clocks.py; clock = GRBM_GUI_ACTIVE / 8 "
                                "/ dispatch time (time-weighted per kernel)", "kernels": res}, indent=1))
