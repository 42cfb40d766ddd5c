"""LDS-bank-conflict scan: per kernel name (all dispatches, all grids) of one rocprofv3 --pmc pass,
the summed SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE and the conflict share of the LDS cycles, with
the kernel's dispatch count and summed duration; kernels by total duration.
usage: python tools/pmc_by_kernel.py <pmc dir> [<pmc dir> ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def scan(dirs):
    acc = defaultdict(lambda: defaultdict(float))
    seen = defaultdict(set)
    dur = defaultdict(float)
    for d in dirs:
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(p)):
                k = r.get("Kernel_Name", "")[:90]
                key = (p, r["Dispatch_Id"])
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
                if key not in seen[k]:
                    seen[k].add(key)
                    if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                        dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    rows = []
    for k, c in acc.items():
        lds = c.get("SQ_LDS_IDX_ACTIVE", 0.0)
        bc = c.get("SQ_LDS_BANK_CONFLICT", 0.0)
        rows.append((dur[k], k, len(seen[k]), lds, bc, bc / lds if lds else 0.0))
    rows.sort(reverse=True)
    print("%10s %5s %12s %12s %6s  %s" % ("us total", "disp", "LDS cycles", "conflict", "share", "kernel"))
    for d, k, n, lds, bc, sh in rows:
        print("%10.0f %5d %12.3g %12.3g %6.3f  %s" % (d, n, lds, bc, sh, k))


if __name__ == "__main__":
    scan(sys.argv[1:])
