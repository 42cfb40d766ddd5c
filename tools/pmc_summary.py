"""Per-dispatch means of rocprofv3 PMC counters for one kernel.

Reads every *counter_collection.csv under the given directories (one rocprofv3 --pmc pass
each), keeps the dispatches whose kernel name contains `kernel` and whose grid size equals
`grid` (threads), sums each counter over its instances (XCDs, SEs) per dispatch and averages
over dispatches.
usage: python tools/pmc_summary.py <kernel substring> <grid threads> <dir> [<dir> ...]  -> JSON"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def summarize(kernel, grid, dirs):
    per = defaultdict(lambda: defaultdict(float))   # (dir, dispatch) -> counter -> value
    dur = {}
    for d in dirs:
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(p)):
                if kernel not in r.get("Kernel_Name", ""):
                    continue
                g = int(r.get("Grid_Size", r.get("Grid_Size_X", "0")))
                if g != grid:
                    continue
                key = (d, r["Dispatch_Id"])
                per[key][r["Counter_Name"]] += float(r["Counter_Value"])
                if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                    dur[key] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    counters = defaultdict(list)
    for key, cs in per.items():
        for c, v in cs.items():
            counters[c].append(v)
    out = {"kernel": kernel, "grid_threads": grid,
           "dispatches": {c: len(v) for c, v in counters.items()},
           "per_dispatch_mean": {c: sum(v) / len(v) for c, v in sorted(counters.items())}}
    if dur:
        out["pmc_dispatch_ns_mean"] = sum(dur.values()) / len(dur)
    # clock and MFMA occupancy from the dispatches that carry GRBM_GUI_ACTIVE (summed over the 8 XCDs):
    # clock = GRBM / 8 / duration; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM / 8)
    clk = [cs["GRBM_GUI_ACTIVE"] / 8.0 / dur[k] for k, cs in per.items() if "GRBM_GUI_ACTIVE" in cs and dur.get(k)]
    busy = [cs["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * cs["GRBM_GUI_ACTIVE"] / 8.0) for cs in per.values()
            if "GRBM_GUI_ACTIVE" in cs and "SQ_VALU_MFMA_BUSY_CYCLES" in cs]
    m = out["per_dispatch_mean"]
    der = {}
    if clk:
        der["clock_ghz"] = sum(clk) / len(clk)
    if busy:
        der["mfma_busy_of_simd_cycles"] = sum(busy) / len(busy)
    if m.get("SQ_INSTS_VALU_MFMA_BF16") and m.get("SQ_INSTS_VALU"):
        der["non_mfma_valu_per_mfma"] = (m["SQ_INSTS_VALU"] - m["SQ_INSTS_VALU_MFMA_BF16"]) / m["SQ_INSTS_VALU_MFMA_BF16"]
    if m.get("SQ_VALU_MFMA_COEXEC_CYCLES") and m.get("SQ_VALU_MFMA_BUSY_CYCLES"):
        der["coexec_of_mfma_busy"] = m["SQ_VALU_MFMA_COEXEC_CYCLES"] / m["SQ_VALU_MFMA_BUSY_CYCLES"]
    if m.get("SQ_LDS_BANK_CONFLICT") and m.get("SQ_LDS_IDX_ACTIVE"):
        der["lds_conflict_of_lds_cycles"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]
    if der:
        out["derived"] = der
    return out


if __name__ == "__main__":
    print(json.dumps(summarize(sys.argv[1], int(sys.argv[2]), sys.argv[3:]), indent=1))
