"""Per-step HBM traffic of k_step from rocprofv3 PMC passes -> profiles/pmc_k_step.json.

Two separate counter passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950):
    rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir>/fetch -o pmc -- python bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d <dir>/write -o pmc -- python bench.py ...
Corrections per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE/WRITE_SIZE are
in KiB; on gfx950 FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane) coalesced
streaming read, so it is doubled; WRITE_SIZE is exact for 16 B/lane stores (the 1 B/lane
action/done stores are uncalibrated widths -- reported as measured). Infinity-Cache hits are
counted by these fabric-side counters, so at 2^20 boards (cache-resident) this is traffic
beyond L2, not necessarily HBM.

usage: python tools/pmc_traffic.py <dir> <boards> [out.json]
"""
import csv
import glob
import json
import os
import re
import sys


def per_dispatch(path_glob, counter):
    """{(dispatch, boards in the launch): counter value summed over XCDs/instances}"""
    vals = {}
    for p in glob.glob(path_glob, recursive=True):
        for r in csv.DictReader(open(p)):
            name = r.get("Kernel_Name", "")
            if r.get("Counter_Name") != counter or "k_step<" not in name:
                continue
            np_ = int(re.search(r"k_step<[^>]*?(\d+)>", name).group(1))  # board pairs per lane (template NP)
            key = (r.get("Dispatch_Id"), int(r.get("Grid_Size", r.get("Grid_Size_X"))) * 2 * np_)
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return vals


def main():
    d, boards = sys.argv[1], int(sys.argv[2])
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join("profiles", "pmc_k_step.json")
    fetch = per_dispatch(os.path.join(d, "fetch", "**", "*counter_collection.csv"), "FETCH_SIZE")
    write = per_dispatch(os.path.join(d, "write", "**", "*counter_collection.csv"), "WRITE_SIZE")
    if not fetch or not write:
        raise SystemExit("no k_step FETCH_SIZE/WRITE_SIZE rows under %s" % d)
    # the bench's step launches: the shard-chain size (n/2 boards from 2^18 boards up)
    launch_boards = boards // 2 if boards >= (1 << 18) else boards
    f = [v for k, v in fetch.items() if k[1] == launch_boards]
    w = [v for k, v in write.items() if k[1] == launch_boards]
    if not f or not w:
        raise SystemExit("no k_step dispatches of %d boards" % launch_boards)
    fk, wk = sum(f) / len(f), sum(w) / len(w)
    per_launch = (2 * fk + wk) * 1024
    steps_share = boards // launch_boards
    res = {"boards": boards, "boards_per_launch": launch_boards, "launches_per_step": steps_share,
           "dispatches": {"fetch": len(f), "write": len(w)},
           "FETCH_SIZE_KiB_per_launch": fk, "WRITE_SIZE_KiB_per_launch": wk,
           "hbm_bytes_per_launch": per_launch, "hbm_bytes_per_step": per_launch * steps_share,
           "algorithmic_bytes_per_step": 34 * boards,
           "correction": "bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (gfx950 FETCH_SIZE halving)"}
    res["traffic_over_algorithmic"] = res["hbm_bytes_per_step"] / res["algorithmic_bytes_per_step"]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
