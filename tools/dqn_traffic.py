"""Per-kernel HBM/fabric traffic of the config-5 update from two rocprofv3 PMC passes of
tools/prof_dqn.py (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950), against each
kernel's algorithmic bytes at the 64K-board minibatch.

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir>/fetch -o pmc -- python3 tools/prof_dqn.py 2
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d <dir>/write -o pmc -- python3 tools/prof_dqn.py 2
    python tools/dqn_traffic.py <dir> [updates]

Corrections per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): both counters are in KiB;
FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced reads on gfx950, so it is doubled
(every kernel listed reads 16 B per lane); WRITE_SIZE is taken as measured. The counters sit
behind L2, so Infinity-Cache hits count: this is traffic beyond L2, an upper bound on HBM bytes.
Only dispatches after the last k_store (the replay store of the last env step) are the updates."""
import collections
import csv
import glob
import os
import sys

A = 65536 * 16 * 64 * 2 / 1e6            # MB of one [64K boards, 16 cells, 64 ch] bf16 activation
M = 65536 * 16 * 8 / 1e6                 # MB of its ReLU-mask bytes
ALGO = {                                 # algorithmic MB per call: reads + writes
    "k_conv3x3<2, 0, 1, 0>": 2 * A,                       # x in, y out (+ tiny stats records)
    "k_conv3x3<1, 0, 1, 0>": 1.5 * A,                     # the stem: 32-plane x in, y out
    "k_conv3x3<2, 2, 2, 0>": 4 * A + 2 * M,               # dy, add, bn_x in (+ both masks), dx out
    "k_conv3x3<2, 1, 2, 0>": 4 * A + M,                   # dy, add, bn_x in (+ mask), dx out
    "k_conv3x3<2, 0, 2, 0>": 3 * A + M,                   # dy, bn_x in (+ mask), dx out
    "k_conv_wgrad<64>": 2 * A,                            # dy, x in (records out: small)
    "k_conv_wgrad<32>": 1.5 * A,
    "k_bn_apply<64, true, true, true>": 3 * A + M,        # y, residual in; z, mask out
    "k_bn_apply<64, true, false, true>": 2 * A + M,
    "k_bn_bwd_apply<64, true, true, true>": 4 * A + M,    # dz, mask, y in; dy, dres out
    "k_bn_bwd_apply<64, true, false, true>": 3 * A + M,
    "k_bn_bwd_reduce<64, true, true>": 2 * A + M,         # dz, mask, y in
    "k_q_head_fwd": A,
    "k_q_head_bwd": 2 * A,                                # h in, dh out (records out: small)
    "k_onehot32": 0.5 * A,
}


def load(path_glob, counter):
    rows = []
    for p in glob.glob(path_glob, recursive=True):
        for r in csv.DictReader(open(p)):
            if r.get("Counter_Name") == counter:
                rows.append(r)
    by = collections.defaultdict(lambda: [None, 0.0, 0])     # dispatch -> [name, value, start]
    for r in rows:
        d = by[r["Dispatch_Id"]]
        d[0] = r["Kernel_Name"]
        d[1] += float(r["Counter_Value"])
        d[2] = int(r.get("Start_Timestamp") or r["Dispatch_Id"])
    return by


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return (name[5:] if name.startswith("void ") else name).split("(")[0]


def per_kernel(by, n):
    items = sorted(by.values(), key=lambda v: v[2])
    last = max(i for i, v in enumerate(items) if "k_store" in v[0])
    tot, cnt = collections.defaultdict(float), collections.Counter()
    for name, val, _ in items[last + 1:]:
        tot[short(name)] += val
        cnt[short(name)] += 1
    return tot, cnt


def main():
    d = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    f, fc = per_kernel(load(os.path.join(d, "fetch", "**", "*counter_collection.csv"), "FETCH_SIZE"), n)
    w, _ = per_kernel(load(os.path.join(d, "write", "**", "*counter_collection.csv"), "WRITE_SIZE"), n)
    print("%-44s %6s %10s %10s %10s %9s" % ("kernel", "calls", "read MB", "write MB", "algo MB", "traffic/algo"))
    tr_all = al_all = 0.0
    for k in sorted(f, key=lambda k: -(f[k] * 2 + w.get(k, 0))):
        calls = fc[k]
        rd, wr = f[k] * 2 * 1024 / 1e6 / calls, w.get(k, 0) * 1024 / 1e6 / calls
        algo = ALGO.get(k)
        tr_all += (rd + wr) * calls / n
        if algo:
            al_all += algo * calls / n
        print("%-44s %6.1f %10.1f %10.1f %10s %9s" % (k[:44], calls / n, rd, wr, "%.1f" % algo if algo else "-",
                                                    "%.3f" % ((rd + wr) / algo) if algo else "-"))
    print("per update: %.0f MB beyond L2 over all kernels; %.0f MB algorithmic for the listed ones" % (tr_all, al_all))


if __name__ == "__main__":
    main()
