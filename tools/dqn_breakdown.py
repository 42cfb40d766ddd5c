"""Per-update kernel breakdown of a tools/prof_dqn.py kernel trace: the dispatches after the last
k_store (the updates), grouped by kernel, divided by the number of updates.
    python tools/dqn_breakdown.py <dqn_kernel_trace.csv> [updates] [> breakdown.txt]"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = max(i for i, r in enumerate(rows) if "k_store" in r["Kernel_Name"])
    upd = rows[last + 1:]
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for r in upd:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        name = (name[5:] if name.startswith("void ") else name).split("(")[0]
        tot[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[name] += 1
    span = (int(upd[-1]["End_Timestamp"]) - int(upd[0]["Start_Timestamp"])) / 1e3 / n
    busy = sum(tot.values()) / n
    print("updates %d: wall span %.1f us per update, kernel time %.1f us per update, %d dispatches per update"
          % (n, span, busy, len(upd) // n))
    print("%-70s %7s %10s %8s" % ("kernel", "calls/u", "us/update", "avg us"))
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print("%-70s %7.1f %10.1f %8.1f" % (k[:70], cnt[k] / n, v / n, v / cnt[k]))


if __name__ == "__main__":
    main()
