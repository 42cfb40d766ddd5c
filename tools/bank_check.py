"""Count 3-source VALU instructions whose VGPR sources share a bank (reg % 4) in chosen blocks
of a kernel (tools/bank_rate.hip measured: all three sources in one bank doubles the issue cost,
two in one bank costs nothing extra).
usage: python tools/bank_check.py build/r48_env.s <kernel substring> <block> [<block> ...]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
m = re.search(r"^(_Z\S*%s\S*):\s*;" % re.escape(sys.argv[2]), s, re.M)
body = s[m.end():s.index(".Lfunc_end", m.end())]
want = set(sys.argv[3:])
tot = collections.Counter()
hits = collections.Counter()
for b in re.split(r"^(?=\.LBB\S+:|; %bb\.)", body, flags=re.M):
    if b.split(":")[0].split()[-1] not in want:
        continue
    for ln in b.splitlines():
        t = ln.split(None, 1)
        if not t or not t[0].startswith("v_") or len(t) < 2:
            continue
        ops = [o.strip() for o in t[1].split(",")]
        srcs = []
        for o in ops[1:]:
            mm = re.match(r"v\[?(\d+)", o)
            if mm:
                srcs.append(int(mm.group(1)))
        if len(srcs) >= 3:
            tot[t[0]] += 1
            banks = collections.Counter(r % 4 for r in srcs)
            if max(banks.values()) >= 3:
                hits[t[0]] += 1
for k in sorted(tot, key=lambda x: -tot[x]):
    print("%-22s 3-VGPR-source %3d  all-same-bank %3d" % (k, tot[k], hits[k]))
