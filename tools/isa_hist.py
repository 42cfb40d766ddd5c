"""Instruction histogram of chosen basic blocks of one kernel in an assembly file, with a modelled
issue cost per SIMD (cycles per wave-instruction measured by tools/instr_rate.hip on MI355X,
profiles/r02/instr_rate.txt; unknown opcodes count as full rate).
usage: python tools/isa_hist.py build/r48_env.s <kernel substring> <block label> [<block label> ...]"""
import collections
import re
import sys

FULL, HALF = 2.25, 4.33
COST = {"v_perm_b32": HALF, "v_bfi_b32": HALF, "v_lshlrev_b32": 4.27, "v_bcnt_u32_b32": 4.35, "v_mul_hi_u32": 4.35,
        "v_mad_u64_u32": 4.58, "v_or3_b32": 4.34, "v_add3_u32": 4.35, "v_and_or_b32": 4.31, "v_lshl_or_b32": 4.35,
        "v_lshl_add_u32": 4.38, "v_bfe_u32": 4.36, "v_min_u32_e32": 4.38, "v_max3_u32": 4.34, "v_alignbit_b32": 4.34,
        "v_bitop3_b32": 2.46, "v_xor3_b32": 2.46, "v_mul_lo_u32": 4.35, "v_cndmask_b32_e32": 4.28,
        "v_cndmask_b32_e64": 4.28, "v_lshrrev_b32": 2.24, "v_ashrrev_i32": 2.21}


def cost(op):
    for suf in ("_e32", "_e64"):
        if op.endswith(suf) and not op.startswith("v_cndmask"):
            op = op[:-len(suf)]
    if op in COST:
        return COST[op]
    if op.startswith("v_cmp"):
        return 2.4     # v_cmp alone (profiles/r02/instr_rate.txt: cmp64_cnd64 - cnd64)
    return FULL


s = open(sys.argv[1]).read()
m = re.search(r"^(_Z\S*%s\S*):\s*;" % re.escape(sys.argv[2]), s, re.M)
body = s[m.end():s.index(".Lfunc_end", m.end())]
want = set(sys.argv[3:])
c = collections.Counter()
for b in re.split(r"^(?=\.LBB\S+:|; %bb\.)", body, flags=re.M):
    if b.split(":")[0].split()[-1] in want:
        for ln in b.splitlines():
            t = ln.split()
            if t and t[0].startswith("v_"):
                c[t[0]] += 1
tot = sum(c.values())
cyc = sum(cost(k) * v for k, v in c.items())
for k, v in sorted(c.items(), key=lambda x: -x[1] * cost(x[0])):
    print("%4d %-26s %6.1f cyc" % (v, k, v * cost(k)))
print("VALU %d, modelled %.0f SIMD cycles per wave pass (%.2f per instruction)" % (tot, cyc, cyc / tot))
