"""Instruction histogram of chosen basic blocks of one kernel in an assembly file, with a modelled
issue cost per SIMD (cycles per wave-instruction measured by tools/instr_rate.hip on MI355X,
profiles/r02/instr_rate.txt; unknown opcodes count as full rate).
usage: python tools/isa_hist.py build/r48_env.s <kernel substring> <block label> [<block label> ...]
       python tools/isa_hist.py build/r48_env.s <kernel substring> --auto-loop
--auto-loop: the loop (by its "Loop: Header=" annotations) holding the most VALU, its
unconditional blocks only (the .LBB-labelled ones; the %bb fall-through blocks of that loop are
its conditional branches: tile sum on the last step, auto-reset)."""
import collections
import re
import sys

FULL, HALF = 2.25, 4.33
COST = {"v_perm_b32": HALF, "v_bfi_b32": HALF, "v_lshlrev_b32": 4.27, "v_bcnt_u32_b32": 4.35, "v_mul_hi_u32": 4.35,
        "v_mad_u64_u32": 4.58, "v_or3_b32": 4.34, "v_add3_u32": 4.35, "v_and_or_b32": 4.31, "v_lshl_or_b32": 4.35,
        "v_lshl_add_u32": 4.38, "v_bfe_u32": 4.36, "v_min_u32_e32": 4.38, "v_max3_u32": 4.34, "v_alignbit_b32": 4.34,
        "v_bitop3_b32": 2.46, "v_xor3_b32": 2.46, "v_mul_lo_u32": 4.35, "v_cndmask_b32_e32": 4.28,
        "v_cndmask_b32_e64": 4.28, "v_lshrrev_b32": 2.24, "v_ashrrev_i32": 2.21,
        "v_xad_u32": 4.31, "v_add_lshl_u32": 4.32, "v_med3_u32": 4.39}   # last three: profiles/r05/env/instr_rate_r05.txt


def cost(op):
    for suf in ("_e32", "_e64"):
        if op.endswith(suf) and not op.startswith("v_cndmask"):
            op = op[:-len(suf)]
    if op in COST:
        return COST[op]
    if op.startswith("v_cmp"):
        return 2.4     # v_cmp alone (profiles/r02/instr_rate.txt: cmp64_cnd64 - cnd64)
    return FULL


def loop_blocks(body):
    """.LBB blocks of the loop with the most VALU (header included)."""
    loops = collections.defaultdict(list)
    for b in re.split(r"^(?=\.LBB\S+:|; %bb\.)", body, flags=re.M):
        lab = b.split(":")[0].split()[-1]
        head = b[:300]
        mm = re.search(r"Header=(BB\S+) Depth", head)
        hd = mm.group(1) if mm else (lab[2:] if "Loop Header" in head else None)
        if hd:
            loops[hd].append((lab, len(re.findall(r"^\s+v_", b, re.M))))
    best = max(loops.values(), key=lambda bl: sum(v for _, v in bl))
    return [lab for lab, _ in best if lab.startswith(".LBB")]


def analyse(path, kernel, blocks=None):
    s = open(path).read()
    m = re.search(r"^(_Z\S*%s\S*):\s*;" % re.escape(kernel), s, re.M)
    body = s[m.end():s.index(".Lfunc_end", m.end())]
    want = set(blocks) if blocks else set(loop_blocks(body))
    c = collections.Counter()
    for b in re.split(r"^(?=\.LBB\S+:|; %bb\.)", body, flags=re.M):
        if b.split(":")[0].split()[-1] in want:
            for ln in b.splitlines():
                t = ln.split()
                if t and t[0].startswith("v_"):
                    c[t[0]] += 1
    return c, sorted(want)


if __name__ == "__main__":
    args = [a for a in sys.argv[3:] if a != "--auto-loop"]
    c, blocks = analyse(sys.argv[1], sys.argv[2], args or None)
    tot = sum(c.values())
    cyc = sum(cost(k) * v for k, v in c.items())
    for k, v in sorted(c.items(), key=lambda x: -x[1] * cost(x[0])):
        print("%4d %-26s %6.1f cyc" % (v, k, v * cost(k)))
    print("blocks %s" % " ".join(blocks))
    print("VALU %d, modelled %.0f SIMD cycles per wave pass (%.2f per instruction)" % (tot, cyc, cyc / tot))
