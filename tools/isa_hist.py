"""Instruction histogram of chosen basic blocks of one kernel in an assembly file, with a modelled
issue cost per SIMD (cycles per wave-instruction measured by tools/instr_rate.hip on MI355X,
profiles/r02/instr_rate.txt; unknown opcodes count as full rate).
usage: python tools/isa_hist.py build/r48_env.s <kernel substring> <block label> [<block label> ...]
       python tools/isa_hist.py build/r48_env.s <kernel substring> --auto-loop
--auto-loop: the loop (by its "Loop: Header=" annotations) holding the most VALU, its
unconditional blocks only (the .LBB-labelled ones; the %bb fall-through blocks of that loop are
its conditional branches: tile sum on the last step, auto-reset).
model(): the opcode costs plus the measured operand costs (literal, inline constant) and the SIMD's
SGPR-read limit (profiles/r05/env/instr_rate_r05.txt)."""
import collections
import re
import sys

FULL, HALF = 2.25, 4.33
COST = {"v_perm_b32": HALF, "v_bfi_b32": HALF, "v_lshlrev_b32": 4.27, "v_bcnt_u32_b32": 4.35, "v_mul_hi_u32": 4.35,
        "v_mad_u64_u32": 4.58, "v_or3_b32": 4.34, "v_add3_u32": 4.35, "v_and_or_b32": 4.31, "v_lshl_or_b32": 4.35,
        "v_lshl_add_u32": 4.38, "v_bfe_u32": 4.36, "v_min_u32_e32": 4.38, "v_max3_u32": 4.34, "v_alignbit_b32": 4.34,
        "v_bitop3_b32": 2.46, "v_xor3_b32": 2.46, "v_mul_lo_u32": 4.35, "v_cndmask_b32_e32": 4.28,
        "v_cndmask_b32_e64": 4.28, "v_lshrrev_b32": 2.24, "v_ashrrev_i32": 2.21,
        "v_xad_u32": 4.31, "v_add_lshl_u32": 4.32, "v_med3_u32": 4.39,   # these three: profiles/r05/env/instr_rate_r05.txt
        # packed 16-bit VALU (the CNN kernels' ReLU / ReLU' masks): half rate (pkmax 4.38, pkadd 4.35 of
        # profiles/r05/env/instr_rate_r05.txt; min / mul_lo assumed the same)
        "v_pk_max_i16": 4.38, "v_pk_add_u16": 4.35, "v_pk_min_u16": 4.38, "v_pk_mul_lo_u16": 4.38,
        # profiles/r06/isa/instr_rate16.txt (8 waves per SIMD)
        "v_cvt_pk_bf16_f32": 4.19, "v_pk_max_f16": 4.26, "v_pk_mul_f16": 4.21, "v_pk_add_f16": 4.20,
        "v_pk_fma_f16": 4.16, "v_max_i16": 2.42, "v_permlane16_swap_b32": 8.15, "v_permlane32_swap_b32": 8.21}


def cost(op):
    for suf in ("_e32", "_e64"):
        if op.endswith(suf) and not op.startswith("v_cndmask"):
            op = op[:-len(suf)]
    if op in COST:
        return COST[op]
    if op.startswith("v_cmp"):
        return 2.4     # v_cmp alone (profiles/r02/instr_rate.txt: cmp64_cnd64 - cnd64)
    return FULL


# operand pricing (profiles/r05/env/instr_rate_r05.txt, 8 waves per SIMD): a 32-bit literal adds ~12 %
# to a full-rate instruction (sub_lit 2.49 / and_lit 2.48 vs 2.23), an inline constant ~7 % (xor_inl
# 2.39); a VALU reading an SGPR issues at ~4.2 cycles back to back (sub_sgpr 4.17, and_sgpr 4.16,
# bitop3_vvs_s 4.21, add_e64_s 4.19) but is free beside VGPR-only instructions (mix_sv 4.52 vs mix_vv
# 4.56 per pair): a SIMD-wide limit of one SGPR-reading VALU per ~4.2 cycles, not a per-instruction
# cost. Half-rate instructions' operand costs are unmeasured (not priced).
LIT_EXTRA, INL_EXTRA, SGPR_CYC = 0.26, 0.16, 4.2
_SDST = ("v_mad_u64_u32", "v_mad_i64_i32", "v_add_co_u32", "v_sub_co_u32", "v_subrev_co_u32", "v_addc_co_u32",
         "v_subb_co_u32", "v_subbrev_co_u32", "v_div_scale_f32", "v_div_scale_f64")
_INLINE_F = {"0.5", "-0.5", "1.0", "-1.0", "2.0", "-2.0", "4.0", "-4.0", "0.15915494"}


def operands(line):
    """(opcode, source operand tokens) of one assembly line: destinations and modifiers dropped."""
    t = line.split(None, 1)
    op = t[0]
    rest = t[1].split(";")[0] if len(t) > 1 else ""
    toks = [x.strip() for x in rest.split(",") if x.strip()]
    toks = [x.split()[0] for x in toks if x.split()]               # "s34 bitop3:0x80" -> "s34"
    toks = [x for x in toks if ":" not in x or x.startswith(("v[", "s["))]
    base = op[:-4] if op.endswith(("_e32", "_e64")) else op
    ndst = 2 if base in _SDST else (1 if not (base.startswith("v_cmp") and op.endswith("_e32")) else 0)
    if base.startswith("v_cmpx"):
        ndst = 0
    return op, toks[ndst:]


def _kind(tok):
    tok = tok.lstrip("-|").rstrip("|")
    if tok.startswith(("v", "a")) and (tok[1:2].isdigit() or tok[1:2] == "["):
        return "vgpr"
    if tok.startswith(("s[", "vcc", "exec", "ttmp", "m0")) or (tok.startswith("s") and tok[1:2].isdigit()):
        return "sgpr"
    try:
        v = int(tok, 0)
        return "inline" if -16 <= v <= 64 else "literal"
    except ValueError:
        pass
    return "inline" if tok in _INLINE_F else "literal"


def model(lines):
    """Modelled SIMD issue cycles of one wave pass over `lines` (VALU assembly lines): the sum of the
    per-opcode issue costs plus the operand costs of full-rate instructions (literal, inline
    constant), and the SIMD's SGPR-read limit as a separate bound; modelled = the larger."""
    base = lit = inl = 0.0
    n_sgpr = n_lit = n_inl = 0
    for ln in lines:
        op, src = operands(ln)
        c = cost(op)
        base += c
        kinds = [_kind(x) for x in src]
        if "sgpr" in kinds:
            n_sgpr += 1
        if c <= FULL + 0.3:
            if "literal" in kinds:
                lit += LIT_EXTRA
                n_lit += 1
            elif "inline" in kinds:
                inl += INL_EXTRA
                n_inl += 1
    total = base + lit + inl
    return {"valu": len(lines), "opcode_cycles": base, "literal_cycles": lit, "inline_cycles": inl,
            "n_literal": n_lit, "n_inline": n_inl, "n_sgpr_read": n_sgpr, "sgpr_bound_cycles": SGPR_CYC * n_sgpr,
            "issue_cycles": total, "modelled_cycles": max(total, SGPR_CYC * n_sgpr),
            "binding": "issue" if total >= SGPR_CYC * n_sgpr else "sgpr reads"}


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


def loop_lines(path, kernel, blocks=None):
    """The VALU lines of the chosen blocks (default: the auto-detected hot loop) and the block labels."""
    s = open(path).read()
    m = re.search(r"^(_Z\S*%s\S*):\s*;" % re.escape(kernel), s, re.M)
    body = s[m.end():s.index(".Lfunc_end", m.end())]
    want = set(blocks) if blocks else set(loop_blocks(body))
    out = []
    for b in re.split(r"^(?=\.LBB\S+:|; %bb\.)", body, flags=re.M):
        if b.split(":")[0].split()[-1] in want:
            for ln in b.splitlines():
                t = ln.split()
                if t and t[0].startswith("v_"):
                    out.append(ln.strip())
    return out, sorted(want)


def analyse(path, kernel, blocks=None):
    lines, want = loop_lines(path, kernel, blocks)
    return collections.Counter(ln.split()[0] for ln in lines), want


if __name__ == "__main__":
    args = [a for a in sys.argv[3:] if a != "--auto-loop"]
    c, blocks = analyse(sys.argv[1], sys.argv[2], args or None)
    tot = sum(c.values())
    cyc = sum(cost(k) * v for k, v in c.items())
    for k, v in sorted(c.items(), key=lambda x: -x[1] * cost(x[0])):
        print("%4d %-26s %6.1f cyc" % (v, k, v * cost(k)))
    print("blocks %s" % " ".join(blocks))
    print("VALU %d, opcode-only %.0f SIMD cycles per wave pass (%.2f per instruction)" % (tot, cyc, cyc / tot))
    mdl = model(loop_lines(sys.argv[1], sys.argv[2], args or None)[0])
    print("with operands: %.0f issue cycles (+%.0f for %d literals, +%.0f for %d inline constants); SGPR-read bound "
          "%.0f (%d reads x %.1f); modelled %.0f (%s-bound)"
          % (mdl["issue_cycles"], mdl["literal_cycles"], mdl["n_literal"], mdl["inline_cycles"], mdl["n_inline"],
             mdl["sgpr_bound_cycles"], mdl["n_sgpr_read"], SGPR_CYC, mdl["modelled_cycles"], mdl["binding"]))
