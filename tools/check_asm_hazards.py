#!/usr/bin/env python3
"""Wait-state check for the inline-asm MFMAs of a gfx950 assembly listing (hipcc -S).

hipcc pads no hazard inside or around an inline-asm statement, so the accumulating MFMAs of
csrc/r48_a3c_train.hip (mfma_acc32 / mfma_acc16) rely on two properties this tool verifies on the
compiled code:
  1. no A/B operand register of an asm MFMA is written by a VALU instruction (including
     v_accvgpr_write / v_accvgpr_mov) within the 2 wait states before it, counting each
     instruction as one state and `s_nop N` as N + 1 (the asm's own leading s_nop counts);
  2. the asm MFMA's accumulator (D = C) is read or written by nothing but the next asm MFMA of
     the same chain (same D, taking it whole as C) for 18 wait states after it (the 16-pass XDL
     write -> read distance, rounded up).
Exit status 1 and one line per violation if either fails.

    python tools/check_asm_hazards.py build/r48_a3c_train.s
"""
import re
import sys

VALU_WRITE_STATES = 2
MFMA_D_STATES = 18


def regs(tok):
    """'v[4:7]' -> {('v',4)..('v',7)}; 'a12' -> {('a',12)}; other operands -> empty."""
    tok = tok.strip()
    m = re.match(r"^([va])\[(\d+):(\d+)\]$", tok)
    if m:
        return {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"^([va])(\d+)$", tok)
    if m:
        return {(m.group(1), int(m.group(2)))}
    return set()


def parse(path):
    """Instructions of the listing: (text, in_asm, operands list)."""
    out, in_asm = [], False
    for raw in open(path):
        line = raw.split(";", 1)[0].strip() if not raw.strip().startswith(";;#ASM") else raw.strip()
        if line.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if line.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not line or line.endswith(":") or line.startswith("."):
            continue
        parts = line.split(None, 1)
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        out.append((parts[0], in_asm, ops, line))
    return out


def states(inst):
    op, _, ops, _ = inst
    if op == "s_nop":
        return int(ops[0], 0) + 1
    return 1


def main():
    insts = parse(sys.argv[1])
    bad = []
    for i, (op, in_asm, ops, line) in enumerate(insts):
        if not (in_asm and op.startswith("v_mfma")):
            continue
        dst = regs(ops[0])
        srcab = regs(ops[1]) | regs(ops[2])
        # 1. VALU write of an A/B operand within 2 wait states before
        ws, k = 0, i - 1
        while k >= 0 and ws < VALU_WRITE_STATES:
            pop, _, pops, pline = insts[k]
            if pop.startswith("v_") and not pop.startswith("v_mfma") and pops and regs(pops[0]) & srcab:
                bad.append("VALU->MFMA operand: %r then %r" % (pline, line))
                break
            ws += states(insts[k])
            k -= 1
        # 2. D readers / writers within 18 wait states after
        ws, k = 0, i + 1
        while k < len(insts) and ws < MFMA_D_STATES:
            pop, pin, pops, pline = insts[k]
            if pin and pop == op and regs(pops[0]) == dst and regs(pops[3]) == dst:
                break                                   # next MFMA of the same chain: forwarded
            touched = set()
            for o in pops:
                touched |= regs(o)
            if touched & dst:
                bad.append("MFMA D too early: %r then %r" % (line, pline))
                break
            ws += states(insts[k])
            k += 1
    for b in bad:
        print(b)
    print("%s: %d asm MFMAs checked, %d violations" % (sys.argv[1], sum(1 for x in insts if x[1] and x[0].startswith("v_mfma")), len(bad)))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
