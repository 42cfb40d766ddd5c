"""Count VALU/SALU instructions per kernel in an assembly file (make asm / hipcc -S).

Per kernel: whole body (to .Lfunc_end), and per basic block for the hot loop of k_step_n
(--blocks prints every block's VALU count, so the loop body can be read off)."""
import re
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
s = open(args[0] if args else "build/r48_env.s").read()
pat = args[1] if len(args) > 1 else ""
for m in re.finditer(r"^(_Z\S+):\s*;", s, re.M):
    name = m.group(1)
    if pat not in name:
        continue
    j = s.index(".Lfunc_end", m.end())
    body = s[m.end():j]
    v = len(re.findall(r"^\s+v_", body, re.M))
    sa = len(re.findall(r"^\s+s_", body, re.M))
    print("%-72s VALU %4d SALU %3d mad64 %2d perm %2d" % (name[:72], v, sa, body.count("v_mad_u64_u32"),
                                                         body.count("v_perm")))
    if "--blocks" in sys.argv:
        for blk in re.split(r"^(?=\.LBB\S+:|; %bb\.)", body, flags=re.M):
            lab = blk.split(":")[0].split()[-1] if blk.startswith((".LBB", "; %bb")) else "(entry)"
            nv = len(re.findall(r"^\s+v_", blk, re.M))
            ns = len(re.findall(r"^\s+s_", blk, re.M))
            br = re.findall(r"^\s+(s_cbranch\w*|s_branch)\s+(\S+)", blk, re.M)
            print("    %-14s VALU %4d SALU %3d  %s" % (lab, nv, ns, " ".join("%s->%s" % b for b in br)))
