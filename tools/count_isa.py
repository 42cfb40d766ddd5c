"""Count VALU/SALU instructions per kernel in build/r48_env.s (make asm)."""
import re
import sys

s = open(sys.argv[1] if len(sys.argv) > 1 else "build/r48_env.s").read()
for m in re.finditer(r"^(_Z\S+):\s*;", s, re.M):
    name = m.group(1)
    j = s.index("s_endpgm", m.end())
    body = s[m.end():j]
    v = len(re.findall(r"^\s+v_", body, re.M))
    sa = len(re.findall(r"^\s+s_", body, re.M))
    print("%-70s VALU %4d SALU %3d mad64 %2d perm %2d" % (name[:70], v, sa, body.count("v_mad_u64_u32"),
                                                         body.count("v_perm")))
