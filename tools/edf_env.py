"""Experiment variant of csrc/r48_env.hip: k_step_n's issue priority from a per-wave schedule
instead of the four progress phases. Each wave reads the core clock (s_memtime) every step; while
it is ahead of its schedule (step t begun before start + t * TREF cycles) it runs at priority 0,
otherwise at 3 -- the waves of a SIMD that fall behind take the issue slots until they catch up.
Writes build/var/r48_env_edf<TREF>.hip for each TREF given (core cycles per step).

    python tools/edf_env.py 7000 7900 9000 && for t in ...; do tools/build_variant.sh \\
        build/var/r48_env_edf$t.hip r48_env build/lib_env_edf$t.so; done"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "rein48_amd", "csrc", "r48_env.hip")


def variant(s, tref):
    a = s.index("        int32_t t = 0;\n#pragma nounroll\n        for (int ph = 0; ph < 4; ph++) {")
    b = s.index("            for (const int32_t end = ends[ph]; t < end; t++) {", a)
    s = s[:a] + ("        uint32_t due = (uint32_t)__builtin_amdgcn_s_memtime();\n"
                 "        int32_t t = 0;\n        {\n"
                 "            for (; t < n_steps; t++) {\n"
                 "                const uint32_t now = (uint32_t)__builtin_amdgcn_s_memtime();\n"
                 "                if ((int32_t)(now - due) < 0)\n"
                 "                    __builtin_amdgcn_s_setprio(0);\n"
                 "                else\n"
                 "                    __builtin_amdgcn_s_setprio(3);\n"
                 "                due += %du;\n" % tref) + s[b + len("            for (const int32_t end = ends[ph]; t < end; t++) {\n"):]
    return s


def main():
    s = open(SRC).read()
    os.makedirs(os.path.join(ROOT, "build", "var"), exist_ok=True)
    for t in sys.argv[1:]:
        out = os.path.join(ROOT, "build", "var", "r48_env_edf%s.hip" % t)
        open(out, "w").write(variant(s, int(t)))
        print(out)


if __name__ == "__main__":
    main()
