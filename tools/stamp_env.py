"""Diagnostic variant of csrc/r48_env.hip with per-wave clock stamps in k_step_n: the core clock
(s_memtime) and the 100 MHz reference clock (s_memrealtime) at entry and exit plus HW_ID (CU /
SIMD / XCC) of every wave, read back by r48_debug_stamps (exported by this build only). The
product source carries no stamp code. Writes build/var/env_stamp.hip and links
build/librein48_stamp.so:
    python tools/stamp_env.py; R48_LIB=build/librein48_stamp.so python tools/exp_stamps.py  (on the GPU)"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "rein48_amd", "csrc", "r48_env.hip")
OUT = os.path.join(ROOT, "build", "var", "env_stamp.hip")

STAMP_DEFS = r"""
__device__ unsigned long long r48_stamp_buf[65536 * 4];
#define R48_STAMP_BEGIN                                                                  \
    const unsigned long long st_t0 = __builtin_amdgcn_s_memtime(), st_r0 = __builtin_amdgcn_s_memrealtime();
#define R48_STAMP_END                                                                    \
    if ((threadIdx.x & 63) == 0) {                                                       \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime(); \
        const unsigned w = blockIdx.x * (kBlock / 64) + threadIdx.x / 64;                \
        if (w < 65536) {                                                                 \
            unsigned hw, xcc;                                                            \
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));             \
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));           \
            hw = (hw & 0x0FFFFFFFu) | ((xcc & 0xFu) << 28);                              \
            r48_stamp_buf[4 * w] = st_t0; r48_stamp_buf[4 * w + 1] = st_r0;              \
            r48_stamp_buf[4 * w + 2] = t1 - st_t0; r48_stamp_buf[4 * w + 3] = ((r1 - st_r0) << 32) | hw; \
        }                                                                                \
    }
"""

EXPORT = r"""
extern "C" int r48_debug_stamps(unsigned long long *out, int64_t n_waves)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(r48_stamp_buf), sizeof(unsigned long long) * 4 * n_waves) == hipSuccess
               ? 0 : -1;
}
"""


def rep(s, old, new):
    assert s.count(old) == 1, old
    return s.replace(old, new, 1)


def main():
    s = open(SRC).read()
    head = "// ---------------------------------------------------------------- K steps in one launch\n"
    s = rep(s, head, STAMP_DEFS + head)
    s = rep(s, "    const int32_t last = n_steps - 1;\n", "    const int32_t last = n_steps - 1;\n    R48_STAMP_BEGIN\n")
    # the kernel's closing lines: the guarded path's end, then the kernel's
    s = rep(s, "                emit<RANDOM, REWARD>(r, i, boards, actions, done, changed, reward, score);\n"
               "            }\n        }\n    }\n}\n",
            "                emit<RANDOM, REWARD>(r, i, boards, actions, done, changed, reward, score);\n"
            "            }\n        }\n    }\n    R48_STAMP_END\n}\n")
    s += EXPORT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    open(OUT, "w").write(s)
    subprocess.check_call(["bash", os.path.join(ROOT, "tools", "build_variant.sh"), OUT, "r48_env",
                           os.path.join(ROOT, "build", "librein48_stamp.so")], cwd=ROOT)
    print(OUT)


if __name__ == "__main__":
    main()
