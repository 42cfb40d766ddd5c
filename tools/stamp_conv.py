"""Diagnostic variant of csrc/r48_conv.hip with clock stamps (s_memtime) in k_conv_wgrad's step
loop: per wave, the cycles spent waiting for the step's DMAs (vmcnt), in the barrier, issuing the
k-steps with the next step's DMAs, summed over its steps, stored (vector stores) over the first words of the
workgroup's record after the record is written (so that build's weight gradients are wrong: timing
only). Writes build/var/conv_stamp.hip and links build/lib_conv_stamp.so.
    python tools/stamp_conv.py; python tools/exp_conv_stamps.py build/lib_conv_stamp.so  (on the GPU)"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "rein48_amd", "csrc", "r48_conv.hip")
OUT = os.path.join(ROOT, "build", "var", "conv_stamp.hip")


def rep(s, old, new):
    assert s.count(old) == 1, old
    return s.replace(old, new, 1)


def main():
    s = open(SRC).read()
    s = rep(s, '#include "../../include/rein48.h"\n', '#include "../../include/rein48.h"\n'
            "#define R48_STAMP(k) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); "
            "st_acc[k] += t_ - st_last; st_last = t_; }\n")
    # phases of a step: 0 vmcnt wait, 1 lgkm wait + barrier, 4 the k-steps with the next DMAs
    # between them (issue time: MFMAs may still run into the next phase)
    s = rep(s, "    for (int64_t i = 0; i < n_my; i++) {\n",
            "    unsigned long long st_acc[8] = {}, st_last = __builtin_amdgcn_s_memtime();\n"
            "    for (int64_t i = 0; i < n_my; i++) {\n        R48_STAMP(4)\n")
    s = rep(s, '        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");\n        __builtin_amdgcn_s_barrier();\n',
            '        R48_STAMP(0)\n        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");\n'
            "        __builtin_amdgcn_s_barrier();\n        R48_STAMP(1)\n")
    s = rep(s, '    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");              // no DMA outlives the kernel\n',
            '    R48_STAMP(4)\n    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");              // no DMA outlives the kernel\n')
    end = "                rec[(t * kCout + 16 * (cot0 + j) + 4 * g + i) * CIN + 16 * ct + i16] = acc[t][j][i];\n}\n"
    s = rep(s, end, end[:-2] + "    if (lane < 8)\n"
            "        reinterpret_cast<unsigned long long *>(rec)[8 * wave + lane] = st_acc[lane];\n}\n")
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    open(OUT, "w").write(s)
    subprocess.check_call(["bash", os.path.join(ROOT, "tools", "build_variant.sh"), OUT, "r48_conv",
                           os.path.join(ROOT, "build", "lib_conv_stamp.so")], cwd=ROOT)
    print(OUT)


if __name__ == "__main__":
    main()
