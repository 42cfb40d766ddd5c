"""Diagnostic variant of csrc/r48_a3c_train.hip with per-phase clock stamps (s_memtime) in
k_cnn_train's tile loop: writes build/var/r48_a3c_train_stamp.hip, whose kernel stores, per wave,
the cycles spent in each phase (summed over its tiles) over the first 8 words of its gradient record
(so that build's gradients are wrong: timing only). The product source holds no diagnostic code.
Phases: 0 tile head (inputs, Xt), 1 forward, 2 loss, 3 dh2 + dWh + dh2^T + db2, 5 position loop.

    python tools/stamp_train.py [source.hip [out.hip]] && tools/build_variant.sh \\
        build/var/r48_a3c_train_stamp.hip r48_a3c_train build/ab/lib_train_stamp.so -mllvm -amdgpu-mfma-vgpr-form=1
    python tools/exp_train_stamps.py build/ab/lib_train_stamp.so      (on the GPU)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "rein48_amd", "csrc", "r48_a3c_train.hip")
OUT = os.path.join(ROOT, "build", "var", "r48_a3c_train_stamp.hip")

MARKS = [
    ("        // ---------------- forward (", 0),
    ("        // ---------------- loss gradient per row", 1),
    ("        // ---------------- dh2 = Wh^T dout", 2),
    ("            fwd_conv2_heads_", 6),
    ("        // ---------------- per conv1 position R", 3),
    ("        const RowIn in = next;", 5),
]


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else SRC
    out = sys.argv[2] if len(sys.argv) > 2 else OUT
    s = open(src).read()
    s = s.replace('#include "r48_cnn_common.h"', '#include "r48_cnn_common.h"\n'
                  "#define R48_STAMP(k) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); "
                  "st_acc[k] += t_ - st_last; st_last = t_; }\n", 1)
    loop = "    for (int64_t tile = first; tile < n_tiles; tile += stride) {"
    assert loop in s
    s = s.replace(loop, "    unsigned long long st_acc[8] = {}, st_last = __builtin_amdgcn_s_memtime();\n" + loop, 1)
    for mark, k in MARKS:
        if s.count(mark) > 1:   # a source with #if alternatives of the call: stamp the first
            mark = mark + s.split(mark, 2)[1].split("(", 1)[0] + "("
        assert s.count(mark) == 1, mark
        s = s.replace(mark, "        R48_STAMP(%d)\n%s" % (k, mark), 1)
    end = "        rec[kOffLoss + 1] = red[6];\n    }\n"
    assert s.count(end) == 1
    s = s.replace(end, end + "    R48_STAMP(5)\n    if (lane == 0)\n        for (int k = 0; k < 8; k++)\n"
                  "            reinterpret_cast<unsigned long long *>(rec)[k] = st_acc[k];\n", 1)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    open(out, "w").write(s)
    print(out)


if __name__ == "__main__":
    main()
