"""Diagnostic variant of csrc/r48_mlp.hip with per-phase clock stamps (s_memtime) in k_mlp_train's
tile loop: writes build/var/r48_mlp_stamp.hip, whose kernel stores, per wave, the cycles spent in
each phase (summed over its tiles) over the first 16 words of its gradient record (so that build's
gradients are wrong: timing only). The product source holds no diagnostic code.
Phases: 0 inputs, 1 forward (actor and critic), 3 loss, 4 stash + exact logits, 5 phase 2.

    python tools/stamp_mlp.py && tools/build_variant.sh build/var/r48_mlp_stamp.hip r48_mlp build/lib_mlp_stamp.so
    python tools/exp_mlp_stamps.py build/lib_mlp_stamp.so      (on the GPU)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "rein48_amd", "csrc", "r48_mlp.hip")
OUT = os.path.join(ROOT, "build", "var", "r48_mlp_stamp.hip")

MARKS = [
    ("            hidden_both(wp, x, acc, c);", 0),
    ("        const float wt = live ? wn[rr] : 0.0f;", 1),
    ("        wave_lds_sync();   // the previous tile's phase 2 has read the stash", 3),
    ("        // ---------------- phase 2: lane = hidden unit", 4),
    ("    }\n    // ---------------- this wave's record", 5),
]


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else SRC
    out = sys.argv[2] if len(sys.argv) > 2 else OUT
    s = open(src).read()
    s = s.replace('#include "r48_board.h"', '#include "r48_board.h"\n'
                  "#define R48_STAMP(k) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); "
                  "st_acc[k] += t_ - st_last; st_last = t_; }\n", 1)
    loop = "    for (int64_t tile = (int64_t)blockIdx.x * kTrainWaves + wave; tile < n_tiles; tile += stride) {"
    assert s.count(loop) == 1
    s = s.replace(loop, "    unsigned long long st_acc[8] = {}, st_last = __builtin_amdgcn_s_memtime();\n" + loop, 1)
    for mark, k in MARKS:
        assert s.count(mark) == 1, mark
        if mark.startswith("    }\n"):
            s = s.replace(mark, "        R48_STAMP(%d)\n%s" % (k, mark), 1)
        else:
            s = s.replace(mark, "        R48_STAMP(%d)\n%s" % (k, mark), 1)
    end = "        rec[kRec - 1] = 0.0f;\n    }\n"
    assert s.count(end) == 1
    s = s.replace(end, end + "    if (lane == 0)\n        for (int k = 0; k < 8; k++)\n"
                  "            reinterpret_cast<unsigned long long *>(rec)[k] = st_acc[k];\n", 1)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    open(out, "w").write(s)
    print(out)


if __name__ == "__main__":
    main()
