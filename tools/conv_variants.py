"""Ablation variants of rein48_amd/csrc/r48_conv.hip for timing experiments (tools/exp_conv.py):
each variant is the product source with one textual edit, written to build/var/ and linked into
build/lib_conv_<name>.so by tools/build_variant.sh. The product source carries no ablation switches.
usage: python tools/conv_variants.py [name ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "rein48_amd", "csrc", "r48_conv.hip")

VARIANTS = {
    # conv3x3: outputs never stored (a runtime condition that is never true keeps the math alive)
    "fwd_nostore": [("            if (live) {\n#pragma unroll\n                    for (int col",
                     "            if (live && boards == -7) {\n#pragma unroll\n                    for (int col")],
    # conv3x3: rows loaded once (prologue), no loads inside the tile loop
    "fwd_noload": [("            load_row(r < 2 ? tile : (next < n_tiles ? next : tile), r < 2 ? r + 2 : r - 2);\n", "")],
    # conv3x3: the same loads and stores with lane-contiguous addresses (the tile's 16 boards x 2 KiB
    # read and written as 1 KiB / 512 B runs per instruction; wrong results: access-shape timing)
    "fwd_coalesced": [
        ("        const uint16_t *src = x + ((b < boards ? b : boards - 1) * 16 + 4 * R) * kCin + 8 * g;",
         "        const uint16_t *src = x + ((t < (boards + 15) / 16 ? t : 0) * 16 * 16 + 4 * R * 16) * kCin + 8 * (threadIdx.x & 63);"),
        ("                xr[R][col][c] = *reinterpret_cast<const uint4 *>(src + col * kCin + 32 * c);",
         "                xr[R][col][c] = *reinterpret_cast<const uint4 *>(src + (col * NC + c) * 512);"),
        ("        uint16_t *yr = y + (live ? b : 0) * 16 * kCout + 4 * g;",
         "        uint16_t *yr = y + (live ? tile : 0) * 16 * 16 * kCout + 4 * lane;"),
        ("                            *reinterpret_cast<uint2 *>(yr + (4 * r + col) * kCout + 16 * (2 * oh + o)) =",
         "                            *reinterpret_cast<uint2 *>(yr + ((4 * r + col) * 4 + 2 * oh + o) * 256) ="),
    ],
    "fwd_coalesced_loads": None,
    "fwd_coalesced_stores": None,
    # wgrad: the next step's DMAs issued between the two k-steps' MFMAs instead of before them
    "wgrad_dma_mid": [
        ("    auto compute = [&](int buf) {\n        const uint16_t *img = lds + buf * kBuf;\n#pragma unroll\n"
         "        for (int ks = 0; ks < kKSteps; ks++) {",
         "    auto compute = [&](int buf, int ks0, int ks1) {\n        const uint16_t *img = lds + buf * kBuf;\n#pragma unroll\n"
         "        for (int ks = ks0; ks < ks1; ks++) {"),
        ("        stage(i + kRing - 1, (buf + kRing - 1) % kRing);          // buffer of step i - 1\n"
         "        compute(buf);\n",
         "        compute(buf, 0, 1);\n        __builtin_amdgcn_sched_barrier(0);\n"
         "        stage(i + kRing - 1, (buf + kRing - 1) % kRing);          // buffer of step i - 1\n"
         "        __builtin_amdgcn_sched_barrier(0);\n        compute(buf, 1, 2);\n")],
    # wgrad: the DMA ring runs, no MFMA work
    "wgrad_nocompute": [("        stage(i + kRing - 1, (buf + kRing - 1) % kRing);          // buffer of step i - 1\n"
                         "        compute(buf);\n",
                         "        stage(i + kRing - 1, (buf + kRing - 1) % kRing);          // buffer of step i - 1\n")],
    # wgrad: MFMA work and barriers over the prologue's buffers, no DMA inside the loop
    "wgrad_nodma": [("        stage(i + kRing - 1, (buf + kRing - 1) % kRing);          // buffer of step i - 1\n", "")],
}


VARIANTS["fwd_coalesced_loads"] = VARIANTS["fwd_coalesced"][:2]
VARIANTS["fwd_coalesced_stores"] = VARIANTS["fwd_coalesced"][2:]


def build(name):
    s = open(SRC).read()
    for old, new in VARIANTS[name]:
        if old not in s:
            raise SystemExit("variant %s: pattern not found" % name)
        s = s.replace(old, new)
    os.makedirs(os.path.join(ROOT, "build", "var"), exist_ok=True)
    path = os.path.join(ROOT, "build", "var", "conv_%s.hip" % name)
    open(path, "w").write(s)
    subprocess.check_call(["bash", os.path.join(ROOT, "tools", "build_variant.sh"), path, "r48_conv",
                           os.path.join(ROOT, "build", "lib_conv_%s.so" % name)], cwd=ROOT)


if __name__ == "__main__":
    for n in sys.argv[1:] or list(VARIANTS):
        build(n)
        print("built", n)
