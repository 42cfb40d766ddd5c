"""GPU experiment: device time of the config-5 update convolutions (r48_conv3x3 forward at 64 and 32
input channels, with the BN statistics epilogue (fwd64s), the data gradient with the BN-backward
reduction epilogue with and without the residual add (dg64bn, add64bn), r48_conv3x3_wgrad at 64 and
32) for the product library and variant libraries
(tools/build_variant.sh), at `boards` boards, with a bit-level digest of every output.

    python tools/exp_conv.py [boards] [lib.so ...]      (CASES=a,b: only those cases)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd import _lib  # noqa: E402
from rein48_amd.dqn import conv as C  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 16
libs = sys.argv[2:] or [_lib.LIB_PATH]
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(0)
# three copies of every input, used in rotation: successive calls read 3 x the Infinity Cache's
# 256 MiB apart at 64K boards (HBM rates, as inside an update), not a cache-resident tensor
NR = 3
x64s = [torch.randn(B, 16, 64, generator=g).to(dev, torch.bfloat16) for _ in range(NR)]
x32s = [torch.randn(B, 16, 32, generator=g).to(dev, torch.bfloat16) for _ in range(NR)]
dys = [torch.randn(B, 16, 64, generator=g).to(dev, torch.bfloat16) for _ in range(NR)]
x64, x32, dy = x64s[0], x32s[0], dys[0]
_rot = [0]


def rot(lst):
    _rot[0] += 1
    return lst[_rot[0] % NR]


w64 = torch.randn(64, 64, 3, 3, generator=g).to(dev) * 0.05
w32 = torch.randn(64, 32, 3, 3, generator=g).to(dev) * 0.05
bias = torch.randn(64, generator=g).to(dev)
f64, f32 = C.pack_conv(w64, 64), C.pack_conv(w32, 32)
masks = [torch.randint(0, 256, (B * 16, 8), generator=g, dtype=torch.uint8).to(dev) for _ in range(NR)]
save = torch.cat([torch.randn(64, generator=g), torch.rand(64, generator=g) + 0.5]).to(dev)
stats = None
part = None


def bn_grad(dy_, add_, bnx, mask, add_mask=None):
    out = torch.empty_like(dy_)
    C.check(_lib.load().r48_conv3x3_bn_grad(C.ptr(dy_), B, C.ptr(f64), C.ptr(add_), C.ptr(add_mask), C.ptr(out), C.ptr(bnx),
                                            C.ptr(mask), C.ptr(save), C.ptr(part), None, C._stream(dy_)))
    return out


coef = torch.cat([torch.rand(64, generator=g) + 0.5, torch.randn(64, generator=g) * 0.1]).to(dev)


def bn_in(x_, res_):
    """r48_conv3x3_bn_in: the previous BN + ReLU (+ residual) applied in the operand load."""
    y_ = torch.empty_like(x_)
    z_ = torch.empty_like(x_)
    m_ = torch.empty((B * 16, 8), dtype=torch.uint8, device=dev)
    C.check(_lib.load().r48_conv3x3_bn_in(C.ptr(x_), B, C.ptr(f64), C.ptr(bias), C.ptr(coef), C.ptr(res_), C.ptr(z_),
                                          C.ptr(m_), C.ptr(y_), C.ptr(stats), None, C._stream(x_)))
    return y_


def digest(t):
    v = t.detach().contiguous().view(-1)
    v = v.view(torch.int16).long() if v.dtype == torch.bfloat16 else v.view(torch.int32).long()
    return int((v * 2654435761).sum()) & 0xFFFFFFFF


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


# algorithmic HBM bytes: activations in + out (bf16); wgrad reads dy and x
io = {"fwd64": B * 16 * (64 + 64) * 2, "fwd32": B * 16 * (32 + 64) * 2, "add64": B * 16 * (64 + 64 + 64) * 2,
      "fwd64s": B * 16 * (64 + 64) * 2, "dg64bn": B * 16 * (3 * 64 * 2 + 8), "add64bn": B * 16 * (4 * 64 * 2 + 8), "addm64bn": B * 16 * (4 * 64 * 2 + 16),
      "in1": B * 16 * (3 * 64 * 2 + 8), "in2": B * 16 * (4 * 64 * 2 + 8),
      "wgrad64": B * 16 * (64 + 64) * 2, "wgrad32": B * 16 * (64 + 32) * 2}
for path in libs:
    _lib.LIB_PATH, _lib._lib = path, None
    C._WS.clear()
    stats = torch.empty(int(_lib.load().r48_conv_stats_floats()), dtype=torch.float32, device=dev)
    part = stats
    runs = {"fwd64": lambda: C.conv3x3(rot(x64s), f64, bias), "fwd32": lambda: C.conv3x3(rot(x32s), f32, bias),
            "add64": lambda: C.conv3x3(rot(x64s), f64, bias, add=rot(dys)),
            "fwd64s": lambda: C.conv3x3(rot(x64s), f64, bias, stats=stats),
            "in1": lambda: bn_in(rot(x64s), None), "in2": lambda: bn_in(rot(x64s), rot(dys)),
            "dg64bn": lambda: bn_grad(rot(dys), None, rot(x64s), rot(masks)),
            "add64bn": lambda: bn_grad(rot(dys), rot(x64s), rot(x64s), rot(masks)),
            "addm64bn": lambda: bn_grad(rot(dys), rot(x64s), rot(x64s), rot(masks), rot(masks)),
            "wgrad64": lambda: C.conv3x3_wgrad(rot(dys), rot(x64s)), "wgrad32": lambda: C.conv3x3_wgrad(rot(dys), rot(x32s))}
    only = os.environ.get("CASES")                     # e.g. CASES=wgrad64,wgrad32
    line = []
    for k, fn in runs.items():
        if only and k not in only.split(","):
            continue
        _rot[0] = -1
        out = fn()
        torch.cuda.synchronize()
        us = timed(fn)
        line.append("%s %7.1f us %5.2f TB/s %08x" % (k, us, io[k] / us / 1e6, digest(out)))
    print("%-40s B=%d  %s" % (os.path.basename(path), B, " | ".join(line)), flush=True)
