"""GPU experiment: device time of the config-5 update convolutions (r48_conv3x3 forward at 64 and 32
input channels, r48_conv3x3_wgrad at 64 and 32) for the product library and variant libraries
(tools/build_variant.sh), at `boards` boards, with a bit-level digest of every output.

    python tools/exp_conv.py [boards] [lib.so ...]
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
x64 = torch.randn(B, 16, 64, generator=g).to(dev, torch.bfloat16)
x32 = torch.randn(B, 16, 32, generator=g).to(dev, torch.bfloat16)
dy = torch.randn(B, 16, 64, generator=g).to(dev, torch.bfloat16)
w64 = torch.randn(64, 64, 3, 3, generator=g).to(dev) * 0.05
w32 = torch.randn(64, 32, 3, 3, generator=g).to(dev) * 0.05
bias = torch.randn(64, generator=g).to(dev)
f64, f32 = C.pack_conv(w64, 64), C.pack_conv(w32, 32)


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
io = {"fwd64": B * 16 * (64 + 64) * 2, "fwd32": B * 16 * (32 + 64) * 2,
      "wgrad64": B * 16 * (64 + 64) * 2, "wgrad32": B * 16 * (64 + 32) * 2}
for path in libs:
    _lib.LIB_PATH, _lib._lib = path, None
    C._WS.clear()
    runs = {"fwd64": lambda: C.conv3x3(x64, f64, bias), "fwd32": lambda: C.conv3x3(x32, f32, bias),
            "wgrad64": lambda: C.conv3x3_wgrad(dy, x64), "wgrad32": lambda: C.conv3x3_wgrad(dy, x32)}
    line = []
    for k, fn in runs.items():
        out = fn()
        torch.cuda.synchronize()
        us = timed(fn)
        line.append("%s %7.1f us %5.2f TB/s %08x" % (k, us, io[k] / us / 1e6, digest(out)))
    print("%-40s B=%d  %s" % (os.path.basename(path), B, " | ".join(line)), flush=True)
