"""Probe: PyTorch-ROCm throughput of a ResNet-10 Q-network on 4x4 boards (config 5 sizing).

Variants: nn.Conv2d (MIOpen) NCHW / channels_last in bf16, and each 3x3 conv (pad 1) on the
4x4 grid as ONE structured dense GEMM [B, 16C] x [16C, 16C] (hipBLASLt). Prints ms and useful
TFLOP/s (valid taps only) for the inference forward at 2^21 boards and fwd+bwd at 2^16.
"""
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

DEV = "cuda"
C = 64
IN = 18


def useful_flops_per_board(c=C):
    taps = 100                     # valid (pos, tap) pairs of a 3x3 pad-1 conv on 4x4
    return 2 * taps * (IN * c + 8 * c * c) + 2 * 16 * c * 4


class ConvNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.stem = nn.Conv2d(IN, C, 3, padding=1)
        self.convs = nn.ModuleList([nn.Conv2d(C, C, 3, padding=1) for _ in range(8)])
        self.head = nn.Linear(16 * C, 4)

    def forward(self, x):
        h = F.relu(self.stem(x))
        for k in range(0, 8, 2):
            y = F.relu(self.convs[k](h))
            h = F.relu(self.convs[k + 1](y) + h)
        return self.head(h.flatten(1))


def dense_of(conv):
    """[16C_out, 16C_in] matrix of a 3x3 pad-1 conv on a 4x4 grid (position-major, channel-minor)."""
    w = conv.weight                  # [co, ci, 3, 3]
    co, ci = w.shape[:2]
    D = torch.zeros(16 * co, 16 * ci, device=w.device, dtype=w.dtype)
    for p in range(16):
        r, c = divmod(p, 4)
        for dr in (-1, 0, 1):
            for dc in (-1, 0, 1):
                rr, cc = r + dr, c + dc
                if 0 <= rr < 4 and 0 <= cc < 4:
                    q = rr * 4 + cc
                    D[p * co:(p + 1) * co, q * ci:(q + 1) * ci] = w[:, :, dr + 1, dc + 1]
    return D


def dense_forward(net, x_pm, mats):
    """x_pm [B, 16*IN] position-major."""
    stem, convs = mats
    h = F.relu(F.linear(x_pm, stem[0], stem[1]))
    for k in range(0, 8, 2):
        y = F.relu(F.linear(h, convs[k][0], convs[k][1]))
        h = F.relu(F.linear(y, convs[k + 1][0], convs[k + 1][1]) + h)
    return h


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    torch.manual_seed(0)
    net = ConvNet().to(DEV).to(torch.bfloat16)
    fl = useful_flops_per_board()
    print("useful MFLOP/board fwd: %.2f" % (fl / 1e6))
    B = 1 << 21
    chunk = 1 << 18
    x = torch.randn(B, IN, 4, 4, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        for name, fmt in (("conv NCHW", torch.contiguous_format), ("conv channels_last", torch.channels_last)):
            n2 = net.to(memory_format=fmt)
            xx = x.contiguous(memory_format=fmt)
            for ck in (1 << 16, 1 << 14):
                try:
                    ms = timeit(lambda: [n2(xx[i:i + ck]) for i in range(0, B, ck)], reps=3)
                    print("%-22s fwd 2^21 (chunks 2^%d): %8.2f ms  %7.1f TFLOP/s useful"
                          % (name, ck.bit_length() - 1, ms, fl * B / ms / 1e9), flush=True)
                    break
                except RuntimeError as e:
                    print("%-22s chunk 2^%d failed: %s" % (name, ck.bit_length() - 1, str(e)[:80]), flush=True)
        mats = ((dense_of(net.stem), net.stem.bias.repeat(16)),
                [(dense_of(c), c.bias.repeat(16)) for c in net.convs])
        xp = torch.randn(B, 16 * IN, device=DEV, dtype=torch.bfloat16)
        ms = timeit(lambda: [dense_forward(net, xp[i:i + chunk], mats) for i in range(0, B, chunk)], reps=3)
        print("%-22s fwd 2^21: %8.2f ms  %7.1f TFLOP/s useful (%.1f dense)" %
              ("structured dense GEMM", ms, fl * B / ms / 1e9, (2 * 16 * 16 * (IN * C + 8 * C * C)) * B / ms / 1e9))
        a = torch.randn(chunk, 1024, device=DEV, dtype=torch.bfloat16)
        w = torch.randn(1024, 1024, device=DEV, dtype=torch.bfloat16)
        ms = timeit(lambda: a @ w.t(), reps=20)
        print("plain GEMM %d x 1024 x 1024 bf16: %.3f ms  %.1f TFLOP/s" % (chunk, ms, 2 * chunk * 1024 * 1024 / ms / 1e9))
    # training step shape
    Bt = 1 << 16
    xt = torch.randn(Bt, IN, 4, 4, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    n2 = net.to(memory_format=torch.channels_last)

    def fb():
        n2.zero_grad(set_to_none=True)
        n2(xt).float().square().mean().backward()
    try:
        ms = timeit(fb, reps=5)
    except RuntimeError as e:
        print("fwd+bwd failed", str(e)[:80])
        return
    print("conv channels_last fwd+bwd 2^16: %.2f ms  %.1f TFLOP/s useful (3x fwd)" % (ms, 3 * fl * Bt / ms / 1e9))


if __name__ == "__main__":
    main()
