"""GPU experiment: A/B of k_step_n builds (the product library and variant libraries from
tools/build_variant.sh) at 2^20 boards, K = 20 (the driver's region) and K = 1000: median device
time per call (HIP events) and median wall time of the bench's region shape, libraries
interleaved over two rounds, with a bit-level digest of the boards after a fixed call sequence.

    python tools/exp_stepn_ab.py lib.so [lib.so ...]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd import VecGame, _lib  # noqa: E402

libs = sys.argv[1:] or [_lib.LIB_PATH]
dev = "cuda:0"
s = torch.cuda.current_stream()
n = 1 << 20


def med(x):
    return sorted(x)[len(x) // 2]


for rnd in range(2):
    for path in libs:
        _lib.LIB_PATH, _lib._lib = path, None
        env = VecGame(n, device=dev, seed=1)
        env.fill_random(7)
        env.step_n(1000, auto_reset=True)
        digest = int((env.boards.view(torch.int32).long() * 2654435761).sum()) & 0xFFFFFFFF
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.3:
            env.step_n(100, auto_reset=True)
            torch.cuda.synchronize()
        line = []
        for K, reps in ((20, 60), (1000, 10)):
            dev_ms, wall_ms = [], []
            for _ in range(reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                a.record(s)
                env.step_n(K, auto_reset=True)
                b.record(s)
                torch.cuda.synchronize()
                wall_ms.append((time.perf_counter() - t1) * 1e3)
                dev_ms.append(a.elapsed_time(b))
            d, w = med(dev_ms), med(wall_ms)
            line.append("K=%d dev %.2f us (%.3f us/step) wall %.2f us = %.1f G" % (K, d * 1e3, d * 1e3 / K, w * 1e3,
                                                                                 n * K / w / 1e6))
        print("%-28s %s | digest %08x" % (os.path.basename(path), " | ".join(line), digest), flush=True)
        del env
        torch.cuda.empty_cache()
