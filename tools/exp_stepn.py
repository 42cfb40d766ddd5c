"""GPU experiment: r48_env_step_n (k_step_n, boards in VGPRs for K steps, one launch per call) and
r48_env_step (k_step, one launch per step, boards through HBM) across board counts and K.

Per configuration: device time per call from HIP events (median of reps), and the wall time of
the bench's timed region (synchronize, t0, one call, synchronize, t1; median). Run one library
build per process: R48_LIB=<path to a variant .so> python tools/exp_stepn.py [tag]."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd import VecGame  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("R48_LIB", "shipped")
dev = "cuda:0"
s = torch.cuda.current_stream()


def med(x):
    return sorted(x)[len(x) // 2]


def settle(env, secs=0.3):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < secs:
        env.step_n(100, auto_reset=True)
        torch.cuda.synchronize()


for n in (1 << 20, 1 << 22, 1 << 26):
    env = VecGame(n, device=dev, seed=1)
    env.fill_random(7)
    settle(env)
    for K in (20, 100, 1000):
        reps = 20 if n * K <= (1 << 30) else 5
        dev_ms, wall_ms = [], []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            a.record(s)
            env.step_n(K, auto_reset=True)
            b.record(s)
            torch.cuda.synchronize()
            wall_ms.append((time.perf_counter() - t0) * 1e3)
            dev_ms.append(a.elapsed_time(b))
        d, w = med(dev_ms), med(wall_ms)
        print("%s n=2^%d K=%4d  step_n: device %.4f ms (%.3f us/step, %.1f G/s)  wall %.4f ms (%.1f G/s, spread %.1f%%)"
              % (tag, n.bit_length() - 1, K, d, d * 1e3 / K, n * K / d / 1e6, w, n * K / w / 1e6,
                 100 * (max(wall_ms) - min(wall_ms)) / w), flush=True)
    # single-step kernel, back-to-back launches
    reps = 200 if n <= (1 << 22) else 20
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record(s)
    for _ in range(reps):
        env.step(None, auto_reset=True)
    b.record(s)
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / reps
    print("%s n=2^%d k_step eager: %.3f us/step (%.1f G/s, %.0f GB/s of 34 B/board-step)"
          % (tag, n.bit_length() - 1, us, n / us / 1e3, n * 34 / us / 1e3), flush=True)
    del env
    torch.cuda.empty_cache()
