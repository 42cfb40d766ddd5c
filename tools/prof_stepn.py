"""Profiling driver: k_step_n at 2^20 boards (random policy + auto-reset), `reps` calls of K steps
after a settle period, for rocprofv3 --kernel-trace --stats and --pmc passes.
usage: python tools/prof_stepn.py [K] [reps] [boards]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd import VecGame  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
n = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 20
env = VecGame(n, device="cuda:0", seed=1)
env.fill_random(7)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:       # settle with the same K, so every dispatch is alike
    env.step_n(K, auto_reset=True)
    torch.cuda.synchronize()
for _ in range(reps):
    env.step_n(K, auto_reset=True)
torch.cuda.synchronize()
print("done", K, reps, n)
