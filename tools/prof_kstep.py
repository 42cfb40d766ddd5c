"""Profiling driver: k_step (one launch per step, boards through HBM) at n boards, `launches`
launches after a settle period -- for the rocprofv3 FETCH_SIZE / WRITE_SIZE passes behind
bench.py's roofline.hbm entries.
usage: python tools/prof_kstep.py <boards> <launches>"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd import VecGame  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
launches = int(sys.argv[2]) if len(sys.argv) > 2 else 100
env = VecGame(n, device="cuda:0", seed=1)
env.fill_random(7)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.2:
    env.step(None, auto_reset=True)
    torch.cuda.synchronize()
for _ in range(launches):
    env.step(None, auto_reset=True)
torch.cuda.synchronize()
print("done", n, launches)
