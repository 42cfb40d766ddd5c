"""GPU probe: why the first timed region of a bench process is slower than its repeats. Runs
bench.timed_steps' region shape six times in one process (each after bench's own warm-up, settle and
untimed pass) and prints per region: host time from t0 until r48_env_step_n returns (the launch
path), wall (t0 -> t1), and the HIP-event device time.

    python tools/exp_first_region.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rein48_amd import VecGame  # noqa: E402

dev = torch.device("cuda", 0)
env = VecGame(1 << 20, device=dev, seed=0x20485EED)
env.fill_random(7)
s = torch.cuda.current_stream(dev)
for region in range(6):
    for c in bench.chunks(5, 20):
        env.step_n(c, auto_reset=True)
    torch.cuda.synchronize(dev)
    t_w = time.perf_counter()
    while time.perf_counter() - t_w < bench.SETTLE_S:
        env.step_n(20, auto_reset=True)
        torch.cuda.synchronize(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    env.step_n(20, auto_reset=True)
    b.record(s)
    b.synchronize()
    torch.cuda.synchronize(dev)
    a.record(s)
    t0 = bench._now()
    env.step_n(20, auto_reset=True)
    t_ret = bench._now()
    b.record(s)
    b.synchronize()
    t1 = bench._now()
    torch.cuda.synchronize(dev)
    print("region %d: launch path %.1f us, wall %.1f us, device %.1f us -> %.1f G"
          % (region, (t_ret - t0) * 1e6, (t1 - t0) * 1e6, a.elapsed_time(b) * 1e3, (1 << 20) * 20 / (t1 - t0) / 1e9),
          flush=True)
