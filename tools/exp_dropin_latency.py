"""GPU experiment: per-call latency of the drop-in Game.step (one board, GPU kernels, host spawn
draws from the global `random`) against the CPU restatement of the reference (oracle/game_port,
the cpu_baseline's per-process engine) on the same host core, for 4x4 and 8x8 boards.
usage: python tools/exp_dropin_latency.py [steps]"""
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.game_port import PortGame, random_action  # noqa: E402
from rein48_amd.game import Game  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3000


def run(make, n):
    random.seed(1)
    g = make()
    done_steps, t0 = 0, time.perf_counter()
    while done_steps < n:
        _, _, d = g.step(random_action())
        done_steps += 1
        if d:
            g = make()
    return (time.perf_counter() - t0) / n * 1e6


for size in (4, 8):
    run(lambda: Game(size), 200)                      # warm-up (library load, allocator)
    gpu = run(lambda: Game(size), steps)
    cpu = run(lambda: PortGame(size), steps)
    print("size %d: drop-in Game.step %.1f us/step (GPU kernels + host draws), CPU port %.1f us/step, "
          "ratio %.1fx" % (size, gpu, cpu, gpu / cpu), flush=True)
