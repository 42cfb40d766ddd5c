"""Probe: kernel breakdown of the config-5 DQN update (batch 2^16) under rocprofv3.

Three train steps (act + env step + store + update) warm up; then `n` updates run back to back
(HIP-event time printed). tools/dqn_breakdown.py splits the kernel trace at the last k_store (the
last env step's replay store) and sums the kernels of the updates after it.
    rocprofv3 --kernel-trace --stats -d <dir> -o dqn -- python3 tools/prof_dqn.py [n]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd.dqn import DQNConfig, DQNTrainer  # noqa: E402

if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    what = sys.argv[2] if len(sys.argv) > 2 else "update"     # "update" | "act" (2^21 boards, bench slice)
    boards = 1 << 21 if what == "act" else 1 << 18
    cfg = DQNConfig(n_boards=boards, replay_capacity=1 << 22, batch=1 << 16, learn_start=1, seed=0)
    tr = DQNTrainer(cfg, device="cuda:0")
    for _ in range(3):
        tr.train_step()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(n):
        tr.update() if what == "update" else tr.act()
    ev[1].record()
    torch.cuda.synchronize()
    print(what, "ms", ev[0].elapsed_time(ev[1]) / n, what + "s", n, flush=True)
