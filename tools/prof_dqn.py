"""Probe: kernel breakdown of one config-5 DQN update (batch 2^16) under rocprofv3."""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from rein48_amd.dqn import DQNConfig, DQNTrainer  # noqa: E402

if __name__ == "__main__":
    cfg = DQNConfig(n_boards=1 << 18, replay_capacity=1 << 22, batch=1 << 16, learn_start=1, seed=0)
    tr = DQNTrainer(cfg, device="cuda:0")
    for _ in range(3):
        tr.train_step()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(5):
        tr.update()
    ev[1].record()
    torch.cuda.synchronize()
    print("update ms", ev[0].elapsed_time(ev[1]) / 5, flush=True)
