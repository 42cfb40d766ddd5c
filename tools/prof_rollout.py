"""Profile target: the config-3 rollout megakernel alone (2^20 boards x 100 steps, CNN bf16,
textbook mode), `iters` rollouts after one warm-up.

    rocprofv3 --pmc ... -- python3 tools/prof_rollout.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd.a3c import A3CConfig, A3CTrainer  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3
cfg = A3CConfig(n_boards=1 << 20, max_steps=100, mode="textbook", net="cnn", bf16=True, features="exponents", seed=1)
tr = A3CTrainer(cfg, device="cuda:0")
for _ in range(iters + 1):
    tr.rollout()
torch.cuda.synchronize()
print("ok")
