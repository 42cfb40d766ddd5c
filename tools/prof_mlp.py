"""Profile target: A3C with the reference MLP (fused rollout + fused update) at 2^20 boards x 100
steps, `iters` train steps after one warm-up step.  rocprofv3 --kernel-trace --stats -- python3 tools/prof_mlp.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd.a3c import A3CConfig, A3CTrainer  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "textbook"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 2
tr = A3CTrainer(A3CConfig(n_boards=1 << 20, max_steps=100, mode=mode, net="mlp", bf16=False,
                          features="values" if mode == "reference" else "exponents", seed=1), device="cuda:0")
for _ in range(iters + 1):
    tr.train_step()
torch.cuda.synchronize()
print("done", mode, iters)
