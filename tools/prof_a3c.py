"""Profile target: A3C config 3 (2^20 boards, CNN bf16, fused policy and update, 100-step
segments): `iters` train steps after one warm-up step.

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_a3c -- python tools/prof_a3c.py [iters] [mode]
mode "textbook" (exponent features, the default) or "reference" (raw tile values, the reference's
broadcast actor loss).
"""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from rein48_amd.a3c import A3CConfig, A3CTrainer  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2
mode = sys.argv[2] if len(sys.argv) > 2 else "textbook"
cfg = A3CConfig(n_boards=1 << 20, max_steps=100, mode=mode, net="cnn", bf16=True,
                features="exponents" if mode == "textbook" else "values", seed=1, update_chunk=10)
tr = A3CTrainer(cfg, device="cuda:0")
tr.train_step()
for _ in range(iters):
    tr.train_step()
torch.cuda.synchronize()
print("ok")
