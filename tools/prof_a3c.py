"""Profile target: A3C (CNN, bf16) rollout + update at 2^20 boards, short segments."""
import sys
import torch
sys.path.insert(0, ".")
from rein48_amd.a3c import A3CConfig, A3CTrainer

net = sys.argv[1] if len(sys.argv) > 1 else "cnn"
cfg = A3CConfig(n_boards=1 << 20, max_steps=10, mode="textbook", net=net, bf16=(net == "cnn"),
                features="exponents", seed=1, update_chunk=10)
tr = A3CTrainer(cfg, device="cuda:0")
for _ in range(3):
    tr.train_step()
torch.cuda.synchronize()
print("ok")
