"""Profiling driver: r48_cnn_train_grad over `rows` synthetic states, `reps` times (for rocprofv3
--kernel-trace / --pmc runs of k_cnn_train alone).

    python tools/prof_train.py [rows] [reps]
"""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from rein48_amd import _lib  # noqa: E402
from rein48_amd.a3c.fused import cnn_train_grad, pack_cnn_train  # noqa: E402
from rein48_amd.a3c.nets import ActorCriticCNN  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(0)
boards = torch.randint(0, 12, (rows, 16), generator=g, dtype=torch.int8).to(dev)
actions = torch.randint(0, 4, (rows,), generator=g, dtype=torch.int8).to(dev)
targets = torch.randn(rows, generator=g).to(dev)
wn = torch.full((rows,), 1.0 / rows, device=dev)
torch.manual_seed(0)
net = ActorCriticCNN(dtype=torch.bfloat16).to(dev)
packed = pack_cnn_train(net)
ws = torch.empty(_lib.load().r48_cnn_train_workspace_floats(), dtype=torch.float32, device=dev)
for _ in range(reps):
    cnn_train_grad(net, boards, actions, targets, wn, None, None, beta=0.01, exponents=True, n_boards=1 << 20,
                   packed=packed, workspace=ws)
torch.cuda.synchronize()
print("ok", rows, reps)
