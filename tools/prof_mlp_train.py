"""Profile target: the fused MLP update kernel alone (r48_mlp_train_grad) on 2^24 synthetic rows
(textbook loss, exponent features), `iters` calls after one warm-up; R48_LIB selects the build.

    rocprofv3 --pmc ... -- python3 tools/prof_mlp_train.py [rows] [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd import _lib  # noqa: E402
from rein48_amd.a3c.fused import mlp_train_grad, pack_mlp  # noqa: E402
from rein48_amd.a3c.nets import ActorCriticMLP  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(0)
boards = torch.randint(0, 12, (rows, 16), generator=g, dtype=torch.int8).to(dev)
actions = torch.randint(0, 4, (rows,), generator=g, dtype=torch.int8).to(dev)
targets = torch.randn(rows, generator=g).to(dev)
wn = torch.full((rows,), 1.0 / rows, device=dev)
torch.manual_seed(0)
net = ActorCriticMLP().to(dev)
w = pack_mlp(net)
ws = torch.empty(int(_lib.load().r48_mlp_train_workspace_floats(rows)), dtype=torch.float32, device=dev)
for _ in range(iters + 1):
    mlp_train_grad(net, boards, actions, targets, wn, beta=0.01, exponents=True, n_boards=1 << 20, w=w, workspace=ws)
torch.cuda.synchronize()
print("ok")
