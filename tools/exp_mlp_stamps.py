"""GPU experiment: per-phase cycles of k_mlp_train from the stamped variant library
(tools/stamp_mlp.py): mean over waves of the cycles per 64-row tile spent in each phase.

    python tools/exp_mlp_stamps.py build/lib_mlp_stamp.so [rows]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd import _lib  # noqa: E402
from rein48_amd.a3c.fused import mlp_train_grad, pack_mlp  # noqa: E402
from rein48_amd.a3c.nets import ActorCriticMLP  # noqa: E402

_lib.LIB_PATH, _lib._lib = sys.argv[1], None
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 100 << 20
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(0)
boards = torch.randint(0, 12, (rows, 16), generator=g, dtype=torch.int8).to(dev)
actions = torch.randint(0, 4, (rows,), generator=g, dtype=torch.int8).to(dev)
targets = torch.randn(rows, generator=g).to(dev)
wn = torch.full((rows,), 1.0 / rows, device=dev)
torch.manual_seed(0)
net = ActorCriticMLP().to(dev)
w = pack_mlp(net)
L = _lib.load()
ws = torch.empty(int(L.r48_mlp_train_workspace_floats()), dtype=torch.float32, device=dev)
names = ["inputs", "forward", "-", "loss", "stash+fix", "phase 2"]
n_rec = 1024 * 4
for rep in range(3):
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    mlp_train_grad(net, boards, actions, targets, wn, beta=0.01, exponents=True, n_boards=1 << 20, w=w, workspace=ws)
    ev1.record()
    torch.cuda.synchronize()
    st = ws[:n_rec * 2504].view(n_rec, 2504)[:, :16].contiguous().view(torch.int64)[:, :6].double()
    tiles = (rows + 63) // 64 / n_rec
    per = st.mean(0) / tiles
    print("rep %d %.2f ms  cycles per tile: " % (rep, ev0.elapsed_time(ev1)) +
          "  ".join("%s %.0f" % (n, v) for n, v in zip(names, per.tolist())) + "  | total %.0f" % float(per.sum()),
          flush=True)
