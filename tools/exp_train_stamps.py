"""GPU experiment: per-phase cycles of k_cnn_train from the stamped variant library
(tools/stamp_train.py): mean over waves of the cycles per tile spent in each phase.

    python tools/exp_train_stamps.py build/librein48_stamp.so [rows]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd import _lib  # noqa: E402
from rein48_amd.a3c.fused import cnn_train_grad, pack_cnn_train, GRAD_FLOATS  # noqa: E402
from rein48_amd.a3c.nets import ActorCriticCNN  # noqa: E402

_lib.LIB_PATH, _lib._lib = sys.argv[1], None
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 24
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(0)
boards = torch.randint(0, 12, (rows, 16), generator=g, dtype=torch.int8).to(dev)
actions = torch.randint(0, 4, (rows,), generator=g, dtype=torch.int8).to(dev)
targets = torch.randn(rows, generator=g).to(dev)
wn = torch.full((rows,), 1.0 / rows, device=dev)
torch.manual_seed(0)
net = ActorCriticCNN(dtype=torch.bfloat16).to(dev)
packed = pack_cnn_train(net)
L = _lib.load()
ws = torch.empty(L.r48_cnn_train_workspace_floats(), dtype=torch.float32, device=dev)
names = ["head", "conv2+heads", "loss", "dh2 phase", "-", "positions", "conv1"]
for rep in range(3):
    cnn_train_grad(net, boards, actions, targets, wn, None, None, beta=0.01, exponents=True, n_boards=1 << 20,
                   packed=packed, workspace=ws)
    torch.cuda.synchronize()
    n_rec = (ws.numel() // GRAD_FLOATS) - 32
    st = ws[:n_rec * GRAD_FLOATS].view(n_rec, GRAD_FLOATS)[:, :16].contiguous().view(torch.int64)[:, :7].double()
    tiles = (rows + 31) // 32 / n_rec
    per = st.mean(0) / tiles
    print("rep %d  cycles per tile: " % rep + "  ".join("%s %.0f" % (n, v) for n, v in zip(names, per.tolist()))
          + "  | total %.0f" % float(per.sum()), flush=True)
