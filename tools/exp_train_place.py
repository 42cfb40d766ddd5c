"""GPU experiment: does k_cnn_train's speed depend on where its per-call tensors sit? One library,
one process: for each trial a dummy allocation of a different size shifts the caching allocator
before the net, the packed weights and the workspace are created; prints their addresses (mod 2 MiB)
and the kernel time (SEG instance, as the trainer runs it). Motivated by the A/A control of
profiles/r05/a3c/train/fence_mask_vmem_ab.txt (session 9).

    python tools/exp_train_place.py [rows]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd import _lib  # noqa: E402
from rein48_amd.a3c.fused import cnn_train_grad, pack_cnn_train  # noqa: E402
from rein48_amd.a3c.nets import ActorCriticCNN  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
dev = torch.device("cuda:0")
n = 1 << 20
g = torch.Generator(device="cpu").manual_seed(0)
boards = torch.randint(0, 12, (rows, 16), generator=g, dtype=torch.int8).to(dev)
actions = torch.randint(0, 4, (rows,), generator=g, dtype=torch.int8).to(dev)
targets = torch.randn(rows, generator=g).to(dev)
T = rows // n
L = torch.randint(1, T + 1, (n,), generator=g, dtype=torch.int32)
segf = torch.zeros((n, 4), dtype=torch.float32)
segf[:, 0] = 1.0 / rows
segf[:, 2] = L.view(torch.float32)
seg = segf.to(dev)
lib = _lib.load()
MB = 1 << 20


def trial(pad_bytes):
    pad = torch.empty(max(pad_bytes, 1), dtype=torch.uint8, device=dev)
    torch.manual_seed(0)
    net = ActorCriticCNN(dtype=torch.bfloat16).to(dev)
    packed = pack_cnn_train(net)
    ws = torch.empty(lib.r48_cnn_train_workspace_floats(), dtype=torch.float32, device=dev)
    run = lambda: cnn_train_grad(net, boards, actions, targets, None, None, None, beta=0.01, exponents=True,
                                 n_boards=n, packed=packed, workspace=ws, seg=seg)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    addr = lambda t: t.data_ptr() % (2 * MB)
    print("pad %9d  wfrag %%2M %7d  bias %%2M %7d  ws %%2M %7d  ws %%64K %5d  %.2f ms per 1e8 rows" % (
        pad_bytes, addr(packed[0]), addr(packed[1]), addr(ws), ws.data_ptr() % 65536, ms * 1e8 / rows), flush=True)
    del pad, net, packed, ws


print("# warm-up trials (pad 0)", flush=True)
t_w = time.time()
while time.time() - t_w < 2.0:   # warm the GPU (exp_train's first-library penalty)
    trial(0)
print("# placement trials", flush=True)
for rnd in range(2):
    for pad in (0, 4096, 65536, MB, MB + 4096, 3 * MB, 5 * MB + 12288, 17 * MB):
        trial(pad)
