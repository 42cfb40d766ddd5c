"""GPU experiment: times r48_cnn_train_grad (k_cnn_train + its two reduction launches) over `rows`
synthetic states for the product library, or for variant libraries given on the command line
(tools/build_variant.sh), with a bit-level digest of the gradient.

    python tools/exp_train.py [rows] [lib.so ...]
"""
import os
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from rein48_amd import _lib  # noqa: E402
from rein48_amd.a3c.fused import cnn_train_grad, pack_cnn_train  # noqa: E402
from rein48_amd.a3c.nets import ActorCriticCNN  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
dev = torch.device("cuda:0")
n = 1 << 20
libs = sys.argv[2:] or [_lib.LIB_PATH]
g = torch.Generator(device="cpu").manual_seed(0)
boards = torch.randint(0, 12, (rows, 16), generator=g, dtype=torch.int8).to(dev)
actions = torch.randint(0, 4, (rows,), generator=g, dtype=torch.int8).to(dev)
targets = torch.randn(rows, generator=g).to(dev)
wn = torch.full((rows,), 1.0 / rows, device=dev)
# R48_EXP_SEG=1: the trainer's path instead -- per-board segment weights (r48_cnn_train_grad_seg,
# the k_cnn_train<MODE, SEG=true> instance): rows = T x n step-major, board b's segment length L in
# 1..T (synthetic), seg[b] = {w0, c0, L (int bits), 0}
SEG = os.environ.get("R48_EXP_SEG") == "1"
seg = None
if SEG:
    T = rows // n
    L = torch.randint(1, T + 1, (n,), generator=g, dtype=torch.int32)
    segf = torch.zeros((n, 4), dtype=torch.float32)
    segf[:, 0] = 1.0 / rows
    segf[:, 2] = L.view(torch.float32)
    seg = segf.to(dev)
    wn = None
for path in libs:
    _lib.LIB_PATH, _lib._lib = path, None
    torch.manual_seed(0)
    net = ActorCriticCNN(dtype=torch.bfloat16).to(dev)
    packed = pack_cnn_train(net)
    ws = torch.empty(_lib.load().r48_cnn_train_workspace_floats(), dtype=torch.float32, device=dev)
    run = lambda: cnn_train_grad(net, boards, actions, targets, wn, None, None, beta=0.01, exponents=True,
                                 n_boards=n, packed=packed, workspace=ws, seg=seg)
    out = run()
    torch.cuda.synchronize()
    grads = torch.cat([t.detach().float().reshape(-1) for t in out[0]])
    digest = int((grads.view(torch.int32).long() * 2654435761).sum()) & 0xFFFFFFFF   # bit-level fingerprint
    # the first library timed in a process ran ~3 % slow (order-balanced runs in
    # profiles/r05/a3c/train/fence_mask_vmem_ab.txt, session 8): warm the GPU for 2 s first
    if path == libs[0]:
        t_w = time.time()
        while time.time() - t_w < 2.0:
            run()
            torch.cuda.synchronize()
    for _ in range(2):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(("seg " if SEG else "") + "%-40s %8.2f ms per %d rows  (%.2f ms per 1e8)  grad digest %08x" % (os.path.basename(path), ms, rows,
                                                                               ms * 1e8 / rows, digest), flush=True)
