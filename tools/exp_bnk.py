"""GPU experiment: r48_bn_forward (with ReLU mask) and r48_bn_backward (mask path) at the config-5
update's shape (bf16 [2^20 rows, 64]) for the product library and variant libraries, inputs rotated
over three copies (HBM rates, as inside an update). Prints device us per call.
    python tools/exp_bnk.py [lib.so ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd import _lib  # noqa: E402
from rein48_amd._lib import check, ptr  # noqa: E402

rows, C, NR = 1 << 20, 64, 3
dev = torch.device("cuda:0")
xs = [torch.randn(rows, C, device=dev).to(torch.bfloat16) for _ in range(NR)]
ds = [torch.randn(rows, C, device=dev).to(torch.bfloat16) for _ in range(NR)]
gamma, beta = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
save = torch.empty(2 * C, device=dev)
ys = [torch.empty_like(xs[0]) for _ in range(NR)]
ms = [torch.empty(rows, 8, dtype=torch.uint8, device=dev) for _ in range(NR)]
dx, dres = torch.empty_like(xs[0]), torch.empty_like(xs[0])
dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
s = torch.cuda.current_stream().cuda_stream
libs = sys.argv[1:] or [_lib.LIB_PATH]


def timed(fn, reps=30):
    fn(0)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(reps):
        fn(i + 1)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for path in libs:
    _lib.LIB_PATH, _lib._lib = path, None
    L = _lib.load()
    ws = torch.empty(L.r48_bn_workspace_floats(rows, C), device=dev)
    fwd = lambda i, res: check(L.r48_bn_forward(ptr(xs[i % NR]), ptr(xs[(i + 1) % NR]) if res else None, rows, C,  # noqa
                                                ptr(gamma), ptr(beta), ptr(rm), ptr(rv), 0.1, 1e-5, 1, ptr(save),
                                                ptr(ws), ptr(ys[i % NR]), ptr(ms[i % NR]), s))
    bwd = lambda i, res: check(L.r48_bn_backward(ptr(ds[i % NR]), None, ptr(ms[i % NR]), ptr(xs[i % NR]), rows, C,  # noqa
                                                 ptr(gamma), ptr(save), 1, ptr(ws), ptr(dx), ptr(dres) if res else None,
                                                 ptr(dg), ptr(db), s))
    out = []
    for name, fn in (("fwd", lambda i: fwd(i, False)), ("fwd+res", lambda i: fwd(i, True)),
                     ("bwd", lambda i: bwd(i, False)), ("bwd+dres", lambda i: bwd(i, True))):
        out.append("%s %6.1f us" % (name, timed(fn)))
    print("%-36s %s" % (os.path.basename(path), " | ".join(out)), flush=True)
