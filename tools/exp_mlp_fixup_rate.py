"""GPU experiment: how often k_mlp_train's exact-decision fix-up runs on real config-3 data. Needs a
counting build (tools/build_variant.sh of a k_mlp_train whose record carries counters at 2503..2508:
tiles, fix-up tiles, fix-up row blocks, edge units, near rows, mask flips). One warm-up update and
one measured update of bench.a3c_config3(net='mlp') per loss mode; the trainer's call is routed
through the counting library.   python tools/exp_mlp_fixup_rate.py lib_count.so"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd import _lib  # noqa: E402

_lib.LIB_PATH, _lib._lib = sys.argv[1], None
import bench  # noqa: E402
from rein48_amd.a3c import fused  # noqa: E402

stats = []


def counting_grad(net, boards, actions, targets, wn, cm=None, counts=None, beta=0.001, exponents=False,
                  n_boards=None, w=None, workspace=None):
    L = _lib.load()
    dev = boards.device
    rows = boards.numel() // 16
    w = fused.pack_mlp(net) if w is None else w
    ws = torch.empty(int(L.r48_mlp_train_workspace_floats(rows)), dtype=torch.float32, device=dev)
    out = torch.zeros(2512, dtype=torch.float32, device=dev)
    p = lambda t: C.c_void_p(0 if t is None else t.data_ptr())
    rc = L.r48_mlp_train_grad(p(boards), rows, int(n_boards or rows), p(actions), p(targets), p(wn), p(cm), p(counts),
                              float(beta), _lib.FEAT_EXPONENTS if exponents else _lib.FEAT_VALUES, p(w), p(ws), p(out),
                              C.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
    assert rc == 0
    c = out[2503:2509].tolist()
    stats.append(dict(rows=rows, tiles=c[0], fix_tiles=c[1], fix_rowblocks=c[2], edge_units=c[3], near_rows=c[4],
                      flips=c[5]))
    return out[:2501], out[2501], out[2502]


fused.mlp_train_grad = counting_grad
d = torch.device("cuda", 0)
for mode, feat in (("reference", "values"), ("textbook", "exponents")):
    stats.clear()
    bench.a3c_config3(d, 0x20485EED, 1 << 20, updates=1, warmup=1, mode=mode, features=feat, net="mlp", bf16=False)
    for s in stats:
        print(mode, {k: (int(v) if isinstance(v, float) else v) for k, v in s.items()},
              "fix-up tiles %.3f  row blocks per fix-up tile %.2f" % (s["fix_tiles"] / s["tiles"], s["fix_rowblocks"] / max(s["fix_tiles"], 1)),
              flush=True)
