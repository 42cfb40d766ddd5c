"""GPU experiment: fused CNN policy inference (r48_cnn_policy_forward with the action draw) over
`n` boards for each library given (default: the product library), ms per call and boards/s.

    python tools/exp_policy.py [n] [lib.so ...]
"""
import sys

import torch

sys.path.insert(0, ".")
from rein48_amd import _lib  # noqa: E402
from rein48_amd.a3c.fused import cnn_forward, pack_cnn  # noqa: E402
from rein48_amd.a3c.nets import ActorCriticCNN  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
libs = sys.argv[2:] or [_lib.LIB_PATH]
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(0)
boards = torch.randint(0, 12, (n, 16), generator=g, dtype=torch.int8).to(dev)
torch.manual_seed(0)
net = ActorCriticCNN(dtype=torch.bfloat16).to(dev)
ref = None
for path in libs:
    _lib.LIB_PATH, _lib._lib = path, None
    wfrag, bias = pack_cnn(net)
    run = lambda: cnn_forward(boards, wfrag, bias, exponents=True, logits=True, value=True, actions=True, seed=1)
    lg, v, a = run()
    torch.cuda.synchronize()
    got = (lg.clone(), v.clone(), a.clone())
    if ref is None:
        ref, same = got, "ref"
    else:
        same = "bit-identical" if all(torch.equal(x, y) for x, y in zip(got, ref)) else "DIFFERS"
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print("%-50s %.4f ms per %d boards (%.1f G boards/s)  %s" % (path, ms, n, n / ms / 1e6, same), flush=True)
