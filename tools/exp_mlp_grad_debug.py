"""GPU diagnostic: r48_mlp_train_grad vs a float64 restatement of the textbook A3C loss gradient of the
reference MLP at several row counts (1 tile per wave, 2 tiles per wave, ...): per-tensor max error
relative to the tensor's scale.  python tools/exp_mlp_grad_debug.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd.a3c.fused import mlp_train_grad  # noqa: E402
from rein48_amd.a3c.nets import ActorCriticMLP  # noqa: E402

DEV = "cuda:0"
torch.manual_seed(11)
net = ActorCriticMLP().to(DEV)
with torch.no_grad():
    for m in (net.a1, net.a2, net.c1, net.c2):
        m.bias.uniform_(-0.5, 0.5)
P = {k: v.detach().double().cpu().numpy() for k, v in net.named_parameters()}


def ref(x, act, tgt, wn, beta=0.001):
    a = x @ P["a1.weight"].T + P["a1.bias"]
    h = np.clip(a, 0, 6)
    zr = h @ P["a2.weight"].T + P["a2.bias"]
    z = np.maximum(zr, 0)
    c = x @ P["c1.weight"].T + P["c1.bias"]
    hc = np.clip(c, 0, 6)
    v = hc @ P["c2.weight"][0] + P["c2.bias"][0]
    p = np.exp(z - z.max(1, keepdims=True))
    p /= p.sum(1, keepdims=True)
    lq = np.log(p + 1e-5)
    gr = -(lq + p / (p + 1e-5))
    gbar = (p * gr).sum(1, keepdims=True)
    td = tgt - v
    oh = np.eye(4)[act]
    dz = -wn[:, None] * (beta * p * (gr - gbar) + td[:, None] * (oh - p))
    dz = np.where(zr > 0, dz, 0.0)
    dv = -2.0 * wn * td
    dh = ((a > 0) & (a < 6)) * (dz @ P["a2.weight"])
    dhc = ((c > 0) & (c < 6)) * (dv[:, None] * P["c2.weight"][0][None, :])
    return [dh.T @ x, dh.sum(0), dz.T @ h, dz.sum(0), dhc.T @ x, dhc.sum(0), (dv[:, None] * hc).sum(0)[None, :],
            np.array([dv.sum()])]


for rows in (30_021, 262_144, 262_208, 524_288, 1_048_616):
    rng = np.random.default_rng(rows)
    b = rng.integers(1, 10, size=(rows, 16)).astype(np.int8)
    b[rng.random((rows, 16)) < 0.4] = 0
    act = rng.integers(0, 4, size=rows)
    tgt = rng.normal(scale=2.0, size=rows)
    wn = np.full(rows, 1.0 / rows)
    x = np.where(b > 0, 2.0 ** b, 0.0)
    want = ref(x, act, tgt, wn)
    g, _, _ = mlp_train_grad(net, torch.from_numpy(b).to(DEV), torch.from_numpy(act.astype(np.int8)).to(DEV),
                             torch.from_numpy(tgt.astype(np.float32)).to(DEV),
                             torch.from_numpy(wn.astype(np.float32)).to(DEV), n_boards=rows)
    g = g.double().cpu().numpy()
    off, errs = 0, []
    for (name, p), w64 in zip(net.named_parameters(), want):
        k = p.numel()
        f = g[off:off + k].reshape(w64.shape)
        off += k
        errs.append("%s %.1e" % (name, np.abs(f - w64).max() / (np.abs(w64).max() + 1e-30)))
    print("rows %9d (%5d tiles): %s" % (rows, (rows + 63) // 64, " | ".join(errs)), flush=True)
