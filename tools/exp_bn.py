"""GPU experiment: fused BN + ReLU (+ add) (r48_bn_*, rein48_amd/dqn/bn.py) vs PyTorch's
channels-last BatchNorm1d + ReLU (+ add) on the config-5 update's activations (bf16 [2^20, 64]:
a 64K-board minibatch x 16 cells), forward and backward, and one full DQN update each way."""
import json
import sys

import torch

sys.path.insert(0, ".")
from rein48_amd.dqn.bn import bn_act  # noqa: E402

DEV = "cuda:0"


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


rows, C = 1 << 20, 64
x = torch.randn(rows, C, device=DEV, dtype=torch.bfloat16).requires_grad_(True)
res = torch.randn(rows, C, device=DEV, dtype=torch.bfloat16).requires_grad_(True)
dy = torch.randn(rows, C, device=DEV, dtype=torch.bfloat16)
bn = torch.nn.BatchNorm1d(C).to(DEV).train()
out = {"rows": rows, "C": C}
for name, r in (("bn_relu", None), ("bn_add_relu", res)):
    def fused_fwd():
        return bn_act(x, bn, r)

    def torch_fwd():
        z = bn(x)
        return torch.relu(z + r if r is not None else z)

    def fb(f):
        return lambda: f().backward(dy)
    mb = rows * C * 2 / 1e6
    fw_k, fw_t = timed(fused_fwd), timed(torch_fwd)
    fb_k, fb_t = timed(fb(fused_fwd)), timed(fb(torch_fwd))
    n_in = 2 if r is None else 3         # fwd bytes: stats read x, apply read x (+res), write y
    algo_fwd = (n_in + 1) * mb
    algo_bwd = (3 + 3 + 1 + (1 if r is not None else 0)) * mb   # reduce dy,y,x; apply dy,y,x -> dx (+dres)
    out[name] = {"fused_fwd_ms": fw_k, "torch_fwd_ms": fw_t, "fused_fwd_bwd_ms": fb_k, "torch_fwd_bwd_ms": fb_t,
                 "fused_fwd_GBs": algo_fwd / fw_k, "fused_fwd_bwd_GBs": (algo_fwd + algo_bwd) / fb_k}
    print(name, json.dumps(out[name]), flush=True)

from rein48_amd.dqn import DQNConfig, DQNTrainer  # noqa: E402
cfg = DQNConfig(n_boards=1 << 18, replay_capacity=1 << 22, batch=1 << 16, learn_start=1, seed=3)
tr = DQNTrainer(cfg, device=DEV)
for _ in range(3):
    tr.env_step()
for fused in (True, False):
    tr.net.fused_bn = fused
    out["dqn_update_ms_" + ("fused_bn" if fused else "torch_bn")] = timed(tr.update, reps=5)
print(json.dumps(out))
