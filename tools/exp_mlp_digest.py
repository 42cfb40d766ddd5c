"""GPU experiment: a bit-level digest of one reference-MLP rollout (actions, values, final boards) and
forward pass per library build, to check that builds claimed bit-identical are.

    R48_LIB=... python tools/exp_mlp_digest.py      (one library per process)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd.a3c import A3CConfig, A3CTrainer  # noqa: E402
from rein48_amd.a3c.fused import mlp_forward  # noqa: E402

dev = torch.device("cuda:0")
cfg = A3CConfig(n_boards=(1 << 16) + 3, max_steps=60, mode="reference", net="mlp", bf16=False, features="values",
                seed=11)
tr = A3CTrainer(cfg, device=dev)
with torch.no_grad():
    for m in (tr.net.a1, tr.net.a2, tr.net.c1, tr.net.c2):
        m.bias.uniform_(-0.5, 0.5)
tr.rollout()
lg, v, _ = mlp_forward(tr.boards[5].contiguous(), tr._mlp_weights(), logits=True, value=True)


def dig(t):
    t = t.contiguous()
    x = t.view(torch.int8).long() if t.element_size() == 1 else t.view(torch.int32).long()
    return int((x * 2654435761).sum()) & 0xFFFFFFFF


print("%-24s actions %08x values %08x boards %08x logits %08x value %08x" % (
    os.path.basename(os.environ.get("R48_LIB", "product")), dig(tr.actions), dig(tr._rollout_v[0]), dig(tr.env.boards),
    dig(lg), dig(v)), flush=True)
