"""GPU diagnostic: fraction of 16-row tiles the hot pass of r48_mlp_train_grad puts on its fix-pass lists
(rein48_amd/csrc/r48_mlp_train.hip), on the training rows of a real config-3 rollout (2^20 boards x 100
steps of the reference MLP), per loss mode / input encoding. Reads the lists' lengths from the
workspace (layout of r48_mlp_train_workspace_floats).

    python tools/exp_mlp_flags.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd.a3c import A3CConfig, A3CTrainer  # noqa: E402

REC, RECS, RED = 2504, 2048, 64
REC_FLOATS = (2 * RECS + (2 * RECS + RED - 1) // RED) * REC

for mode, feat in (("reference", "values"), ("textbook", "exponents")):
    tr = A3CTrainer(A3CConfig(n_boards=1 << 20, max_steps=100, mode=mode, net="mlp", bf16=False, features=feat,
                              seed=1), device="cuda:0")
    for _ in range(3):
        tr.train_step()
    tr.rollout()
    tr.update()
    torch.cuda.synchronize()
    ws = tr._mlp_ws
    rows = 100 * (1 << 20)
    tiles = (rows + 15) // 16
    cap = max(1, (tiles + RECS - 1) // RECS)
    lens = ws[REC_FLOATS + 2 * RECS * cap: REC_FLOATS + 2 * RECS * cap + RECS].view(torch.int32)
    tot = int(lens.long().sum())
    print("%-9s %-9s flagged tiles %d of %d = %.2f %%  (per wave: min %d max %d)" % (
        mode, feat, tot, tiles, 100.0 * tot / tiles, int(lens.min()), int(lens.max())), flush=True)
