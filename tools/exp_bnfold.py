"""GPU experiment: ResNetTrainStep (config-5 update's forward + backward) at the bench's 64K-board
minibatch with the BN applies folded into the next conv (fold_bn=True) vs separate apply passes:
median device time per step over 20 steps, alternated, after warm-up.

    python tools/exp_bnfold.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd.a3c.optim import FlatParams  # noqa: E402
from rein48_amd.dqn.conv import board_onehot32  # noqa: E402
from rein48_amd.dqn.nets import ResNet10Q  # noqa: E402
from rein48_amd.dqn.train_step import ResNetTrainStep  # noqa: E402

DEV = "cuda:0"
B = 1 << 16
torch.manual_seed(0)
net = ResNet10Q(dtype=torch.bfloat16).to(DEV).train()
FlatParams(net)
rng = np.random.default_rng(0)
x = board_onehot32(torch.from_numpy(rng.integers(0, 14, size=(B, 16)).astype(np.int8)).to(DEV)).view(B, 512)
a = torch.from_numpy(rng.integers(0, 4, size=B).astype(np.int8)).to(DEV)
y = torch.from_numpy(rng.normal(size=B).astype(np.float32)).to(DEV)
steps = {f: ResNetTrainStep(net, fold_bn=f) for f in (False, True)}
for f in steps:
    for _ in range(5):
        steps[f](x, a, y)
torch.cuda.synchronize()
res = {False: [], True: []}
s = torch.cuda.current_stream()
for rnd in range(4):
    for f in (False, True):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(5):
            steps[f](x, a, y)
        e1.record(s)
        torch.cuda.synchronize()
        res[f].append(e0.elapsed_time(e1) / 5)
for f in (False, True):
    v = sorted(res[f])
    print("fold_bn=%s: %.3f ms per forward+backward (rounds %s)" % (f, v[len(v) // 2], ["%.3f" % t for t in res[f]]))
