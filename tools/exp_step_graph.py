"""GPU experiment: the config-5 training step (train_step.ResNetTrainStep at the 64K minibatch) eager
vs replayed from a HIP graph captured with torch.cuda.graph (the same launches, static buffers).
Alternated rounds; prints ms per step and whether the graph's outputs equal the eager step's.
    python tools/exp_step_graph.py [rounds]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd.a3c.optim import FlatParams  # noqa: E402
from rein48_amd.dqn.conv import board_onehot32  # noqa: E402
from rein48_amd.dqn.nets import ResNet10Q  # noqa: E402
from rein48_amd.dqn.train_step import ResNetTrainStep  # noqa: E402

dev = torch.device("cuda:0")
B = 1 << 16
torch.manual_seed(0)
net = ResNet10Q(dtype=torch.bfloat16).to(dev).train()
flat = FlatParams(net)
rng = np.random.default_rng(0)
x = board_onehot32(torch.from_numpy(rng.integers(0, 14, size=(B, 16)).astype(np.int8)).to(dev)).view(B, 512)
action = torch.from_numpy(rng.integers(0, 4, size=B).astype(np.int8)).to(dev)
target = torch.from_numpy(rng.normal(size=B).astype(np.float32)).to(dev)
step = ResNetTrainStep(net)
for _ in range(3):
    out_e = step(x, action, target)
torch.cuda.synchronize()
g_eager = flat.grad.clone()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        step(x, action, target)
torch.cuda.current_stream().wait_stream(s)
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    out_g = step(x, action, target)
graph.replay()
torch.cuda.synchronize()
print("graph gradient == eager gradient:", torch.equal(flat.grad, g_eager), flush=True)


def timed(fn, n=20):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
for r in range(rounds):
    arms = [("eager", lambda: step(x, action, target)), ("graph", graph.replay)]
    if r % 2:
        arms.reverse()
    print(" ".join("%s %.3f ms" % (k, timed(f)) for k, f in arms), flush=True)
