"""GPU probe: the config-5 training step (dqn/train_step.ResNetTrainStep, 64K boards) eager vs
replayed from a HIP graph captured with torch.cuda.CUDAGraph (static input buffers): device ms
per step from HIP events over 20 back-to-back steps, and whether the gradients agree bit for bit.

    python tools/probe_graph.py [batch]"""
import sys

import torch

sys.path.insert(0, ".")
from rein48_amd.dqn import DQNConfig  # noqa: E402
from rein48_amd.dqn.conv import board_onehot32  # noqa: E402
from rein48_amd.dqn.trainer import DQNLearner  # noqa: E402
from rein48_amd.dqn.train_step import ResNetTrainStep  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 16
dev = torch.device("cuda:0")
lr = DQNLearner(DQNConfig(batch=B, seed=3), device=dev)
lr.net.train()
step = ResNetTrainStep(lr.net)
g = torch.Generator(device="cpu").manual_seed(1)
x = board_onehot32(torch.randint(0, 12, (B, 16), generator=g, dtype=torch.int8).to(dev)).view(B, 512)
a = torch.randint(0, 4, (B,), generator=g, dtype=torch.int8).to(dev)
y = torch.randn(B, generator=g).to(dev)
s = torch.cuda.current_stream()


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def eager():
    lr.flat.zero_grad()
    return step(x, a, y)


for _ in range(3):
    eager()
torch.cuda.synchronize()
ms_eager = timed(eager)
eager()
g_eager = lr.flat.grad.clone()
side = torch.cuda.Stream()
side.wait_stream(s)
with torch.cuda.stream(side):
    for _ in range(2):
        eager()
s.wait_stream(side)
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    lr.flat.zero_grad()
    out = step(x, a, y)
torch.cuda.synchronize()
ms_graph = timed(graph.replay)
graph.replay()
torch.cuda.synchronize()
same = torch.equal(lr.flat.grad, g_eager)
print("batch %d: eager %.3f ms per step, graph replay %.3f ms per step (%.1f%%), gradients bit-identical: %s"
      % (B, ms_eager, ms_graph, 100 * (ms_graph / ms_eager - 1), same), flush=True)
