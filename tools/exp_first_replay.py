"""GPU experiment: is the first replay of a prepared step_n graph slower than later ones?"""
import sys
import torch
sys.path.insert(0, ".")
from rein48_amd import VecGame

env = VecGame(1 << 20, device="cuda:0", seed=1)
env.reset()
env.step_n(200, auto_reset=True)
env.prepare_step_n(1000, auto_reset=True)
torch.cuda.synchronize()
s = torch.cuda.current_stream()
for i in range(5):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    env.step_n(1000, auto_reset=True)
    b.record(s)
    torch.cuda.synchronize()
    print("replay %d: %.2f us/step" % (i, a.elapsed_time(b)), flush=True)
