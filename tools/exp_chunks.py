"""GPU experiment: per-step time of VecGame.step_n for several chunk sizes / board counts."""
import sys
import time
import torch
sys.path.insert(0, ".")
from rein48_amd import VecGame

for n in (1 << 20, 1 << 22, 1 << 26):
    env = VecGame(n, device="cuda:0", seed=1)
    env.reset()
    for chunk in (100, 1000, 4096):
        env.step_n(chunk, auto_reset=True)
        torch.cuda.synchronize()
        reps = max(1, 8192 // chunk) if n <= (1 << 22) else 1
        s = torch.cuda.current_stream()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        a.record(s)
        for _ in range(reps):
            env.step_n(chunk, auto_reset=True)
        b.record(s)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / (reps * chunk)
        print("n=%9d chunk=%4d  gpu %.2f us/step  wall %.2f us/step  -> %.1f G steps/s"
              % (n, chunk, a.elapsed_time(b) * 1e3 / (reps * chunk), wall * 1e6, n / wall / 1e9), flush=True)
    # eager single-kernel for reference
    torch.cuda.synchronize()
    a.record(s)
    for _ in range(200 if n <= (1 << 22) else 10):
        env.step(None, auto_reset=True)
    b.record(s)
    torch.cuda.synchronize()
    print("n=%9d eager      gpu %.2f us/step" % (n, a.elapsed_time(b) * 1e3 / (200 if n <= (1 << 22) else 10)))
    del env
    torch.cuda.empty_cache()
