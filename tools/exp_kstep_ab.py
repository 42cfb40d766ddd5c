"""GPU experiment: k_step (one step per launch, boards through HBM) at 2^26 boards -- the HBM-honest
point -- of one library build (default: the product library; a variant from tools/build_variant.sh
to A/B); median device time per launch over 3 rounds of 30 back-to-back launches after a settle,
and a digest of the boards.

    python tools/exp_kstep_ab.py [lib.so]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd import VecGame, _lib  # noqa: E402

if len(sys.argv) > 1:
    _lib.LIB_PATH, _lib._lib = sys.argv[1], None

dev = "cuda:0"
n = 1 << 26
env = VecGame(n, device=dev, seed=1)
env.fill_random(7)
s = torch.cuda.current_stream()
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:
    env.step(None, auto_reset=True)
    torch.cuda.synchronize()
per = []
for _ in range(3):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(30):
        env.step(None, auto_reset=True)
    b.record(s)
    torch.cuda.synchronize()
    per.append(a.elapsed_time(b) / 30)
ms = sorted(per)[1]
digest = int((env.boards.view(torch.int32).long() * 2654435761).sum()) & 0xFFFFFFFF
print("%s k_step 2^26: %.1f us/launch = %.0f GB/s (34 B/board) = %.3f of 8 TB/s | rounds %s | digest %08x"
      % (os.path.basename(_lib.LIB_PATH), ms * 1e3, n * 34 / (ms * 1e-3) / 1e9,
         n * 34 / (ms * 1e-3) / 8e12, ["%.1f" % (p * 1e3) for p in per], digest), flush=True)
