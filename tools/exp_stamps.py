"""GPU experiment: per-wave clock stamps of k_step_n (diagnostic build made by tools/stamp_env.py).

Build:  python tools/stamp_env.py
Run:    R48_LIB=build/librein48_stamp.so python tools/exp_stamps.py [boards] [K]
Prints, for one K-step call after a settle period: the effective core clock of each wave
(s_memtime ticks / s_memrealtime at 100 MHz), wave lifetimes, the span from the first wave's
start to the last wave's end, and the mean number of waves alive per SIMD over that span."""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd import VecGame, _lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
env = VecGame(n, device="cuda:0", seed=1)
env.fill_random(7)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:
    env.step_n(K, auto_reset=True)
    torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
env.step_n(K, auto_reset=True)
b.record()
torch.cuda.synchronize()
ev_ms = a.elapsed_time(b)
waves = min(65536, n // 128)
buf = (C.c_ulonglong * (4 * waves))()
lib = _lib.load()
lib.r48_debug_stamps.argtypes = [C.c_void_p, C.c_int64]
assert lib.r48_debug_stamps(buf, waves) == 0
s = np.frombuffer(buf, dtype=np.uint64).reshape(waves, 4).astype(np.int64)
r0 = s[:, 1]
cyc = s[:, 2]
rdur = (s[:, 3] >> 32)                     # 100 MHz ticks
hw = s[:, 3] & 0xFFFFFFFF
ghz = cyc / np.maximum(rdur, 1) / 10.0     # ticks per 10 ns
span = (r0 + rdur).max() - r0.min()
simds = 1024
print("boards 2^%d  K=%d  event %.4f ms  waves %d" % (n.bit_length() - 1, K, ev_ms, waves))
print("wave lifetime us: mean %.2f min %.2f max %.2f" % (rdur.mean() / 100, rdur.min() / 100, rdur.max() / 100))
print("start offsets us: max %.2f  (p50 %.2f)   end offsets us: min %.2f max %.2f" % (
    (r0 - r0.min()).max() / 100, np.median(r0 - r0.min()) / 100,
    ((r0 + rdur) - r0.min()).min() / 100, ((r0 + rdur) - r0.min()).max() / 100))
print("span first start -> last end: %.2f us" % (span / 100))
print("effective core clock GHz: mean %.3f  min %.3f  max %.3f" % (ghz.mean(), ghz.min(), ghz.max()))
print("mean waves alive per SIMD over the span: %.2f" % (rdur.sum() / span / simds))
# HW_ID (gfx9): wave slot [3:0], SIMD [5:4], CU [11:8], SH [12], SE [15:13]; XCC id in [31:28]
slot = (hw >> 28) * 1000000 + ((hw >> 13) & 7) * 10000 + ((hw >> 12) & 1) * 1000 + ((hw >> 8) & 15) * 10 + ((hw >> 4) & 3)
u, cnt = np.unique(slot, return_counts=True)
print("distinct SIMDs %d; waves per SIMD: min %d max %d mean %.2f" % (len(u), cnt.min(), cnt.max(), cnt.mean()))
late = (r0 - r0.min()) > 200          # started > 2 us after the first wave
print("waves starting > 2 us late: %d (%.1f%%)" % (late.sum(), 100 * late.mean()))
# max concurrency per SIMD: sweep start/end events
mx = []
for sid in u:
    m = slot == sid
    ev = sorted([(int(t), 1) for t in r0[m]] + [(int(t), -1) for t in (r0 + rdur)[m]], key=lambda e: (e[0], e[1]))
    c = best = 0
    for _, d in ev:
        c += d
        best = max(best, c)
    mx.append(best)
mx = np.array(mx)
print("max concurrent waves per SIMD: min %d max %d mean %.2f" % (mx.min(), mx.max(), mx.mean()))
h = np.bincount(mx)
print("histogram of per-SIMD max concurrency:", {i: int(v) for i, v in enumerate(h) if v})
