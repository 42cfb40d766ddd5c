"""GPU experiment: where the wall time of the driver's K = 20 region goes beyond the kernel.
Times the bench's timed region (one r48_env_step_n launch of K steps over 2^20 boards) with
variants of the host-side bracketing, 30 regions each after a settle period (median, spread):
  events_in     bench.py's round-2 region: event record, launch, event record, device synchronize
  events_pre    the opening event recorded before t0 (its host cost no longer delays the launch)
  no_events     launch + device synchronize only
  stream_sync   launch + stream synchronize
  event_sync    launch + record + event synchronize
With --spin the process first sets hipDeviceScheduleSpin (the host thread spins instead of yielding
while it waits) before the HIP context exists.

    python tools/exp_sync.py [--spin] [K]"""
import ctypes
import os
import statistics
import sys
import time

SPIN = "--spin" in sys.argv
args = [a for a in sys.argv[1:] if a != "--spin"]
K = int(args[0]) if args else 20
if SPIN:
    hip = ctypes.CDLL("libamdhip64.so")
    print("hipSetDeviceFlags(spin) ->", hip.hipSetDeviceFlags(ctypes.c_uint(1)), flush=True)

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd import VecGame  # noqa: E402

dev = torch.device("cuda:0")
n = 1 << 20
env = VecGame(n, device=dev, seed=0x20485EED)
env.fill_random(7)
s = torch.cuda.current_stream(dev)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:
    env.step_n(K, auto_reset=True)
    torch.cuda.synchronize(dev)


def region(kind):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    b.record(s)
    torch.cuda.synchronize(dev)
    env.step_n(K, auto_reset=True)     # settle between regions, like bench.py's repeats
    torch.cuda.synchronize(dev)
    if kind == "events_pre":
        a.record(s)
    t = time.perf_counter()
    if kind == "events_in":
        a.record(s)
    env.step_n(K, auto_reset=True)
    if kind in ("events_in", "events_pre", "event_sync"):
        b.record(s)
    if kind == "stream_sync":
        s.synchronize()
    elif kind == "event_sync":
        b.synchronize()
    else:
        torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t
    dms = a.elapsed_time(b) if kind in ("events_in", "events_pre") else float("nan")
    return wall * 1e6, dms * 1e3


for kind in ("events_in", "events_pre", "no_events", "stream_sync", "event_sync", "events_in"):
    r = [region(kind) for _ in range(30)]
    w = [x[0] for x in r]
    d = [x[1] for x in r]
    print("%-12s spin=%d K=%d  wall us median %.1f min %.1f max %.1f | device us median %.1f  -> %.1f G env-steps/s"
          % (kind, SPIN, K, statistics.median(w), min(w), max(w), statistics.median(d), n * K / statistics.median(w) / 1e3),
          flush=True)
