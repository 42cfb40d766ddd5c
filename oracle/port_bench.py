"""TEST/BENCH INFRASTRUCTURE ONLY -- the CPU baseline leg of bench.py.

Times oracle/game_port.py (the faithful pure-Python restatement of the reference Game + Rand,
calibrated against the reference in BASELINE.md) on P worker processes, one board each, for a
bounded number of seconds, plus the 1-process figure. Prints one JSON object.
bench.py runs this as a child process before it touches the GPU, so the workers fork from a
process that never initialised HIP.

    python -m oracle.port_bench --procs 16 --seconds 10 --single-seconds 5
"""
import argparse
import json
import multiprocessing as mp
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHUNK = 5_000


def _worker(args):
    seconds, seed = args
    from oracle import game_port
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        game_port.run_steps(CHUNK, seed=seed)
        steps += CHUNK
        seed += 1000
    return steps, time.perf_counter() - t0


def default_procs(cap=16):
    """Worker count: the CPUs this process may run on, capped at the GPU box's 16-CPU share."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(cap, n))


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def run(procs, seconds, single_seconds):
    s_steps, s_dt = _worker((single_seconds, 1)) if single_seconds > 0 else (0, 1.0)
    with mp.get_context("fork").Pool(procs) as pool:
        res = pool.map(_worker, [(seconds, 100 + k) for k in range(procs)])
    total = sum(s for s, _ in res)
    value = sum(s / dt for s, dt in res)
    return {"value": value, "unit": "env steps/s", "cores": procs, "kind": "port",
            "single_process_value": s_steps / s_dt if single_seconds > 0 else None,
            "sample": "oracle/game_port.py (list-of-lists, deepcopy per move, global random, auto-restart on "
                      "game over; one board per process): %d steps on %d processes x %.1f s, plus %d steps on "
                      "1 process in %.1f s; %s, Python %s"
                      % (total, procs, seconds, s_steps, s_dt, cpu_model(), platform.python_version())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=0, help="0 = default_procs()")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--single-seconds", type=float, default=5.0)
    a = ap.parse_args()
    print(json.dumps(run(a.procs or default_procs(), a.seconds, a.single_seconds)), flush=True)


if __name__ == "__main__":
    main()
