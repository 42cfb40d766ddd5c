"""GPU experiment: VecGame.step_n per-step time for librein48 builds (one child process each).

    python tools/exp_step_variants.py [--pingpong-min N] [lib.so ...]   (default: the product library)

Variant libraries come from tools/build_variant.sh, e.g. the zero-compute floor with the same
launch structure and I/O as the env step:
    tools/build_variant.sh rein48_amd/csrc/r48_env.hip r48_env build/var/copy.so -DR48_ABLATE_STEP_COPY
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys, time, torch
sys.path.insert(0, %(root)r)
from rein48_amd import _lib
_lib.LIB_PATH, _lib._lib = %(lib)r, None
from rein48_amd import VecGame
out = {}
# deterministic result check first: every build / chain count / ping-pong setting must agree
env = VecGame(300_001, device="cuda:0", seed=5)
if %(pp)d >= 0:
    env.set_pingpong_min(%(pp)d)
env.fill_random(7)
env.step_n(777, auto_reset=True)
env.step_n(64, auto_reset=True)
out["check_hash"] = int(env.boards.view(torch.int32).long().mul(2654435761).sum()) & 0xFFFFFFFF
del env
for n, chunk, reps in ((1 << 20, 1000, 8), (1 << 22, 1000, 2), (1 << 26, 200, 1)):
    env = VecGame(n, device="cuda:0", seed=1)
    if %(pp)d >= 0:
        env.set_pingpong_min(%(pp)d)
    env.fill_random(7)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.15:          # clock ramp + graph capture
        env.step_n(chunk, auto_reset=True)
        torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        env.step_n(chunk, auto_reset=True)
    b.record(s)
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / (reps * chunk)
    out[str(n)] = {"us_per_step": us, "G_env_steps_per_s": n / us / 1e3, "GBs_34B": n * 34 / us / 1e3}
    del env
    torch.cuda.empty_cache()
print(json.dumps(out))
"""


def main():
    args = sys.argv[1:]
    pp = -1
    if args[:1] == ["--pingpong-min"]:
        pp, args = int(args[1]), args[2:]
    libs = args or [os.path.join(ROOT, "rein48_amd", "lib", "librein48.so")]
    for lib in libs:
        p = subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT, "lib": os.path.abspath(lib), "pp": pp}],
                           capture_output=True, text=True, timeout=300)
        if p.returncode != 0:
            print(lib, "FAILED", p.stderr[-800:], flush=True)
            sys.exit(1)
        r = json.loads(p.stdout.strip().splitlines()[-1])
        print("%-30s pp=%-9d check hash %d" % (os.path.basename(lib), pp, r.pop("check_hash")), flush=True)
        for n, v in r.items():
            print("%-30s pp=%-9d n=%9s  %8.3f us/step  %6.1f G steps/s  %6.0f GB/s" %
                  (os.path.basename(lib), pp, n, v["us_per_step"], v["G_env_steps_per_s"], v["GBs_34B"]), flush=True)


if __name__ == "__main__":
    main()
