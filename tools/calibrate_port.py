"""Calibrate oracle/game_port.py (the CPU baseline that travels to the GPU box) against the real
reference (nevertiree/Rein48 game/GameClient.py + control/rand.py), same core, same seeds,
interleaved rounds. Runs only where /root/reference exists. Writes profiles/calibration_port.json."""
import json
import os
import platform
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import game_port  # noqa: E402

sys.dont_write_bytecode = True
sys.path.insert(0, "/root/reference")
from game.GameClient import Game  # noqa: E402  (reference)
from control.rand import Rand  # noqa: E402  (reference)


def ref_run(n, seed):
    random.seed(seed)
    g, e = Game(), 0
    for _ in range(n):
        _, _, d = g.step(Rand.random_action(g.state_matrix))
        if d:
            e += 1
            g = Game()
    return e


def main():
    n, rounds = 200_000, 5
    res = {"ref": [], "port": []}
    for r in range(rounds):
        for name, f in (("ref", ref_run), ("port", game_port.run_steps)):
            t = time.perf_counter()
            e = f(n, r)
            res[name].append(n / (time.perf_counter() - t))
        assert ref_run(5000, 99 + r) == game_port.run_steps(5000, 99 + r)  # same seeded episodes
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    out = {"steps_per_round": n, "rounds": rounds, "reference_steps_per_s": res["ref"], "port_steps_per_s": res["port"],
           "median_reference": med["ref"], "median_port": med["port"], "port_over_reference": med["port"] / med["ref"],
           "host": platform.processor() or platform.machine(), "python": platform.python_version()}
    json.dump(out, open(os.path.join(ROOT, "profiles", "calibration_port.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
