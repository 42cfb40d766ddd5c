"""Golden fixtures for the transition store FROM THE REFERENCE's algorithm/ddpg/replay.py.

Runs only in the build container (the read-only reference lives at /root/reference). Imports
the reference Replay class, drives it through scripted store/sample sequences under
random.seed, and writes the inputs and the outputs it produced (data only) to
tests/golden/replay.json:
  transitions   the stored (state, action, reward, next_state) tuples, boards as tile values
  sample        the dict list_2_dict returned (replay.py:36-43), as lists
  picked        for each sampled row, the index of the stored transition it came from
  filled / cur_size_after   replay.py:15-16 before sampling, cur_size after (clear())

Usage:  python tests/golden/make_replay_golden.py
"""
import json
import os
import random
import sys

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

# (name, replay_size, n_store, batch_size or None for the default, seed)
SCENARIOS = [
    ("subset", 100, 30, 10, 11),       # random.sample of 10 out of 30
    ("overflow_all", 100, 120, 200, 12),  # store drops past 100; batch > len -> whole buffer in order
    ("exact_perm", 5, 5, 5, 13),       # batch == len -> random.sample = a permutation
    ("empty", 100, 0, None, 14),       # default batch (MINI_BATCH_SIZE = 10) on an empty buffer
    ("fewer", 100, 3, 10, 15),         # batch > len -> all 3 in insertion order
    ("default_batch", 100, 40, None, 16),
]


def board(rng):
    e = rng.integers(0, 12, size=(4, 4))
    e[rng.random((4, 4)) < 0.4] = 0
    return [[int(1 << v) if v else 0 for v in row] for row in e]


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    from algorithm.ddpg import replay as R  # noqa: E402  (the reference module)

    out = {"mini_batch_size": R.MINI_BATCH_SIZE, "scenarios": []}
    for name, size, n_store, batch, seed in SCENARIOS:
        rng = np.random.default_rng(seed)
        trans = [[board(rng), int(rng.integers(0, 4)), int(rng.integers(0, 64)), board(rng)] for _ in range(n_store)]
        random.seed(seed)
        rep = R.Replay(replay_size=size)
        for t in trans:
            rep.store(t)
        filled = rep.filled()
        cur = rep.cur_size
        smp = rep.sample() if batch is None else rep.sample(batch_size=batch)
        keys = [json.dumps(t) for t in trans]
        picked = []
        for i in range(len(smp["action"])):
            row = [smp["state"][i].tolist(), int(smp["action"][i]), int(smp["reward"][i]), smp["next_state"][i].tolist()]
            picked.append(keys.index(json.dumps(row)))
        out["scenarios"].append({
            "name": name, "replay_size": size, "batch_size": batch, "seed": seed, "transitions": trans,
            "filled": bool(filled), "cur_size_before": cur, "cur_size_after": rep.cur_size,
            "sample": {k: np.asarray(v).tolist() for k, v in smp.items()},
            "sample_shapes": {k: list(np.asarray(v).shape) for k, v in smp.items()},
            "picked": picked,
        })
    path = os.path.join(HERE, "replay.json")
    with open(path, "w") as f:
        json.dump(out, f)
    print("wrote", path, [(s["name"], s["picked"][:5]) for s in out["scenarios"]])


if __name__ == "__main__":
    main()
