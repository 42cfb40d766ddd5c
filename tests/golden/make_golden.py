"""Generate the golden fixtures for the 2048 env hot path FROM THE REFERENCE ITSELF.

Runs only in the survey/build container, where the read-only reference lives at
/root/reference. It imports the reference's own `game/GameClient.py` and
`control/rand.py`, drives them, and writes small DATA fixtures next to this
script. No reference source (or bytecode) is copied: the fixtures are inputs and
the outputs the reference produced for them.

Fixtures written:
  kats.json             the reference test file's KATs (GameClientTest.py:10-31, :49-331),
                        parsed from the test file's text, each re-run through the
                        reference Game to record its actual output.
  trajectories.npz      seeded random-policy episodes (main.py:36-42 loop with
                        Rand.random_action, control/rand.py:9-11), with every RNG draw
                        the reference made (randint rank, uniform) recorded per step.
  line_table.json       SHA-256 of the exhaustive 18^4-line x 4-direction move table
                        produced by Game.update_matrix (GameClient.py:129-254).
  fingerprint.json      random-policy statistics (episode length, score, max tile,
                        no-op fraction) over seeds 100-107 x 2500 episodes.

Usage:  python tests/golden/make_golden.py [--skip-fingerprint]
"""
import argparse
import copy
import hashlib
import json
import os
import re
import sys

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
DIRS = {"UP": 0, "DOWN": 1, "LEFT": 2, "RIGHT": 3}


def _import_reference():
    sys.dont_write_bytecode = True  # the reference tree is read-only
    sys.path.insert(0, REF)
    import game.GameClient as gc  # noqa: E402  (reference module)
    import control.rand as cr  # noqa: E402
    return gc, cr


def exp_of(v):
    """Raw tile value (0, 2, 4, ...) -> exponent (0 = empty)."""
    if v == 0:
        return 0
    e = int(v).bit_length() - 1
    assert (1 << e) == v, v
    return e


def board_to_exp(m):
    return [exp_of(v) for row in m for v in row]


# --------------------------------------------------------------------------- KATs
def make_kats(gc):
    text = open(os.path.join(REF, "game", "GameClientTest.py")).read()
    out = {"source": "game/GameClientTest.py", "line_moves": [], "filled": [], "game_over": []}
    # line-move KATs: split by test function, read (test_matrix, except_matrix, direction string)
    for fn in re.finditer(r"def (test_update_matrix_\w+)\(self\):(.*?)(?=\n    def |\Z)", text, re.S):
        body = fn.group(2)
        ins = re.findall(r"test_matrix = (\[.*?\])\n", body)
        exps = re.findall(r"except_matrix = (\[.*?\])\n", body)
        acts = re.findall(r"update_matrix\(test_matrix, \"(\w+)\"\)", body)
        assert len(ins) == len(exps) == len(acts) == 10, fn.group(1)
        for k, (i, e, a) in enumerate(zip(ins, exps, acts)):
            mi, me = json.loads(i), json.loads(e)
            got, reward, changed = gc.Game.update_matrix(copy.deepcopy(mi), a)
            out["line_moves"].append({"test": fn.group(1), "case": k + 1, "action": a,
                                      "input": mi, "expected": me, "reference_output": got,
                                      "reference_reward": reward, "reference_changed": bool(changed)})
    # filled / game-over KATs (GameClientTest.py:10-31)
    for name, key, fnc in (("test_has_matrix_filled", "filled", gc.Game.has_table_filled),
                           ("test_is_game_over", "game_over", gc.Game.has_game_over)):
        m = re.search(r"def %s\(self\):(.*?)(?=\n    def )" % name, text, re.S)
        body = m.group(1)
        for mt in re.finditer(r"test_matrix = (\[.*?\])\n\s+assert (not )?", body):
            mat = json.loads(mt.group(1).replace(", ]", "]"))
            expected = mt.group(2) is None
            out[key].append({"input": mat, "expected": expected, "reference_output": bool(fnc(mat))})
    assert len(out["filled"]) == 3 and len(out["game_over"]) == 3, (out["filled"], out["game_over"])
    for rec in out["filled"] + out["game_over"]:
        assert rec["expected"] == rec["reference_output"]
    return out


# ------------------------------------------------------------------ trajectories
class _Recorder:
    """Stands in for the `random` module inside the reference GameClient and records
    every draw it makes, while delegating to the real global MT19937 stream (which the
    reference's Rand policy shares, control/rand.py:3,11)."""

    def __init__(self, real):
        self.real = real
        self.log = []

    def randint(self, a, b):
        r = self.real.randint(a, b)
        self.log.append(("randint", b - a + 1, r))
        return r

    def uniform(self, a, b):
        u = self.real.uniform(a, b)
        self.log.append(("uniform", None, u))
        return u


def make_trajectories(gc, cr, seeds, max_steps=5000):
    import random as real_random
    rec = _Recorder(real_random)
    gc.random = rec  # reference module attribute; restored below
    rows = {k: [] for k in ("seed", "episode", "t", "before", "action", "moved", "changed",
                            "n_blank", "rank", "four", "after", "done")}
    starts = {k: [] for k in ("seed", "episode", "board", "rank", "four")}
    try:
        for seed in seeds:
            real_random.seed(seed)
            for ep in range(2):  # two episodes back to back from one seed (main.py style, fresh Game)
                rec.log.clear()
                g = gc.Game()
                assert len(rec.log) == 2 and rec.log[0][1] == 16
                starts["seed"].append(seed); starts["episode"].append(ep)
                starts["board"].append(board_to_exp(g.state_matrix))
                starts["rank"].append(rec.log[0][2]); starts["four"].append(int(rec.log[1][2] <= 0.1))
                done, t = False, 0
                while not done and t < max_steps:
                    before = copy.deepcopy(g.state_matrix)
                    a_str = cr.Rand.random_action(before)
                    moved, _, changed = gc.Game.update_matrix(copy.deepcopy(before), a_str)
                    rec.log.clear()
                    state, reward, done = g.step(a_str)
                    assert reward == 0
                    if changed:
                        assert len(rec.log) == 2, rec.log
                        nb, rank = rec.log[0][1], rec.log[0][2]
                        four = int(rec.log[1][2] <= 0.1)
                    else:
                        assert len(rec.log) == 0
                        nb, rank, four = sum(1 for r in moved for v in r if v == 0), -1, -1
                    for k, v in (("seed", seed), ("episode", ep), ("t", t),
                                 ("before", board_to_exp(before)), ("action", DIRS[a_str]),
                                 ("moved", board_to_exp(moved)), ("changed", int(bool(changed))),
                                 ("n_blank", nb), ("rank", rank), ("four", four),
                                 ("after", board_to_exp(state)), ("done", int(done))):
                        rows[k].append(v)
                    t += 1
    finally:
        gc.random = real_random
    arr = {"step_" + k: np.asarray(v, dtype=np.int8 if k in ("before", "moved", "after") else np.int32)
           for k, v in rows.items()}
    arr.update({"start_" + k: np.asarray(v, dtype=np.int8 if k == "board" else np.int32)
                for k, v in starts.items()})
    return arr


# ---------------------------------------------------------------- line table
def line_table_sha(gc):
    """Exhaustive: every line of 4 cells with exponents 0..17, every direction, through the
    reference update_matrix on a 1x4 (LEFT/RIGHT) or 4x1 (UP/DOWN) matrix. Table layout:
    int8[4 dir][18^4 line][4 cell] (+ uint8 changed[4][18^4]) in index order
    line = ((c0*18 + c1)*18 + c2)*18 + c3, cells listed in the move's line order."""
    import itertools
    n = 18 ** 4
    out = np.zeros((4, n, 4), np.int8)
    chg = np.zeros((4, n), np.uint8)
    for idx, cells in enumerate(itertools.product(range(18), repeat=4)):
        vals = [0 if e == 0 else (1 << e) for e in cells]
        for d, a in ((0, "UP"), (1, "DOWN"), (2, "LEFT"), (3, "RIGHT")):
            if d < 2:
                m = [[v] for v in vals]
            else:
                m = [list(vals)]
            res, _, c = gc.Game.update_matrix(m, a)
            flat = [r[0] for r in res] if d < 2 else res[0]
            out[d, idx] = [exp_of(v) for v in flat]
            chg[d, idx] = 1 if c else 0
    h = hashlib.sha256()
    h.update(out.tobytes()); h.update(chg.tobytes())
    return {"layout": "int8[4][18^4][4] then uint8 changed[4][18^4]; dir 0=UP 1=DOWN 2=LEFT 3=RIGHT; "
                      "line index = ((c0*18+c1)*18+c2)*18+c3 with c0 the first cell of the matrix "
                      "(top for UP/DOWN, left for LEFT/RIGHT)",
            "sha256": h.hexdigest(), "n_lines": n,
            "sample_rows": {str(i): {"cells": [int(x) for x in np.unravel_index(i, (18,) * 4)],
                                     "out": out[:, i].tolist(), "changed": chg[:, i].tolist()}
                            for i in (0, 1, 18 + 1, 5 * 18 ** 3 + 5 * 18 ** 2 + 5 * 18 + 5, n - 1)}}


# ---------------------------------------------------------------- fingerprint
def fingerprint(gc, cr, seeds=range(100, 108), episodes=2500):
    import random as real_random
    lens, scores, maxt, noop, steps = [], [], [], 0, 0
    for s in seeds:
        real_random.seed(s)
        for _ in range(episodes):
            g = gc.Game()
            done, t = False, 0
            while not done:
                before = copy.deepcopy(g.state_matrix)
                state, _, done = g.step(cr.Rand.random_action(g.state_matrix))
                if state == before:
                    noop += 1
                t += 1
            steps += t
            lens.append(t)
            scores.append(int(np.sum(g.state_matrix)))
            maxt.append(int(max(max(r) for r in g.state_matrix)))
    lens, scores, maxt = map(np.asarray, (lens, scores, maxt))
    hist = {int(k): int(v) for k, v in zip(*np.unique(maxt, return_counts=True))}
    st = lambda x: {"mean": float(x.mean()), "sd": float(x.std(ddof=1)), "min": int(x.min()), "max": int(x.max())}
    return {"seeds": list(seeds), "episodes_per_seed": episodes, "n_episodes": int(lens.size),
            "episode_length": st(lens), "score": st(scores), "max_tile": st(maxt),
            "max_tile_hist": hist, "noop_fraction": noop / steps, "total_steps": int(steps),
            "episode_length_hist": {int(k): int(v) for k, v in zip(*np.unique(lens, return_counts=True))}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-fingerprint", action="store_true")
    ap.add_argument("--skip-table", action="store_true")
    args = ap.parse_args()
    gc, cr = _import_reference()
    kats = make_kats(gc)
    json.dump(kats, open(os.path.join(HERE, "kats.json"), "w"), indent=1)
    print("kats:", len(kats["line_moves"]), "line moves,", len(kats["filled"]), "filled,",
          len(kats["game_over"]), "game-over")
    traj = make_trajectories(gc, cr, seeds=range(64))
    np.savez_compressed(os.path.join(HERE, "trajectories.npz"), **traj)
    print("trajectories:", traj["step_t"].size, "steps")
    if not args.skip_table:
        tab = line_table_sha(gc)
        json.dump(tab, open(os.path.join(HERE, "line_table.json"), "w"), indent=1)
        print("line table sha256:", tab["sha256"])
    if not args.skip_fingerprint:
        fp = fingerprint(gc, cr)
        json.dump(fp, open(os.path.join(HERE, "fingerprint.json"), "w"), indent=1)
        print("fingerprint:", fp["episode_length"], fp["noop_fraction"])


if __name__ == "__main__":
    main()
