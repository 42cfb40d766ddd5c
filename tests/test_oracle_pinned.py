"""The oracle is pinned to the reference before anything is checked against it (CPU).

Fixtures in tests/golden/ were produced by running the reference (nevertiree/Rein48
game/GameClient.py + control/rand.py) in the build container; see make_golden.py.
"""
import hashlib
import random

import numpy as np
import pytest

from oracle import game_port, native as O
from conftest import to_exp_scaled

DIR = {"U": 0, "UP": 0, "D": 1, "DOWN": 1, "L": 2, "LEFT": 2, "R": 3, "RIGHT": 3}


def test_line_kats(golden):
    """GameClientTest.py:49-331 -- 40 line moves (values x2 to be powers of two)."""
    kats = golden["kats"]["line_moves"]
    assert len(kats) == 40
    for k in kats:
        assert k["expected"] == k["reference_output"], k  # the reference agrees with its own KATs
        a = DIR[k["action"]]
        rows, cols = len(k["input"]), len(k["input"][0])
        cells = to_exp_scaled(k["input"])
        want = to_exp_scaled(k["expected"])
        line = cells if a in (0, 2) else cells[::-1]
        got, changed = O.move_line(line)
        got = list(got) if a in (0, 2) else list(got)[::-1]
        assert got == want, (k["test"], k["case"])
        assert changed == k["reference_changed"]
        assert (rows, cols) in ((4, 1), (1, 4))


def test_filled_and_game_over_kats(golden):
    """GameClientTest.py:10-31."""
    for k in golden["kats"]["filled"]:
        assert O.filled(to_exp_scaled(k["input"])) == k["expected"]
    for k in golden["kats"]["game_over"]:
        assert O.game_over(to_exp_scaled(k["input"])) == k["expected"]


def test_exhaustive_line_table_matches_reference(golden):
    """All 18^4 lines x 4 directions through the reference's update_matrix -> SHA-256."""
    out, chg = O.line_table()
    h = hashlib.sha256()
    h.update(out.tobytes())
    h.update(chg.tobytes())
    assert h.hexdigest() == golden["table"]["sha256"]
    for idx, row in golden["table"]["sample_rows"].items():
        assert out[:, int(idx)].tolist() == row["out"]


def test_reference_trajectories_replay_bit_exact(golden):
    """128 seeded reference episodes (main.py loop, Rand policy) replayed by the oracle's
    CPython-compatible MT19937: every board, action, draw and done flag."""
    z = golden["traj"]
    for seed in range(64):
        rng = O.PyRand(seed)
        for ep in range(2):
            e = rng.episode()
            m = (z["step_seed"] == seed) & (z["step_episode"] == ep)
            sm = (z["start_seed"] == seed) & (z["start_episode"] == ep)
            assert np.array_equal(e["start"], z["start_board"][sm][0])
            for k in ("before", "action", "after", "done", "rank", "four", "changed"):
                assert np.array_equal(e[k], z["step_" + k][m].astype(e[k].dtype)), (seed, ep, k)


def test_moved_boards_match_reference(golden):
    z = golden["traj"]
    for i in range(0, len(z["step_t"]), 7):
        b, c = O.move(z["step_before"][i], z["step_action"][i])
        assert np.array_equal(b, z["step_moved"][i])
        assert c == bool(z["step_changed"][i])


def test_cpython_random_compat():
    for seed in (0, 1, 1234, 2 ** 32 + 5):
        random.seed(seed)
        r = O.PyRand(seed)
        for n in (1, 2, 3, 4, 15, 16):
            assert r.randbelow(n) == random.randrange(n)
        assert r.random() == random.random()
        assert r.getrandbits(7) == random.getrandbits(7)


def test_philox_known_answers():
    """Random123 philox4x32-10 KAT vectors."""
    assert O.philox([0, 0, 0, 0], [0, 0]).tolist() == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert O.philox([0xffffffff] * 4, [0xffffffff] * 2).tolist() == [0x408f276d, 0x41c83b0e, 0xa20bc7c6,
                                                                     0x6d5451fd]
    assert O.philox([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0]).tolist() == \
        [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


def _philox_py(ctr, key, rounds):
    """Philox4x32-R restated in plain Python from the Random123 paper (Salmon et al., SC'11): the
    check of the oracle's round-count parameter (Random123's KATs above cover 10 rounds only)."""
    c0, c1, c2, c3 = ctr
    k0, k1 = key
    m = 0xFFFFFFFF
    for _ in range(rounds):
        p0, p1 = 0xD2511F53 * c0, 0xCD9E8D57 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & m, p1 & m, ((p0 >> 32) ^ c3 ^ k1) & m, p0 & m
        k0, k1 = (k0 + 0x9E3779B9) & m, (k1 + 0xBB67AE85) & m
    return [c0, c1, c2, c3]


def test_philox_rounds_parameter():
    """The oracle's Philox4x32-R (draw contract 3: the env step's draws use R = 7) equals the
    plain-Python restatement, which itself reproduces the 10-round KATs."""
    assert _philox_py([0, 0, 0, 0], [0, 0], 10) == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    rng = np.random.default_rng(7)
    for _ in range(64):
        ctr = [int(v) for v in rng.integers(0, 2 ** 32, 4)]
        key = [int(v) for v in rng.integers(0, 2 ** 32, 2)]
        for rounds in (7, 10):
            assert O.philox(ctr, key, rounds).tolist() == _philox_py(ctr, key, rounds), (ctr, key, rounds)


def test_python_port_matches_reference_trajectories(golden):
    """oracle/game_port.py (the CPU baseline) plays the same seeded games as the reference."""
    z = golden["traj"]
    for seed in range(0, 64, 4):
        random.seed(seed)
        for ep in range(2):
            g = game_port.PortGame()
            m = (z["step_seed"] == seed) & (z["step_episode"] == ep)
            after = z["step_after"][m]
            for t in range(after.shape[0]):
                _, _, done = g.step(game_port.random_action(g.state_matrix))
                exps = [0 if v == 0 else int(v).bit_length() - 1 for r in g.state_matrix for v in r]
                assert exps == after[t].tolist(), (seed, ep, t)
            assert done


def test_philox_mode_matches_reference_fingerprint(golden):
    """The kernel's Philox draw contract (restated in the oracle) reproduces the reference's
    random-policy statistics: episode length over complete episodes that start in the first
    window (no truncation bias)."""
    fp = golden["fingerprint"]
    n, T, start_window = 2048, 1400, 700
    boards = O.reset_philox(np.zeros((n, 16), np.int8), seed=77, reset_ctr=0)
    start = np.zeros(n, np.int64)
    lengths = []
    for t in range(T):
        r = O.step_philox(boards, seed=77, step=t, flags=O.AUTO_RESET | O.RANDOM_POLICY)
        boards = r["boards"]
        d = np.nonzero(r["done"])[0]
        for i in d:
            if start[i] < start_window:
                lengths.append(t + 1 - start[i])
        start[d] = t + 1
    lengths = np.asarray(lengths, np.float64)
    ref = fp["episode_length"]
    se = np.sqrt(ref["sd"] ** 2 / lengths.size + ref["sd"] ** 2 / fp["n_episodes"])
    assert lengths.size > 5000
    assert abs(lengths.mean() - ref["mean"]) < 4 * se, (lengths.mean(), ref["mean"], se)
    assert abs(lengths.std(ddof=1) - ref["sd"]) < 0.05 * ref["sd"]


def test_philox_mode_matches_whole_reference_fingerprint(golden):
    """Draw contract 3 (Philox4x32-7 step draws, r48_board.h kStepRounds) against every statistic of
    the reference fingerprint (tests/fingerprint_check.py): episode-length histogram (chi-square),
    score mean / sd, max-tile histogram (chi-square) and the no-op fraction. Boards are stepped
    without auto-reset so that the final board of every episode is seen, then reset by the masked
    Philox reset (GameClient.py:33-38's contract, r48_env_reset)."""
    from fingerprint_check import check
    n, T, window = 4096, 1400, 700
    seed = 0x5EED7
    boards = O.reset_philox(np.zeros((n, 16), np.int8), seed=seed, reset_ctr=0)
    start = np.zeros(n, np.int64)
    noop = np.zeros(n, np.int64)
    L, S, M, N = [], [], [], []
    for t in range(T):
        r = O.step_philox(boards, seed=seed, step=t, flags=O.RANDOM_POLICY, want_score=True)
        noop += r["changed"] == 0
        d = np.nonzero(r["done"])[0]
        keep = d[start[d] < window]
        L.append(t + 1 - start[keep])
        S.append(r["score"][keep])
        M.append(1 << r["boards"][keep].max(1).astype(np.int64))
        N.append(noop[keep].copy())
        start[d] = t + 1
        noop[d] = 0
        boards = O.reset_philox(r["boards"], seed=seed, reset_ctr=t + 1, mask=r["done"]) if d.size else r["boards"]
    res = check(golden["fingerprint"], *(np.concatenate(x) for x in (L, S, M, N)), sd_tol=0.05)
    assert res["episodes"] > 15_000, res


def test_oracle_rejects_bad_action():
    with pytest.raises(ValueError):
        O.move(np.zeros(16, np.int8), 7)


def test_fill_random_distribution():
    """Synthetic bench boards (no reference counterpart -- statistics only):
    cells empty w.p. 1/2, tiles uniform over 1..max_exp, shard-independent."""
    b = O.fill_random(200_000, 0x20485EED, 7)
    assert abs((b == 0).mean() - 0.5) < 0.003
    counts = np.bincount(b[b > 0].astype(np.int64), minlength=8)[1:]
    exp = counts.sum() / 7
    chi2 = float(((counts - exp) ** 2 / exp).sum())
    assert chi2 < 30, chi2                        # 6 dof; p ~ 4e-5
    assert np.array_equal(O.fill_random(100, 0x20485EED, 7, board_offset=5000), b[5000:5100])
