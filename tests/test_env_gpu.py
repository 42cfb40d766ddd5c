"""GPU parity of the hot path: librein48.so's gfx950 kernels vs the oracle and the reference.

Bit-exact everywhere (integer/byte work). Covers: the reference's KATs, the exhaustive
18^4-line table, 128 seeded reference episodes replayed with the reference's own draws,
Philox mode vs the oracle (random policy, given actions incl. bad bytes, merge reward,
auto-reset, score), reset, move/spawn halves, rollout == repeated steps, sharding
invariance, full-size (2^20 boards) properties, and the random-policy fingerprint.
"""
import numpy as np
import pytest
import torch

from oracle import native as O
from conftest import to_exp_scaled

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def vec(n, seed=0, offset=0):
    from rein48_amd import VecGame
    return VecGame(n, device=DEV, seed=seed, board_offset=offset)


def rand_boards(rng, n, emax=9, p_empty=0.5):
    b = rng.integers(1, emax + 1, size=(n, 16)).astype(np.int8)
    b[rng.random((n, 16)) < p_empty] = 0
    return b


def put(v, boards):
    v.boards.copy_(torch.from_numpy(np.ascontiguousarray(boards, np.int8)).to(DEV))


def host(t):
    return t.detach().cpu().numpy()


# ---------------------------------------------------------------- reference KATs / table
def test_line_kats_on_gpu(golden):
    """GameClientTest.py:49-331 through the exponent kernel (values x2) and through the
    value-domain kernel with the KATs' raw values (1, 2, 4, ...)."""
    from rein48_amd.game import Game
    kats = golden["kats"]["line_moves"]
    code = {"U": 0, "D": 1, "LEFT": 2, "R": 3}
    boards, acts, want = [], [], []
    for k in kats:
        a = code[k["action"]]
        cells = to_exp_scaled(k["input"])
        b = np.zeros(16, np.int8)
        exp = np.zeros(16, np.int8)
        w = to_exp_scaled(k["expected"])
        for i in range(4):
            if a < 2:
                b[4 * i + 1], exp[4 * i + 1] = cells[i], w[i]
            else:
                b[4 + i], exp[4 + i] = cells[i], w[i]
        boards.append(b)
        acts.append(a)
        want.append(exp)
    v = vec(len(kats))
    put(v, np.stack(boards))
    changed, _ = v.move(torch.tensor(acts, dtype=torch.int8, device=DEV))
    assert np.array_equal(host(v.boards), np.stack(want))
    assert host(changed).astype(bool).tolist() == [k["reference_changed"] for k in kats]
    # the drop-in static method on the raw KAT matrices (value 1 and all)
    for k in kats:
        m = [list(r) for r in k["input"]]
        out, reward, changed = Game.update_matrix(m, k["action"])
        assert out == k["expected"] and out is m and reward == 0 and changed == k["reference_changed"]


def test_filled_game_over_kats_on_gpu(golden):
    from rein48_amd.game import Game
    for k in golden["kats"]["filled"]:
        assert Game.has_table_filled(k["input"]) == k["expected"]
    for k in golden["kats"]["game_over"]:
        assert Game.has_game_over(k["input"]) == k["expected"]


def test_exhaustive_line_table_on_gpu():
    """Every line of 4 cells with exponents 0..17, every direction: GPU == reference table."""
    out, chg = O.line_table()
    n = O.LINE_TABLE_N
    idx = np.arange(n)
    cells = np.stack([(idx // 18 ** (3 - k)) % 18 for k in range(4)], axis=1).astype(np.int8)
    for d in range(4):
        nb = n // 4  # 18^4 is divisible by 4: four lines per board
        b = np.zeros((nb, 4, 4), np.int8)
        want = np.zeros((nb, 4, 4), np.int8)
        c4 = cells.reshape(nb, 4, 4)       # [board, slot, cell]
        o4 = out[d].reshape(nb, 4, 4)
        if d < 2:   # columns
            b[:] = np.transpose(c4, (0, 2, 1))
            want[:] = np.transpose(o4, (0, 2, 1))
        else:       # rows
            b[:] = c4
            want[:] = o4
        v = vec(nb)
        put(v, b.reshape(nb, 16))
        changed, _ = v.move(torch.full((nb,), d, dtype=torch.int8, device=DEV))
        assert np.array_equal(host(v.boards), want.reshape(nb, 16)), d
        any_chg = chg[d].reshape(nb, 4).max(axis=1)
        assert np.array_equal(host(changed), any_chg), d


# ---------------------------------------------------------------- reference trajectories
def test_reference_trajectories_replayed_with_injected_draws(golden):
    """All 128 reference episodes in lockstep: start board from reset_with_draws with the
    reference's first two draws, then each step with the reference's action, randint rank
    and uniform-derived 4/2 flag: every board and done flag bit-exact."""
    z = golden["traj"]
    keys = list(zip(z["start_seed"].tolist(), z["start_episode"].tolist()))
    ne = len(keys)
    lens = [int(((z["step_seed"] == s) & (z["step_episode"] == e)).sum()) for s, e in keys]
    T = max(lens)
    act = np.zeros((T, ne), np.int8)
    rank = np.zeros((T, ne), np.uint8)
    four = np.zeros((T, ne), np.uint8)
    after = np.zeros((T, ne, 16), np.int8)
    done = np.zeros((T, ne), np.uint8)
    for j, (s, e) in enumerate(keys):
        m = (z["step_seed"] == s) & (z["step_episode"] == e)
        L = lens[j]
        act[:L, j] = z["step_action"][m]
        rank[:L, j] = np.maximum(z["step_rank"][m], 0)
        four[:L, j] = np.maximum(z["step_four"][m], 0)
        after[:L, j] = z["step_after"][m]
        done[:L, j] = z["step_done"][m]
    v = vec(ne)
    v.reset_with_draws(torch.tensor(z["start_rank"], dtype=torch.uint8, device=DEV),
                       torch.tensor(z["start_four"], dtype=torch.uint8, device=DEV))
    assert np.array_equal(host(v.boards), z["start_board"])
    for t in range(T):
        v.step_with_draws(torch.from_numpy(act[t]).to(DEV), torch.from_numpy(rank[t]).to(DEV),
                          torch.from_numpy(four[t]).to(DEV))
        live = np.array([t < L for L in lens])
        assert np.array_equal(host(v.boards)[live], after[t][live]), t
        assert np.array_equal(host(v.done)[live], done[t][live]), t


def test_drop_in_game_reproduces_reference_episodes(golden):
    """rein48_amd.game.Game + rein48_amd.control.Rand under random.seed(s): the reference's
    exact episodes (main.py:36-42 loop), with state aliasing preserved."""
    import random
    from rein48_amd.control import Rand
    from rein48_amd.game import Game
    z = golden["traj"]
    for seed in range(6):
        random.seed(seed)
        for ep in range(2):
            g = Game()
            sm = (z["start_seed"] == seed) & (z["start_episode"] == ep)
            m = (z["step_seed"] == seed) & (z["step_episode"] == ep)
            assert to_exp_list(g.state_matrix) == z["start_board"][sm][0].tolist()
            after, dn = z["step_after"][m], z["step_done"][m]
            state0 = g.state_matrix
            for t in range(after.shape[0]):
                state, reward, done = g.step(Rand.random_action(g.state_matrix))
                assert state is state0 and reward == 0
                assert to_exp_list(state) == after[t].tolist(), (seed, ep, t)
                assert done == bool(dn[t])


def to_exp_list(m):
    return [0 if v == 0 else int(v).bit_length() - 1 for r in m for v in r]


def test_game_step1_candidates_equal_injected_draw_steps():
    """r48_game_step1 (the drop-in Game.step's one launch): candidate 2r + f equals the injected-draw
    step (rank r, tile 2 or 4) of the same board, and its game-over bit equals that step's done, for
    every blank rank, on random boards incl. full ones (unchanged moves: every candidate is the
    unchanged board) and every action."""
    from rein48_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(11)
    boards = np.concatenate([rand_boards(rng, 60), rand_boards(rng, 20, emax=3, p_empty=0.0),
                             rand_boards(rng, 20, p_empty=0.85)])
    nb = int(lib.r48_game_step1_out_bytes())
    out = torch.empty(nb, dtype=torch.uint8, device=DEV)
    env = vec(32)
    ranks = torch.arange(32, device=DEV, dtype=torch.int32).div(2, rounding_mode="floor").to(torch.uint8)
    fours = (torch.arange(32, device=DEV) % 2).to(torch.uint8)
    for i, b in enumerate(boards):
        for a in range(4):
            bb = np.ascontiguousarray(b)
            _lib.check(lib.r48_game_step1(bb.ctypes.data, a, out.data_ptr(), torch.cuda.current_stream().cuda_stream))
            h = out.cpu().numpy()
            changed, n_blank = int(h[512]), int(h[513])
            mask = int.from_bytes(h[516:520].tobytes(), "little")
            env.boards.copy_(torch.from_numpy(np.repeat(b[None], 32, 0)))
            _, _, done = env.step_with_draws(torch.full((32,), a, dtype=torch.int8, device=DEV), ranks, fours)
            ref = env.boards.cpu().numpy()
            assert changed == int(env.changed[0])
            for c in range(32):
                if changed and (c >> 1) >= n_blank:
                    continue
                assert np.array_equal(h[16 * c:16 * c + 16].view(np.int8), ref[c]), (i, a, c)
                assert (mask >> c & 1) == int(done[c]), (i, a, c)
            if changed:
                assert n_blank == int((ref[0] == 0).sum()) + 1


def test_drop_in_game_surface():
    from rein48_amd.game import Game
    g = Game()
    assert (g.action_space_size, g.reward_space_size, g.state_space_size) == (4, 1, 4)
    assert sum(v != 0 for r in g.state_matrix for v in r) == 1
    for bad in ("X", 4, -1, None, "upward"):
        with pytest.raises(ValueError):
            g.step(bad)
    for alias in ("Up", "d", "LEFT", "r", 0, 1, 2, 3, True, 2.0):
        g.step(alias)
    g5 = Game(5)
    assert g5.state_space_size == 5 and len(g5.state_matrix) == 5 and len(g5.state_matrix[0]) == 5
    assert sum(v != 0 for r in g5.state_matrix for v in r) == 1
    assert Game(3).state_space_size == 4


@pytest.mark.parametrize("size", [5, 6, 9])
def test_drop_in_game_larger_boards_follow_reference_rules(size):
    """Game(n > 4) (GameClient.py:19-27 accepts any n >= 4): the value-domain grid kernels + the
    host spawn draws reproduce the reference rules under random.seed -- checked against
    oracle/game_port.PortGame(n), the pure-Python restatement of the reference Game, step for
    step with the same seeds (parity pinned to the 4x4 reference fixtures through the port;
    the reference ships no n > 4 fixtures)."""
    import random
    from oracle.game_port import PortGame, random_action
    from rein48_amd.game import Game
    for seed in range(3):
        random.seed(seed)
        g = Game(size)
        state = [r[:] for r in g.state_matrix]
        random.seed(seed)
        p = PortGame(size)
        assert p.state_matrix == state
        for t in range(400):
            st = random.getstate()
            a = random_action()
            s1, _, d1 = g.step(a)
            random.setstate(st)
            a2 = random_action()
            s2, _, d2 = p.step(a2)
            assert a == a2 and s1 == s2 and d1 == d2, (size, seed, t)
            if d1:
                break


def test_static_helpers_on_any_shape():
    """update_matrix / has_game_over / has_table_filled on rectangular matrices beyond 4x4
    (r48_values_move_grid / r48_values_check_grid) == the port's restatement."""
    from oracle.game_port import PortGame
    from rein48_amd.game import Game
    rng = np.random.default_rng(3)
    for rows, cols in ((5, 7), (1, 9), (9, 1), (6, 6), (12, 5)):
        for _ in range(30):
            m = (2 ** rng.integers(0, 4, size=(rows, cols))) * (rng.random((rows, cols)) < 0.6)
            m = m.astype(int).tolist()
            for a in range(4):
                want = [r[:] for r in m]
                _, _, wc = PortGame.move(want, a)
                got = [r[:] for r in m]
                rows_before = [id(r) for r in got]
                _, rw, gc = Game.update_matrix(got, a)
                assert got == want and gc == wc and rw == 0, (rows, cols, a)
                assert [id(r) for r in got] == rows_before          # mutated in place
        full = (2 ** (1 + (np.arange(36).reshape(6, 6) % 5))).tolist()     # no equal neighbours? check
        assert Game.has_table_filled(full)
        over_want = PortGame.over(full)
        assert Game.has_game_over(full) == over_want
        full[2][3] = 0
        assert not Game.has_table_filled(full) and not Game.has_game_over(full)


def _ref_game_over(m):
    """GameClient.py:65-100 restated literally: has_table_filled over every item, then i and j
    over range(len(m)) (the row count) -- on a non-square matrix a leading square block, or an
    IndexError when the rows outnumber the columns."""
    if 0 in [x for row in m for x in row]:
        return False
    n = len(m)
    for i in range(n):
        for j in range(n):
            if (i != 0 and m[i][j] == m[i - 1][j]) or (j != 0 and m[i][j] == m[i][j - 1]) or \
                    (i != n - 1 and m[i][j] == m[i + 1][j]) or (j != n - 1 and m[i][j] == m[i][j + 1]):
                return False
    return True


@pytest.mark.parametrize("rows,cols", [(2, 4), (3, 5), (1, 4), (4, 2), (6, 3), (5, 9)])
def test_game_over_on_non_square_matrices_follows_reference_loop(rows, cols):
    """has_game_over on rectangles (<= 4x4: r48_values_check; larger: r48_values_check_grid)
    reproduces the reference's square-index loop: columns past the row count are never compared,
    a zero anywhere means not over, and a filled matrix with more rows than columns raises
    IndexError like the reference unless its first row's scan meets an equal pair first."""
    from rein48_amd.game import Game
    rng = np.random.default_rng(rows * 31 + cols)
    for trial in range(40):
        m = (2 ** rng.integers(1, 5, size=(rows, cols))).astype(int)
        if trial % 4 == 0:          # equal neighbours only beyond the leading square block
            m = (2 ** (1 + (np.add.outer(np.arange(rows), np.arange(cols)) % 2) * 3 +
                       (np.arange(cols)[None, :] >= rows) * 0)).astype(int)
            if cols > rows:
                m[:, rows:] = 2
        if trial % 5 == 1:
            m[rng.integers(rows), rng.integers(cols)] = 0
        m = m.tolist()
        try:
            want = _ref_game_over(m)
        except IndexError:
            with pytest.raises(IndexError):
                Game.has_game_over(m)
            continue
        assert Game.has_game_over(m) == want, (rows, cols, m)
        assert Game.has_table_filled(m) == (0 not in [x for r in m for x in r])


# ---------------------------------------------------------------- Philox mode vs oracle
@pytest.mark.parametrize("off", [12345, 1 << 20])   # odd: guarded per-board path; even: pair fast path
@pytest.mark.parametrize("flags", [O.RANDOM_POLICY, O.RANDOM_POLICY | O.AUTO_RESET,
                                   O.RANDOM_POLICY | O.AUTO_RESET | O.MERGE_REWARD])
def test_philox_random_policy_matches_oracle(flags, off):
    rng = np.random.default_rng(flags)
    n, seed = 100_003, 0x2048_5EED
    b0 = rand_boards(rng, n)
    v = vec(n, seed=seed, offset=off)
    put(v, b0)
    ob = b0
    score = torch.zeros(n, dtype=torch.int32, device=DEV)
    for step in range(4):
        v.step(None, auto_reset=bool(flags & O.AUTO_RESET), merge_reward=bool(flags & O.MERGE_REWARD),
               want_changed=True, score=score)
        r = O.step_philox(ob, seed, step, flags, board_offset=off, want_score=True)
        ob = r["boards"]
        assert np.array_equal(host(v.boards), ob), step
        assert np.array_equal(host(v.actions), r["actions"])
        assert np.array_equal(host(v.done), r["done"])
        assert np.array_equal(host(v.changed), r["changed"])
        assert np.array_equal(host(score), r["score"])
        if flags & O.MERGE_REWARD:
            assert np.array_equal(host(v.reward), r["reward"])
    assert v.counters == (4, 0)


def test_given_actions_with_bad_bytes_match_oracle():
    rng = np.random.default_rng(5)
    n = 65_536
    b0 = rand_boards(rng, n, emax=17, p_empty=0.3)
    acts = rng.integers(0, 4, n).astype(np.int8)
    bad = rng.random(n) < 0.01
    acts[bad] = rng.choice(np.array([-128, -1, 4, 5, 100, 127], np.int8), bad.sum())
    v = vec(n, seed=99)
    put(v, b0)
    v.error_count(clear=True)
    v.step(torch.from_numpy(acts).to(DEV), merge_reward=True, want_changed=True)
    r = O.step_philox(b0, 99, 0, O.MERGE_REWARD, actions=acts)
    assert np.array_equal(host(v.boards), r["boards"])
    assert np.array_equal(host(v.done), r["done"])
    assert np.array_equal(host(v.changed), r["changed"])
    assert np.array_equal(host(v.reward), r["reward"])
    assert np.array_equal(host(v.boards)[bad], b0[bad])  # a bad action leaves the board as it was
    assert v.error_count() == int(bad.sum()) == r["bad"]


def test_injected_draws_match_oracle():
    rng = np.random.default_rng(11)
    n = 50_000
    b0 = rand_boards(rng, n)
    acts = rng.integers(0, 4, n).astype(np.int8)
    rank = rng.integers(0, 256, n).astype(np.uint8)
    four = rng.integers(0, 2, n).astype(np.uint8)
    v = vec(n)
    put(v, b0)
    v.step_with_draws(torch.from_numpy(acts).to(DEV), torch.from_numpy(rank).to(DEV),
                      torch.from_numpy(four).to(DEV), merge_reward=True)
    r = O.step_draws(b0, acts, rank, four, flags=O.MERGE_REWARD)
    assert np.array_equal(host(v.boards), r["boards"])
    assert np.array_equal(host(v.done), r["done"])
    assert np.array_equal(host(v.changed), r["changed"])
    assert np.array_equal(host(v.reward), r["reward"])


def test_move_then_spawn_equals_step_with_draws():
    rng = np.random.default_rng(12)
    n = 40_000
    b0 = rand_boards(rng, n)
    acts = torch.from_numpy(rng.integers(0, 4, n).astype(np.int8)).to(DEV)
    rank = torch.from_numpy(rng.integers(0, 256, n).astype(np.uint8)).to(DEV)
    four = torch.from_numpy(rng.integers(0, 2, n).astype(np.uint8)).to(DEV)
    a, b = vec(n), vec(n)
    put(a, b0)
    put(b, b0)
    changed, n_blank = a.move(acts)
    moved = host(a.boards)
    assert np.array_equal(host(n_blank), (moved == 0).sum(1))
    a.spawn(rank, four, mask=changed.clone())
    b.step_with_draws(acts, rank, four)
    assert np.array_equal(host(a.boards), host(b.boards))
    assert np.array_equal(host(a.done), host(b.done))


def test_reset_matches_oracle():
    n, seed = 70_000, 31337
    v = vec(n, seed=seed, offset=7)
    mask = (np.arange(n) % 3 != 0).astype(np.uint8)
    put(v, np.full((n, 16), 5, np.int8))
    v.reset()
    v.reset(mask=torch.from_numpy(mask).to(DEV))
    ob = O.reset_philox(np.full((n, 16), 5, np.int8), seed, 0, board_offset=7)
    ob = O.reset_philox(ob, seed, 1, mask=mask, board_offset=7)
    assert np.array_equal(host(v.boards), ob)
    nz = (ob != 0).sum(1)
    assert (nz == 1).all()
    assert v.counters == (0, 2)


@pytest.mark.parametrize("max_exp", [7, 17])
def test_fill_random_matches_oracle(max_exp):
    """Synthetic start boards: bit-exact vs the oracle, independent of the
    shard split (board_offset), counters untouched, then a step runs from them."""
    n, seed = 50_001, 0x20485EED
    v = vec(n, seed=seed, offset=123)
    v.fill_random(max_exp)
    want = O.fill_random(n, seed, max_exp, board_offset=123)
    assert np.array_equal(host(v.boards), want)
    lo = vec(1000, seed=seed, offset=123 + 20_000)
    lo.fill_random(max_exp)
    assert np.array_equal(host(lo.boards), want[20_000:21_000])
    assert v.counters == (0, 0)
    assert abs((want == 0).mean() - 0.5) < 0.01 and want.max() == max_exp and want[want > 0].min() == 1
    with pytest.raises(Exception):
        v.fill_random(0)


# pair fast path (even n, even offset) / byte-stored trajectory rows inside the fast path (odd n,
# even offset) / guarded per-board path (odd offset)
@pytest.mark.parametrize("n,offset", [(30_000, 98), (30_001, 98), (30_001, 97)])
def test_rollout_equals_repeated_steps(n, offset):
    K, seed = 37, 4242
    rng = np.random.default_rng(3)
    b0 = rand_boards(rng, n, emax=6, p_empty=0.4)
    a, b = vec(n, seed=seed, offset=offset), vec(n, seed=seed, offset=offset)
    put(a, b0)
    put(b, b0)
    acts = torch.empty((K, n), dtype=torch.int8, device=DEV)
    dn = torch.empty((K, n), dtype=torch.uint8, device=DEV)
    a.rollout(K, actions=acts, done=dn)
    for t in range(K):
        b.step(None, auto_reset=True)
        assert torch.equal(acts[t], b.actions) and torch.equal(dn[t], b.done), t
    assert torch.equal(a.boards, b.boards)
    assert a.counters == b.counters == (K, 0)


def test_sharded_envs_equal_one_env():
    """Philox keyed by global board id: two half-size shards == one env (multi-GPU invariance)."""
    n, seed = 20_000, 8
    rng = np.random.default_rng(8)
    b0 = rand_boards(rng, n)
    whole = vec(n, seed=seed)
    lo, hi = vec(n // 2, seed=seed, offset=0), vec(n // 2, seed=seed, offset=n // 2)
    put(whole, b0)
    put(lo, b0[: n // 2])
    put(hi, b0[n // 2:])
    for _ in range(5):
        for e in (whole, lo, hi):
            e.step(None, auto_reset=True)
    assert torch.equal(whole.boards, torch.cat([lo.boards, hi.boards]))


def test_score_matches_oracle():
    rng = np.random.default_rng(4)
    b0 = rand_boards(rng, 10_000, emax=17)
    v = vec(10_000)
    put(v, b0)
    assert np.array_equal(host(v.score()), O.score(b0))


# ---------------------------------------------------------------- full-size properties
def test_full_size_properties():
    """BASELINE config 2 size (2^20 boards): a move conserves the tile-value sum, a spawn adds
    exactly one 2 or 4 iff the board changed, a sampled subset is bit-exact vs the oracle,
    and the run is deterministic."""
    n = 1 << 20
    rng = np.random.default_rng(2048)
    b0 = rand_boards(rng, n, emax=7)
    acts = torch.from_numpy(rng.integers(0, 4, n).astype(np.int8)).to(DEV)
    v = vec(n, seed=1)
    put(v, b0)
    s0 = v.score().to(torch.int64)
    changed, _ = v.move(acts)
    s1 = v.score().to(torch.int64)
    assert torch.equal(s0, s1)
    put(v, b0)
    v.step(acts, want_changed=True)
    s2 = v.score().to(torch.int64)
    diff = s2 - s0
    ch = v.changed.to(torch.bool)
    assert torch.equal(ch, changed.to(torch.bool))
    assert bool(((diff == 2) | (diff == 4))[ch].all()) and bool((diff == 0)[~ch].all())
    nz_delta = (v.boards != 0).sum(1) - torch.from_numpy((b0 != 0).sum(1)).to(DEV)
    assert bool((nz_delta <= 1).all())
    # sampled boards bit-exact vs the oracle (its draws are keyed by the global board id)
    got, ah = host(v.boards), host(acts)
    for i in rng.choice(n, 512, replace=False):
        rr = O.step_philox(b0[i:i + 1], 1, 0, 0, actions=ah[i:i + 1], board_offset=int(i))
        assert np.array_equal(got[i], rr["boards"][0])
    w = vec(n, seed=1)
    put(w, b0)
    w.step(acts)
    assert torch.equal(w.boards, v.boards)


def test_fingerprint_distribution_on_gpu(golden):
    """Random policy on 65,536 boards: episode length statistics over complete episodes that
    start in the first 1,000 steps (reference: mean 142.36, sd 47.27, 20,000 episodes)."""
    fp = golden["fingerprint"]
    n, T, window = 65_536, 3_000, 1_000
    v = vec(n, seed=2024)
    v.reset()
    dn = torch.empty((T, n), dtype=torch.uint8, device=DEV)
    v.rollout(T, done=dn)
    d = host(dn).astype(bool)
    lengths = []
    t_idx, b_idx = np.nonzero(d)
    order = np.lexsort((t_idx, b_idx))
    t_idx, b_idx = t_idx[order], b_idx[order]
    prev_b = -1
    for t, b in zip(t_idx, b_idx):
        if b != prev_b:
            s = 0
            prev_b = b
        if s < window:
            lengths.append(t + 1 - s)
        s = t + 1
    lengths = np.asarray(lengths, np.float64)
    from fingerprint_check import check_lengths
    assert lengths.size > 300_000
    print(check_lengths(fp, lengths))    # histogram chi-square, mean (4 SE), sd (3 %)
    assert lengths.min() >= 10 and lengths.max() < 1500


def test_whole_fingerprint_on_gpu(golden):
    """Draw contract 3 (the step's Philox4x32-7, r48_board.h kStepRounds) against EVERY statistic of
    the reference fingerprint (tests/fingerprint_check.py): episode-length histogram chi-square,
    score mean / sd, max-tile histogram chi-square, no-op fraction (0.1602) within 4 SE.
    k_step_n (the bench kernel, K = 1 per call) steps 65,536 boards without auto-reset so that the
    final board of every episode is seen; done boards are then reset by r48_env_reset (mask).
    Episodes counted: complete ones that start in the first 1,000 of 3,000 steps."""
    from fingerprint_check import check
    n, T, window = 65_536, 3_000, 1_000
    v = vec(n, seed=0x7E57)
    v.reset()
    sc = torch.zeros(n, dtype=torch.int32, device=DEV)
    start = torch.zeros(n, dtype=torch.int32, device=DEV)
    noop = torch.zeros(n, dtype=torch.int32, device=DEV)
    L = torch.zeros((T, n), dtype=torch.int16, device=DEV)     # 0: no counted episode ended here
    S = torch.zeros((T, n), dtype=torch.int32, device=DEV)
    M = torch.zeros((T, n), dtype=torch.int8, device=DEV)
    N = torch.zeros((T, n), dtype=torch.int16, device=DEV)
    zero = torch.zeros((), dtype=torch.int32, device=DEV)
    for t in range(T):
        v.step_n(1, auto_reset=False, want_changed=True, score=sc)
        noop += (v.changed == 0).to(torch.int32)
        d = v.done.bool()
        keep = d & (start < window)
        L[t] = torch.where(keep, (t + 1) - start, zero).to(torch.int16)
        S[t] = torch.where(keep, sc, zero)
        M[t] = torch.where(keep, v.boards.amax(1).to(torch.int32), zero).to(torch.int8)
        N[t] = torch.where(keep, noop, zero).to(torch.int16)
        start = torch.where(d, torch.full_like(start, t + 1), start)
        noop.masked_fill_(d, 0)
        v.reset(mask=v.done)
    m = L > 0
    lengths, scores = host(L[m]).astype(np.int64), host(S[m]).astype(np.int64)
    maxt, noops = 1 << host(M[m]).astype(np.int64), host(N[m]).astype(np.int64)
    assert lengths.size > 400_000, lengths.size
    res = check(golden["fingerprint"], lengths, scores, maxt, noops)
    print(res)


def test_input_validation():
    v = vec(8)
    with pytest.raises(TypeError):
        v.step(torch.zeros(8, dtype=torch.int32, device=DEV))
    with pytest.raises(ValueError):
        v.step(torch.zeros(7, dtype=torch.int8, device=DEV))
    with pytest.raises(ValueError):
        v.step(torch.zeros(8, dtype=torch.int8))  # host tensor


def _step_n_vs_steps(n, off, K, flags, seed, rng, actions=None, emax=8, p_empty=0.5):
    """step_n(K) on one env vs K single-step launches (k_step) on a twin: every output plane,
    the boards, the counters and the bad-action counter must be identical."""
    b0 = rand_boards(rng, n, emax=emax, p_empty=p_empty)
    a, b = vec(n, seed=seed, offset=off), vec(n, seed=seed, offset=off)
    put(a, b0)
    put(b, b0)
    kw = dict(auto_reset=bool(flags & O.AUTO_RESET), merge_reward=bool(flags & O.MERGE_REWARD), want_changed=True)
    sa = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    sb = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    acts = None if actions is None else torch.from_numpy(actions).to(DEV)
    _, ra, da = a.step_n(K, acts, score=sa, **kw)
    for _ in range(K):
        _, rb, db = b.step(acts, score=sb, **kw)
    torch.cuda.synchronize()
    assert torch.equal(a.boards, b.boards), (n, off, K)
    assert torch.equal(da, db) and torch.equal(ra, rb) and torch.equal(a.changed, b.changed)
    assert torch.equal(sa, sb) and torch.equal(a.actions, b.actions)
    assert a.counters == b.counters == (K, 0)
    assert a.error_count() == b.error_count()
    return a, b0


@pytest.mark.parametrize("off", [0, 3])              # even: pair fast path; odd: guarded per-board path
@pytest.mark.parametrize("K", [1, 2, 20, 4096])
def test_step_n_equals_repeated_steps(K, off):
    """r48_env_step_n (k_step_n: one launch, boards in VGPRs for all K steps) == K k_step
    launches, random policy + auto-reset + merge reward + changed + score, on a ragged size (the
    grid's partial last tile)."""
    rng = np.random.default_rng(K * 10 + off)
    _step_n_vs_steps(300_001, off, K, O.RANDOM_POLICY | O.AUTO_RESET | O.MERGE_REWARD, 77, rng)


@pytest.mark.parametrize("flags", [O.RANDOM_POLICY, O.RANDOM_POLICY | O.MERGE_REWARD])
@pytest.mark.parametrize("K", [1, 3, 20, 300])
def test_step_n_random_policy_without_auto_reset(K, flags):
    """Random policy WITHOUT auto-reset (VecGame.step_n's default): boards that end the call done
    are not reset, so k_step_n must return them to rows from the line form of their last action
    (not leave them transposed / reversed). Near-full boards (5 % blanks, exponents up to 12) so
    that many boards are done after a few steps, with every last action; == K single steps."""
    rng = np.random.default_rng(900 + K)
    a, _ = _step_n_vs_steps(100_003, 0, K, flags, 31, rng, emax=12, p_empty=0.05)
    done = host(a.done)
    assert done.mean() > 0.1, done.mean()
    acts = host(a.actions)[done != 0]
    assert len(np.unique(acts)) == 4   # done boards whose last action was each of the four


@pytest.mark.parametrize("flags", [0, O.AUTO_RESET | O.MERGE_REWARD])
def test_step_n_given_actions_with_bad_bytes(flags):
    """Given actions (constant over the K steps) incl. bytes outside 0..3: the board stays, and
    the error counter grows by K per bad byte, exactly as K single steps."""
    n, K = 70_001, 9
    rng = np.random.default_rng(5)
    acts = rng.integers(0, 4, n).astype(np.int8)
    acts[rng.random(n) < 0.05] = 7
    a, _ = _step_n_vs_steps(n, 0, K, flags, 12, rng, actions=acts)
    assert a.error_count() == K * int((acts > 3).sum())


@pytest.mark.parametrize("off", [0, 1])
def test_step_n_past_the_infinity_cache(off):
    """2^24 + 6 boards (268 MB of boards, more than the 256 MiB Infinity Cache; the size where
    round 1's step_n ping-ponged through a scratch copy): K = 20 and 4096 on the pair path, K = 20
    on the guarded path, == single steps."""
    n = (1 << 24) + 6
    rng = np.random.default_rng(off)
    for K in ((20, 4096) if off == 0 else (20,)):
        a, _ = _step_n_vs_steps(n, off, K, O.RANDOM_POLICY | O.AUTO_RESET, 4242, rng)
        del a
        torch.cuda.empty_cache()


@pytest.mark.parametrize("off", [3, 0])               # odd: guarded per-board path; even: pair fast path
@pytest.mark.parametrize("n", [300_001, 9_000_003])
def test_step_n_wide_envs_match_oracle(n, off):
    """Large envs, odd sizes (the partial tile): two step_n calls == eager steps == the oracle, on
    both the pair fast path (even offset) and the guarded path (odd offset)."""
    seed = 4040
    rng = np.random.default_rng(n)
    b0 = rand_boards(rng, n, emax=6)
    a, b = vec(n, seed=seed, offset=off), vec(n, seed=seed, offset=off)
    put(a, b0)
    put(b, b0)
    a.step_n(2, auto_reset=True)
    a.step_n(2, auto_reset=True)
    for _ in range(4):
        b.step(None, auto_reset=True)
    assert torch.equal(a.boards, b.boards)
    assert torch.equal(a.done, b.done) and torch.equal(a.actions, b.actions)
    want = b0
    for t in range(4):
        want = O.step_philox(want, seed, t, O.RANDOM_POLICY | O.AUTO_RESET, board_offset=off)["boards"]
    assert np.array_equal(host(a.boards), want)


def test_play_loop_matches_reference_score(golden):
    """main.py's play() with the rand policy under random.seed: same final score as the
    reference episode (tile sum, main.py:48)."""
    import random
    from rein48_amd.game import Game
    from rein48_amd.main import play
    z = golden["traj"]
    for seed in range(3):
        random.seed(seed)
        score = play(Game(), control="rand", show_result=False)
        m = (z["step_seed"] == seed) & (z["step_episode"] == 0)
        last = z["step_after"][m][-1].astype(np.int64)
        assert score == int(np.where(last > 0, 1 << last, 0).sum())


@pytest.mark.parametrize("n", [1, 2, 3, 511, 512, 513, 1025])
def test_tiny_and_ragged_envs_match_oracle(n):
    """Edge sizes (one board, a partial pair, a partial tile, one tile +- 1): eager steps under the
    random policy, given actions read through views at odd offsets (the pair path's 2-byte stores
    fall back to the per-board path for misaligned planes), and a step_n chunk, all == the oracle.
    Boards hold exponents up to 29, so merges reach 2^30 (the largest exponent the int8 cell and
    the int32 merge reward both hold)."""
    rng = np.random.default_rng(n)
    seed = 31337
    b0 = rand_boards(rng, n, emax=29, p_empty=0.3)
    v = vec(n, seed=seed)
    put(v, b0)
    ob = b0
    flags = O.RANDOM_POLICY | O.MERGE_REWARD
    v.step(None, merge_reward=True)
    r = O.step_philox(ob, seed, 0, flags)
    ob = r["boards"]
    assert np.array_equal(host(v.boards), ob) and np.array_equal(host(v.reward), r["reward"])
    # given actions and done/reward outputs through odd-offset views of larger buffers
    acts = rng.integers(0, 4, n).astype(np.int8)
    abuf = torch.zeros(n + 1, dtype=torch.int8, device=DEV)
    abuf[1:] = torch.from_numpy(acts).to(DEV)
    dbuf = torch.zeros(n + 1, dtype=torch.uint8, device=DEV)
    _, rew, done = v.step(abuf[1:], merge_reward=True, done_out=dbuf[1:])
    r = O.step_philox(ob, seed, 1, O.MERGE_REWARD, actions=acts)
    ob = r["boards"]
    assert np.array_equal(host(v.boards), ob)
    assert np.array_equal(host(done), r["done"]) and np.array_equal(host(rew), r["reward"])
    v.step_n(3, auto_reset=True)
    for k in range(3):
        ob = O.step_philox(ob, seed, 2 + k, O.RANDOM_POLICY | O.AUTO_RESET)["boards"]
    assert np.array_equal(host(v.boards), ob)
    assert v.counters == (5, 0)
