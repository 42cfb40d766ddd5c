"""ctypes/numpy wrapper of oracle/r48_oracle.c -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Builds the C oracle on first use if the shared object is missing (gcc, seconds).
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libr48oracle.so")
_lib = None

AUTO_RESET, RANDOM_POLICY, MERGE_REWARD = 1, 2, 4
LINE_TABLE_N = 18 ** 4


def build():
    src = os.path.join(_HERE, "r48_oracle.c")
    if not os.path.exists(_SO) or os.path.getmtime(_SO) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _SO


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(_SO)
        P = C.c_void_p
        sig = {
            "orc_move": (C.c_int, [P, C.c_int, P]),
            "orc_move_line": (C.c_int, [P, C.c_int]),
            "orc_line_table": (None, [P, P]),
            "orc_filled": (C.c_int, [P]),
            "orc_game_over": (C.c_int, [P]),
            "orc_blank_count": (C.c_int, [P]),
            "orc_spawn": (C.c_int, [P, C.c_int, C.c_int]),
            "orc_mt_state_size": (C.c_int, []),
            "orc_mt_seed": (None, [P, C.c_uint64]),
            "orc_mt_getrandbits": (C.c_uint32, [P, C.c_int]),
            "orc_mt_randbelow": (C.c_uint32, [P, C.c_uint32]),
            "orc_mt_random": (C.c_double, [P]),
            "orc_pyrand_episode": (C.c_int, [P, C.c_int] + [P] * 9),
            "orc_philox4x32_10": (None, [P, P, P]),
            "orc_philox4x32_r": (None, [P, P, P, C.c_int]),
            "orc_step_philox": (C.c_int64, [P, C.c_int64, C.c_uint64, C.c_int64, C.c_uint32, C.c_uint32,
                                            P, P, P, P, P]),
            "orc_step_draws": (C.c_int64, [P, C.c_int64, P, P, P, P, P, P, C.c_uint32]),
            "orc_reset_philox": (None, [P, C.c_int64, C.c_uint64, C.c_int64, C.c_uint32, P]),
            "orc_score": (None, [P, C.c_int64, P]),
            "orc_fill_random": (None, [P, C.c_int64, C.c_uint64, C.c_int64, C.c_uint32]),
            "orc_replay_ring_index": (None, [C.c_uint64, C.c_uint32, C.c_int64, C.c_int64, P]),
            "orc_replay_perm_index": (None, [C.c_uint64, C.c_uint32, C.c_int64, C.c_int64, P]),
            "orc_bench_pyrand": (C.c_int64, [C.c_uint64, C.c_int64]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _boards(b):
    b = np.ascontiguousarray(b, dtype=np.int8).reshape(-1, 16)
    return b


# ---------------------------------------------------------------- single-board helpers
def move(board, action, with_reward=False):
    """update_matrix on one board (int8[16] exponents). Returns (new, changed[, reward])."""
    b = np.array(board, dtype=np.int8).reshape(16).copy()
    rw = np.zeros(1, np.int64)
    c = lib().orc_move(_p(b), int(action), _p(rw))
    if c < 0:
        raise ValueError("bad action %r" % (action,))
    return (b, bool(c), int(rw[0])) if with_reward else (b, bool(c))


def game_over(board):
    b = np.array(board, dtype=np.int8).reshape(16)
    return bool(lib().orc_game_over(_p(b)))


def filled(board):
    b = np.array(board, dtype=np.int8).reshape(16)
    return bool(lib().orc_filled(_p(b)))


def line_table():
    out = np.zeros((4, LINE_TABLE_N, 4), np.int8)
    chg = np.zeros((4, LINE_TABLE_N), np.uint8)
    lib().orc_line_table(_p(out), _p(chg))
    return out, chg


def move_line(cells):
    line = np.array(cells, dtype=np.int8)
    c = lib().orc_move_line(_p(line), line.size)
    return line, bool(c)


# ---------------------------------------------------------------- batched (kernel contract)
def step_philox(boards, seed, step, flags, actions=None, board_offset=0, want_score=False):
    """Batched Philox-mode step, in place on a copy. Returns dict of outputs."""
    b = _boards(boards).copy()
    n = b.shape[0]
    act = np.zeros(n, np.int8) if actions is None else np.ascontiguousarray(actions, np.int8).copy()
    done = np.zeros(n, np.uint8)
    chg = np.zeros(n, np.uint8)
    rw = np.zeros(n, np.int32)
    sc = np.zeros(n, np.int32) if want_score else None
    bad = lib().orc_step_philox(_p(b), n, seed, board_offset, step, flags, _p(act), _p(done), _p(chg),
                                _p(rw), _p(sc))
    return {"boards": b, "actions": act, "done": done, "changed": chg, "reward": rw, "score": sc, "bad": bad}


def step_draws(boards, actions, rank, four, flags=0):
    b = _boards(boards).copy()
    n = b.shape[0]
    act = np.ascontiguousarray(actions, np.int8)
    rk = np.ascontiguousarray(rank, np.uint8)
    fr = np.ascontiguousarray(four, np.uint8)
    done = np.zeros(n, np.uint8)
    chg = np.zeros(n, np.uint8)
    rw = np.zeros(n, np.int32)
    bad = lib().orc_step_draws(_p(b), n, _p(act), _p(rk), _p(fr), _p(done), _p(chg), _p(rw), flags)
    return {"boards": b, "done": done, "changed": chg, "reward": rw, "bad": bad}


def reset_philox(boards, seed, reset_ctr, mask=None, board_offset=0):
    b = _boards(boards).copy()
    m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
    lib().orc_reset_philox(_p(b), b.shape[0], seed, board_offset, reset_ctr, _p(m))
    return b


def fill_random(n, seed, max_exp=7, board_offset=0):
    b = np.zeros((n, 16), np.int8)
    lib().orc_fill_random(_p(b), n, seed, board_offset, max_exp)
    return b


def replay_index(seed, sample_ctr, size, n, ring=True):
    """Slots drawn by r48_replay_sample: ring (uniform, with replacement) or fill-drain
    (Feistel permutation, without replacement; n <= size)."""
    out = np.zeros(n, np.int64)
    f = lib().orc_replay_ring_index if ring else lib().orc_replay_perm_index
    f(seed, sample_ctr, size, n, _p(out))
    return out


def score(boards):
    b = _boards(boards)
    out = np.zeros(b.shape[0], np.int32)
    lib().orc_score(_p(b), b.shape[0], _p(out))
    return out


def philox(ctr, key, rounds=10):
    c = np.ascontiguousarray(ctr, np.uint32)
    k = np.ascontiguousarray(key, np.uint32)
    out = np.zeros(4, np.uint32)
    if rounds == 10:
        lib().orc_philox4x32_10(_p(c), _p(k), _p(out))
    else:
        lib().orc_philox4x32_r(_p(c), _p(k), _p(out), int(rounds))
    return out


# ---------------------------------------------------------------- CPython random replay
class PyRand:
    """CPython-compatible `random` stream (MT19937), for replaying reference trajectories."""

    def __init__(self, seed):
        self.state = np.zeros(lib().orc_mt_state_size(), np.uint8)
        lib().orc_mt_seed(_p(self.state), seed)

    def getrandbits(self, k):
        return lib().orc_mt_getrandbits(_p(self.state), k)

    def randbelow(self, n):
        return lib().orc_mt_randbelow(_p(self.state), n)

    def random(self):
        return lib().orc_mt_random(_p(self.state))

    def episode(self, max_steps=100000):
        """One main.py-style episode (Game() then Rand.random_action until done)."""
        start = np.zeros(16, np.int8)
        sd = np.zeros(2, np.int32)
        before = np.zeros((max_steps, 16), np.int8)
        after = np.zeros((max_steps, 16), np.int8)
        action = np.zeros(max_steps, np.int32)
        done = np.zeros(max_steps, np.uint8)
        chg = np.zeros(max_steps, np.uint8)
        rank = np.zeros(max_steps, np.int32)
        four = np.zeros(max_steps, np.int32)
        t = lib().orc_pyrand_episode(_p(self.state), max_steps, _p(start), _p(sd), _p(before), _p(action),
                                     _p(after), _p(done), _p(chg), _p(rank), _p(four))
        return {"start": start, "start_draw": sd, "before": before[:t], "action": action[:t],
                "after": after[:t], "done": done[:t], "changed": chg[:t], "rank": rank[:t], "four": four[:t]}


def bench_pyrand(seed, steps):
    return lib().orc_bench_pyrand(seed, steps)
