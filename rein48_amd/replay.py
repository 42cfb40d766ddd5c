"""HBM-resident transition store (config 5), over the C-ABI r48_replay_* (r48_replay.hip).

ReplayStore  -- batched device API (the product path): store n transitions straight from the
               env's device arrays, sample/gather into device tensors. Two modes:
               "ring"       overwrite the oldest, uniform sampling with replacement (DQN);
               "fill_drain" the reference Replay semantics (algorithm/ddpg/replay.py:8-47).
Replay       -- drop-in for algorithm/ddpg/replay.py:Replay (same names, arguments and
               return shapes): store([state, action, reward, next_state]) takes GameClient
               boards (list-of-lists of tile values); sample() returns the dict of numpy
               arrays of list_2_dict and clears. Backed by a fill_drain ReplayStore on the GPU.
               Differences, by design: transitions are stored by value (the reference keeps
               the list objects, so state and next_state alias Game.state_matrix,
               ddpg.py:22-31); actions are stored as codes 0..3 (GameClient.py:140-230
               aliases); rewards come back as float32; the random.sample draw is a keyed
               Philox/Feistel permutation seeded from Python's `random` (so random.seed
               reproduces it), not CPython's MT sequence.
"""
import ctypes as C
import random

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr

MINI_BATCH_SIZE = 10      # replay.py:5
_MODES = {"ring": _lib.REPLAY_RING, "fill_drain": _lib.REPLAY_FILL_DRAIN}


class ReplayStore:
    """capacity transitions of (state int8[16], action int8, reward f32, next_state int8[16],
    done u8) = 38 B each, resident on `device`."""

    def __init__(self, capacity, device="cuda:0", mode="ring", seed=0):
        if mode not in _MODES:
            raise ValueError("mode must be 'ring' or 'fill_drain'")
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("ReplayStore needs a GPU device (the store lives in HBM)")
        self._lib = _lib.load()
        self.mode = mode
        h = C.c_void_p()
        check(self._lib.r48_replay_create(C.byref(h), self.device.index or 0, int(capacity), _MODES[mode],
                                          int(seed) & (2 ** 64 - 1)))
        self._h = h
        self.capacity = int(capacity)

    def _s(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    @property
    def counters(self):
        size, head, ctr = C.c_int64(), C.c_int64(), C.c_uint32()
        check(self._lib.r48_replay_get_counters(self._h, C.byref(size), C.byref(head), C.byref(ctr)))
        return size.value, head.value, ctr.value

    def set_counters(self, size, head, sample_ctr):
        check(self._lib.r48_replay_set_counters(self._h, int(size), int(head), int(sample_ctr)))

    def __len__(self):
        return self.counters[0]

    def filled(self):
        """replay.py:15-16."""
        return len(self) >= self.capacity

    def clear(self):
        check(self._lib.r48_replay_clear(self._h))

    def _check_inputs(self, state, action, reward, next_state, done):
        n = action.numel()
        for name, t, dt, shape in (("state", state, torch.int8, (n, 16)), ("next_state", next_state, torch.int8, (n, 16)),
                                   ("action", action, torch.int8, (n,)), ("reward", reward, torch.float32, (n,)),
                                   ("done", done, torch.uint8, (n,))):
            if t is None:
                if name in ("reward", "done"):
                    continue
                raise ValueError("%s is required" % name)
            if t.device != self.device or t.dtype != dt or not t.is_contiguous() or tuple(t.reshape(-1, *shape[1:]).shape) != shape:
                raise ValueError("%s must be a contiguous %s tensor of shape %s on %s" % (name, dt, shape, self.device))
        return n

    def store(self, state, action, reward, next_state, done=None):
        """Store n transitions (device tensors). Returns how many were kept."""
        n = self._check_inputs(state, action, reward, next_state, done)
        kept = C.c_int64()
        check(self._lib.r48_replay_store(self._h, ptr(state), ptr(action), ptr(reward), ptr(next_state), ptr(done), n,
                                         C.byref(kept), self._s()))
        return kept.value

    def _outs(self, n):
        d = self.device
        return (torch.empty((n, 16), dtype=torch.int8, device=d), torch.empty(n, dtype=torch.int8, device=d),
                torch.empty(n, dtype=torch.float32, device=d), torch.empty((n, 16), dtype=torch.int8, device=d),
                torch.empty(n, dtype=torch.uint8, device=d), torch.empty(n, dtype=torch.int64, device=d))

    def sample(self, batch):
        """-> dict(state, action, reward, next_state, done, index) of device tensors."""
        size = len(self)
        n = min(batch, size) if self.mode == "fill_drain" else batch
        s, a, r, s2, dn, idx = self._outs(n)
        cnt = C.c_int64()
        check(self._lib.r48_replay_sample(self._h, int(batch), ptr(s), ptr(a), ptr(r), ptr(s2), ptr(dn), ptr(idx),
                                          C.byref(cnt), self._s()))
        assert cnt.value == n
        return {"state": s, "action": a, "reward": r, "next_state": s2, "done": dn, "index": idx}

    def gather(self, index):
        index = index.to(self.device, torch.int64).contiguous()
        n = index.numel()
        s, a, r, s2, dn, _ = self._outs(n)
        check(self._lib.r48_replay_gather(self._h, ptr(index), n, ptr(s), ptr(a), ptr(r), ptr(s2), ptr(dn), self._s()))
        return {"state": s, "action": a, "reward": r, "next_state": s2, "done": dn, "index": index}

    def error_count(self):
        v = C.c_uint64()
        check(self._lib.r48_replay_error_count(self._h, C.byref(v)))
        return v.value

    def close(self):
        if getattr(self, "_h", None):
            self._lib.r48_replay_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _board_exponents(matrix):
    """4x4 list of tile values -> int8[16] exponents (0 = empty)."""
    a = np.asarray(matrix, dtype=np.int64).reshape(-1)
    if a.size != 16:
        raise ValueError("Replay stores 4x4 GameClient boards")
    e = np.zeros(16, np.int8)
    nz = a > 0
    lg = np.log2(a[nz]).astype(np.int64)
    if np.any((1 << lg) != a[nz]) or np.any(a < 0):
        raise ValueError("board cells must be 0 or powers of two")
    e[nz] = lg
    return e


def _action_code(action):
    from .game.GameClient import action_code
    return action_code(action)       # ValueError on an unknown action, like GameClient.py:254


class Replay:
    """Drop-in for algorithm/ddpg/replay.py:Replay (see the module docstring)."""

    def __init__(self, replay_size=100, device="cuda:0"):
        self.max_size = replay_size
        self._store = ReplayStore(replay_size, device=device, mode="fill_drain",
                                  seed=random.getrandbits(64))
        self._pending = []          # host-side staging: one batched store per flush

    @property
    def cur_size(self):
        return min(self.max_size, len(self._store) + len(self._pending))

    @property
    def buffer(self):
        raise AttributeError("Replay.buffer lives in HBM; use sample()")

    def filled(self):
        return self.max_size <= self.cur_size

    def store(self, trans):
        """replay.py:18-21: keep [state, action, reward, next_state] until max_size is held."""
        if self.cur_size < self.max_size:
            state, action, reward, next_state = trans
            self._pending.append((_board_exponents(state), _action_code(action), float(reward),
                                  _board_exponents(next_state)))

    def _flush(self):
        if not self._pending:
            return
        dev = self._store.device
        st = torch.from_numpy(np.stack([p[0] for p in self._pending])).to(dev)
        ac = torch.tensor([p[1] for p in self._pending], dtype=torch.int8, device=dev)
        rw = torch.tensor([p[2] for p in self._pending], dtype=torch.float32, device=dev)
        nx = torch.from_numpy(np.stack([p[3] for p in self._pending])).to(dev)
        self._pending = []
        self._store.store(st, ac, rw, nx)

    def sample(self, batch_size=MINI_BATCH_SIZE):
        """replay.py:23-27: random.sample(batch_size) (or everything, in order, when fewer are
        held), as list_2_dict's numpy arrays; then clear()."""
        self._flush()
        out = self._store.sample(batch_size)
        e = out["state"].cpu().numpy().astype(np.int64)
        e2 = out["next_state"].cpu().numpy().astype(np.int64)
        val = lambda x: np.where(x > 0, np.left_shift(1, x), 0).reshape(-1, 4, 4)
        return {"state": val(e), "action": out["action"].cpu().numpy().astype(np.int64),
                "reward": out["reward"].cpu().numpy(), "next_state": val(e2)}

    def clear(self):
        self._pending = []
        self._store.clear()

    @staticmethod
    def sub_list(raw_list, num):
        """replay.py:29-34 (host lists; kept for API completeness)."""
        return raw_list if num > len(raw_list) else random.sample(raw_list, num)

    @staticmethod
    def list_2_dict(raw_list):
        """replay.py:36-43."""
        return {"state": np.array([x[0] for x in raw_list]), "action": np.array([x[1] for x in raw_list]),
                "reward": np.array([x[2] for x in raw_list]), "next_state": np.array([x[3] for x in raw_list])}
