"""VecGame -- the batched, device-resident form of the reference's Game.

nevertiree/Rein48 steps ONE board per Python call (game/GameClient.py:40-51). VecGame holds
N int8[16] boards in HBM (row-major cells, exponent e = tile 2^e, 0 empty) and advances all
of them per call through librein48.so's gfx950 kernels. Boards, actions and flags are torch
tensors on the env's GPU; every call is asynchronous on torch's current stream.

Spawn randomness (GameClient.py:121,125) comes from a per-lane Philox4x32-7 keyed by
(seed, global board id): a VecGame sharded across ranks with board_offset = rank * N is
bit-identical to one unsharded VecGame.
"""
import ctypes as C

import torch

from . import _lib
from ._lib import AUTO_RESET, MERGE_REWARD, RANDOM_POLICY, check, ptr

ACTIONS = ("UP", "DOWN", "LEFT", "RIGHT")  # codes 0..3, GameClient.py:140,182,206,230


def _stream(device):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


try:    # torch's raw current-stream query: a few microseconds cheaper per call than the Stream object
    _raw_stream = torch._C._cuda_getCurrentRawStream
except AttributeError:  # pragma: no cover
    _raw_stream = None


class VecGame:
    """N boards stepped in lockstep on one GPU.

    Mirrors Game's surface in batched form: reset() / step(actions) -> (boards, reward, done),
    plus the size attributes (GameClient.py:21-27).
    """

    reward_space_size = 1
    action_space_size = 4
    state_space_size = 4

    def __init__(self, n_boards, device=None, seed=0, board_offset=0):
        lib = _lib.load()
        if not torch.cuda.is_available():
            raise RuntimeError("VecGame needs a ROCm GPU (torch.cuda.is_available() is False)")
        dev = torch.device(device if device is not None else "cuda")
        if dev.type != "cuda":
            raise ValueError("VecGame device must be a GPU, got %s" % dev)
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        n = int(n_boards)
        if n <= 0:
            raise ValueError("n_boards must be positive")
        self.device = dev
        self.n = n
        self.seed = int(seed) & (2 ** 64 - 1)
        self.board_offset = int(board_offset)
        self.boards = torch.zeros((n, 16), dtype=torch.int8, device=dev)
        self.actions = torch.zeros(n, dtype=torch.int8, device=dev)
        self.done = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.changed = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.reward = torch.zeros(n, dtype=torch.int32, device=dev)
        self._zero_reward = torch.zeros(n, dtype=torch.int32, device=dev)  # reference reward is always 0
        self._env = C.c_void_p()
        check(lib.r48_env_create(C.byref(self._env), dev.index, n, self.seed, self.board_offset))
        check(lib.r48_env_bind_boards(self._env, ptr(self.boards)))
        self._lib = lib
        self._argcache = {}

    # ------------------------------------------------------------------ helpers
    def _t(self, t, dtype, name, n=None):
        if t is None:
            return None
        if not isinstance(t, torch.Tensor):
            t = torch.as_tensor(t, dtype=dtype, device=self.device)
        if t.device != self.device:
            raise ValueError("%s must be on %s, got %s" % (name, self.device, t.device))
        if t.dtype != dtype:
            raise TypeError("%s must be %s, got %s" % (name, dtype, t.dtype))
        if not t.is_contiguous():
            raise ValueError("%s must be contiguous" % name)
        if t.numel() != (self.n if n is None else n):
            raise ValueError("%s must have %d elements, got %d" % (name, self.n if n is None else n, t.numel()))
        return t

    def _s(self):
        return _stream(self.device)

    # ------------------------------------------------------------------ counters
    @property
    def counters(self):
        s, r = C.c_uint32(), C.c_uint32()
        check(self._lib.r48_env_get_counters(self._env, C.byref(s), C.byref(r)))
        return s.value, r.value

    @counters.setter
    def counters(self, value):
        s, r = value
        check(self._lib.r48_env_set_counters(self._env, int(s), int(r)))

    # ------------------------------------------------------------------ reset
    def reset(self, mask=None):
        """Game.reset (GameClient.py:33-38) for the masked boards (all if None)."""
        mask = self._t(mask, torch.uint8, "mask")
        check(self._lib.r48_env_reset(self._env, ptr(mask), self._s()))
        return self.boards

    def reset_with_draws(self, rank, four, mask=None):
        rank = self._t(rank, torch.uint8, "rank")
        four = self._t(four, torch.uint8, "four")
        mask = self._t(mask, torch.uint8, "mask")
        check(self._lib.r48_env_reset_with_draws(self._env, ptr(mask), ptr(rank), ptr(four), self._s()))
        return self.boards

    def fill_random(self, max_exp=7):
        """Synthetic start boards (SURVEY.md 8(d) bench input): each cell empty w.p. 1/2, else
        exponent ~ U{1..max_exp}, Philox keyed by (seed, global board id). Counters unchanged."""
        check(self._lib.r48_env_fill_random(self._env, int(max_exp), self._s()))
        return self.boards

    # ------------------------------------------------------------------ step
    def step(self, actions=None, auto_reset=False, merge_reward=False, want_changed=False, score=None,
             done_out=None, reward_out=None):
        """Game.step (GameClient.py:40-51) for every board.

        actions: int8[N] tensor of 0..3; None = in-kernel uniform random policy
        (control/rand.py:9-11), the drawn actions land in self.actions.
        Returns (boards, reward, done); reward is all-zero like the reference unless
        merge_reward. done is evaluated before any auto-reset. done_out (uint8[N]) /
        reward_out (int32[N], with merge_reward) receive done / reward instead of the env's own
        buffers (a rollout's trajectory rows, no copies).
        """
        flags = (AUTO_RESET if auto_reset else 0) | (MERGE_REWARD if merge_reward else 0)
        if actions is None:
            flags |= RANDOM_POLICY
            act = self.actions
        else:
            act = self._t(actions, torch.int8, "actions")
        score = self._t(score, torch.int32, "score")
        done = self.done if done_out is None else self._t(done_out, torch.uint8, "done_out")
        rew = self.reward if reward_out is None else self._t(reward_out, torch.int32, "reward_out")
        check(self._lib.r48_env_step(self._env, ptr(act), flags, ptr(done),
                                     ptr(self.changed) if want_changed else None,
                                     ptr(rew) if merge_reward else None, ptr(score), self._s()))
        return self.boards, (rew if merge_reward else self._zero_reward), done

    def _step_n_args(self, actions, auto_reset, merge_reward, want_changed, score):
        flags = (AUTO_RESET if auto_reset else 0) | (MERGE_REWARD if merge_reward else 0)
        if actions is None:
            flags |= RANDOM_POLICY
            act = self.actions
        else:
            act = self._t(actions, torch.int8, "actions")
        score = self._t(score, torch.int32, "score")
        return (ptr(act), flags, ptr(self.done), ptr(self.changed) if want_changed else None,
                ptr(self.reward) if merge_reward else None, ptr(score))

    def step_n(self, n_steps, actions=None, auto_reset=False, merge_reward=False, want_changed=False,
               score=None):
        """n_steps consecutive step() calls with the same arguments in ONE kernel launch
        (k_step_n: every board stays in registers for all n_steps steps). Outputs hold the last
        step's values, exactly as after n_steps step() calls."""
        if actions is None and score is None and _raw_stream is not None:
            # the random-policy loop's call: argument tuple cached, raw stream handle
            key = (auto_reset, merge_reward, want_changed)
            a = self._argcache.get(key)
            if a is None:
                a = self._argcache[key] = self._step_n_args(None, auto_reset, merge_reward, want_changed, None)
            st = C.c_void_p(_raw_stream(self.device.index))
        else:
            a = self._step_n_args(actions, auto_reset, merge_reward, want_changed, score)
            st = self._s()
        check(self._lib.r48_env_step_n(self._env, int(n_steps), a[0], a[1], *a[2:], st))
        return self.boards, (self.reward if merge_reward else self._zero_reward), self.done

    def step_with_draws(self, actions, rank, four, merge_reward=False):
        """Parity mode: Game.step with the reference's spawn draws injected."""
        act = self._t(actions, torch.int8, "actions")
        rank = self._t(rank, torch.uint8, "rank")
        four = self._t(four, torch.uint8, "four")
        check(self._lib.r48_env_step_with_draws(self._env, ptr(act), ptr(rank), ptr(four),
                                                MERGE_REWARD if merge_reward else 0, ptr(self.done),
                                                ptr(self.changed), ptr(self.reward), self._s()))
        return self.boards, self.reward, self.done

    def move(self, actions, n_blank=None, merge_reward=False):
        """update_matrix only (GameClient.py:129-254): returns (changed, n_blank)."""
        act = self._t(actions, torch.int8, "actions")
        if n_blank is None:
            n_blank = torch.empty(self.n, dtype=torch.uint8, device=self.device)
        n_blank = self._t(n_blank, torch.uint8, "n_blank")
        check(self._lib.r48_env_move(self._env, ptr(act), MERGE_REWARD if merge_reward else 0,
                                     ptr(self.changed), ptr(n_blank), ptr(self.reward), self._s()))
        return self.changed, n_blank

    def spawn(self, rank, four, mask=None):
        """random_fill_grid with injected draws where mask, then has_game_over -> done."""
        rank = self._t(rank, torch.uint8, "rank")
        four = self._t(four, torch.uint8, "four")
        mask = self._t(mask, torch.uint8, "mask")
        check(self._lib.r48_env_spawn(self._env, ptr(mask), ptr(rank), ptr(four), ptr(self.done), self._s()))
        return self.done

    def rollout(self, n_steps, actions=None, done=None):
        """n_steps random-policy steps with auto-reset, boards kept in registers.
        actions/done: optional int8/uint8 [n_steps, N] trajectory outputs."""
        actions = self._t(actions, torch.int8, "actions", n=n_steps * self.n)
        done = self._t(done, torch.uint8, "done", n=n_steps * self.n)
        check(self._lib.r48_env_rollout(self._env, int(n_steps), ptr(actions), ptr(done), self._s()))
        return self.boards

    # ------------------------------------------------------------------ observation helpers
    def score(self, out=None):
        """main.py:48's np.sum(state_matrix) per board (int32[N])."""
        if out is None:
            out = torch.empty(self.n, dtype=torch.int32, device=self.device)
        out = self._t(out, torch.int32, "out")
        check(self._lib.r48_env_score(self._env, ptr(out), self._s()))
        return out

    def values(self):
        """Boards as raw tile values int32[N,4,4] (the reference's state_matrix encoding)."""
        e = self.boards.to(torch.int32)
        return torch.where(e > 0, torch.ones_like(e) << e, torch.zeros_like(e)).view(self.n, 4, 4)

    def error_count(self, clear=False):
        v = C.c_int64()
        check(self._lib.r48_env_error_count(self._env, C.byref(v), self._s()))
        if clear:
            check(self._lib.r48_env_clear_errors(self._env, self._s()))
        return v.value

    def close(self):
        if getattr(self, "_env", None) is not None and self._env.value:
            self._lib.r48_env_destroy(self._env)
            self._env = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
