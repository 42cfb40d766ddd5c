"""Torch-facing wrappers of the value-based-training HIP kernels (rein48_amd/csrc/r48_dqn.hip)."""
import torch

from .. import _lib
from .._lib import check, ptr
from ..a3c.kernels import _dev, _stream

PLANES = 18


def board_onehot(boards, dtype=torch.bfloat16, out=None):
    """int8 boards [n, 16] -> one-hot planes [n, 16 * 18] (position-major, exponent-minor)."""
    _dev(boards, "boards", torch.int8)
    n = boards.numel() // 16
    if out is None:
        out = torch.empty((n, 16 * PLANES), dtype=dtype, device=boards.device)
    _dev(out, "out", dtype)
    code = {torch.float32: _lib.F32, torch.bfloat16: _lib.BF16}[dtype]
    check(_lib.load().r48_board_onehot(ptr(boards), n, code, ptr(out), _stream(boards)))
    return out


def egreedy_actions(q, eps, seed, ctr, gid0=0, out=None):
    """Epsilon-greedy over q float [n, 4] (r48_egreedy_actions' Philox contract)."""
    _dev(q, "q", torch.float32)
    n = q.numel() // 4
    if out is None:
        out = torch.empty(n, dtype=torch.int8, device=q.device)
    check(_lib.load().r48_egreedy_actions(ptr(q), n, float(eps), int(seed) & (2 ** 64 - 1), int(gid0),
                                          int(ctr) & 0xFFFFFFFF, ptr(out), _stream(q)))
    return out


def td_target(reward, done, q_next_target, q_next_online=None, gamma=0.99, log2_reward=False):
    """y = r + gamma (1 - done) Q'(s', argmax) (double DQN when q_next_online is given); r =
    log2(1 + reward) when log2_reward (the trainer's reward transform, in the same launch)."""
    _dev(reward, "reward", torch.float32)
    _dev(q_next_target, "q_next_target", torch.float32)
    if done is not None:
        _dev(done, "done", torch.uint8)
    if q_next_online is not None:
        _dev(q_next_online, "q_next_online", torch.float32)
    y = torch.empty_like(reward)
    check(_lib.load().r48_td_target(ptr(reward), ptr(done), ptr(q_next_target), ptr(q_next_online), reward.numel(),
                                    float(gamma), int(bool(log2_reward)), ptr(y), _stream(reward)))
    return y
