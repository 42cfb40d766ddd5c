"""Torch-facing wrappers of the A3C HIP kernels in librein48.so (include/rein48.h)."""
import ctypes as C

import torch

from .. import _lib
from .._lib import check, ptr


def _stream(t):
    return C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _dev(t, name, dtype=None):
    if not t.is_cuda:
        raise ValueError("%s must be a GPU tensor (the A3C kernels have no CPU path)" % name)
    if dtype is not None and t.dtype != dtype:
        raise TypeError("%s must be %s, got %s" % (name, dtype, t.dtype))
    if not t.is_contiguous():
        raise ValueError("%s must be contiguous" % name)
    return t


def board_features(boards, exponents=False, dtype=torch.float32, out=None):
    """int8 boards [..., 16] -> network input [..., 16]: raw tile values (a3c.py:139) or exponents."""
    _dev(boards, "boards", torch.int8)
    n = boards.numel() // 16
    if out is None:
        out = torch.empty(boards.shape, dtype=dtype, device=boards.device)
    _dev(out, "out", dtype)
    code = {torch.float32: _lib.F32, torch.bfloat16: _lib.BF16}[dtype]
    check(_lib.load().r48_board_features(ptr(boards), n, _lib.FEAT_EXPONENTS if exponents else _lib.FEAT_VALUES,
                                         code, ptr(out), _stream(boards)))
    return out


def sample_actions(logits, seed, ctr, gid0=0, want_logp=False, want_entropy=False):
    """choose_action (a3c.py:89-93) for every row of logits [n, 4] (post-ReLU, pre-softmax)."""
    _dev(logits, "logits", torch.float32)
    n = logits.numel() // 4
    act = torch.empty(n, dtype=torch.int8, device=logits.device)
    logp = torch.empty(n, dtype=torch.float32, device=logits.device) if want_logp else None
    ent = torch.empty(n, dtype=torch.float32, device=logits.device) if want_entropy else None
    check(_lib.load().r48_sample_actions(ptr(logits), n, int(seed) & (2 ** 64 - 1), int(gid0), int(ctr) & 0xFFFFFFFF,
                                         ptr(act), ptr(logp), ptr(ent), _stream(logits)))
    return act, logp, ent


def discounted_returns(rewards, lengths, bootstrap, gamma=0.9, drop_last=True):
    """_get_target_value_list (a3c.py:246-256) for n segments: rewards [T, n] -> targets [T, n]."""
    _dev(rewards, "rewards", torch.float32)
    _dev(lengths, "lengths", torch.int32)
    _dev(bootstrap, "bootstrap", torch.float32)
    T, n = rewards.shape
    out = torch.empty_like(rewards)
    check(_lib.load().r48_discounted_returns(ptr(rewards), ptr(lengths), ptr(bootstrap), T, n, float(gamma),
                                             1 if drop_last else 0, ptr(out), _stream(rewards)))
    return out


def segment_stats(actions, lengths, values=None, targets=None):
    """losses.segment_stats for segments of `lengths` steps (mask = t < lengths), as one launch:
    actions int8 [T, n], lengths int32 [n], values/targets float32 [T, n] (both or neither) ->
    dict(B [n], counts [n, 4], and td_sum [n] when values/targets are given)."""
    _dev(actions, "actions", torch.int8)
    _dev(lengths, "lengths", torch.int32)
    if (values is None) != (targets is None):
        raise ValueError("values and targets go together")
    if values is not None:
        _dev(values, "values", torch.float32)
        _dev(targets, "targets", torch.float32)
    T, n = actions.shape
    dev = actions.device
    out = {"B": torch.empty(n, dtype=torch.float32, device=dev),
           "counts": torch.empty((n, 4), dtype=torch.float32, device=dev)}
    if values is not None:
        out["td_sum"] = torch.empty(n, dtype=torch.float32, device=dev)
    check(_lib.load().r48_a3c_segment_stats(ptr(values), ptr(targets), ptr(actions), ptr(lengths), T, n, ptr(out["B"]),
                                            ptr(out.get("td_sum")), ptr(out["counts"]), _stream(actions)))
    return out


def row_weights(lengths, B, T, td_sum=None):
    """The fused update's per-row weights [T, n]: wn = mask / B / n and, with td_sum (the
    reference loss), cm = td_sum / (4 B B) * mask / n, in the tensor form's operation order."""
    _dev(lengths, "lengths", torch.int32)
    _dev(B, "B", torch.float32)
    n = lengths.numel()
    wn = torch.empty((T, n), dtype=torch.float32, device=lengths.device)
    cm = torch.empty_like(wn) if td_sum is not None else None
    if td_sum is not None:
        _dev(td_sum, "td_sum", torch.float32)
    check(_lib.load().r48_a3c_row_weights(ptr(lengths), ptr(B), ptr(td_sum), T, n, ptr(wn), ptr(cm), _stream(wn)))
    return wn, cm


def segments(rewards, lengths, bootstrap, gamma=0.9, drop_last=True, values=None, actions=None):
    """The fused update's per-board pass (r48_a3c_segments), one launch: targets [T, n] exactly as
    discounted_returns, seg [n, 4] = (w0, c0, L as int32 bits, 0) -- row_weights' wn / cm at every row
    t < L -- and, with values + actions (the reference loss), counts [n, 4] and c0 from the td sum.
    -> (targets, seg, counts or None)."""
    _dev(rewards, "rewards", torch.float32)
    _dev(lengths, "lengths", torch.int32)
    _dev(bootstrap, "bootstrap", torch.float32)
    if (values is None) != (actions is None):
        raise ValueError("values and actions go together (the reference loss)")
    if values is not None:
        _dev(values, "values", torch.float32)
        _dev(actions, "actions", torch.int8)
    T, n = rewards.shape
    dev = rewards.device
    targets = torch.empty_like(rewards)
    seg = torch.empty((n, 4), dtype=torch.float32, device=dev)
    counts = torch.empty((n, 4), dtype=torch.float32, device=dev) if values is not None else None
    check(_lib.load().r48_a3c_segments(ptr(rewards), ptr(values), ptr(actions), ptr(lengths), ptr(bootstrap), T, n,
                                       float(gamma), 1 if drop_last else 0, ptr(targets), ptr(seg), ptr(counts),
                                       _stream(rewards)))
    return targets, seg, counts


def rmsprop_tf1_(var, grad, ms, mom, lr, decay=0.9, momentum=0.0, eps=1e-10):
    """In-place TF1 RMSProp step on flat float32 buffers."""
    for t, name in ((var, "var"), (grad, "grad"), (ms, "ms"), (mom, "mom")):
        _dev(t, name, torch.float32)
    check(_lib.load().r48_rmsprop_tf1(ptr(var), ptr(grad), ptr(ms), ptr(mom), var.numel(), float(lr), float(decay),
                                      float(momentum), float(eps), _stream(var)))
