"""Host side of the fused ResNet-10 inference kernel (r48_resnet_q_forward, csrc/r48_resnet.hip).

pack_resnet(net) folds eval-mode BatchNorm into each conv (ResNet10Q.folded) and lays the
weights out as the kernel's v_mfma_f32_16x16x32_bf16 A-operand fragments (1 KiB each; lane l:
row r = l & 15, channel group g = l >> 4, element j). The k order of k-chunk c is channel
16(2c + (j >> 2)) + 4g + (j & 3) -- the layout in which a finished 16x16 accumulator tile leaves
the layer output in the lanes, so the next layer's B operand needs no movement:
  stem (tap t, row tile o):              W0[16o + r][8g + j][t // 3][t % 3]      (planes >= 18: 0)
  conv (tap t, row tile o, k-chunk c):   W[16o + r][16(2c + (j>>2)) + 4g + (j&3)][t // 3][t % 3]
  head (cell p, k-chunk c):              Wh[r][64 p + the same channel]          (rows r >= 4: 0)
each block followed by one bias fragment (64 folded conv biases, or the 4 head biases, as f32,
zero padded to 1 KiB): blob = stem (36 + 1) | conv1 .. conv8 (72 + 1 each) | head (32 + 1).
pack_resnet_gpu does the same in one HIP launch (r48_resnet_pack); the trainer repacks after
every update with it.
"""
import ctypes as C

import numpy as np
import torch

from .. import _lib
from .._lib import check, ptr

_MAPS = {}


def _maps():
    """Index maps into the flattened fp32 weights (-1 = zero) for the stem, conv and head
    fragments, each [frags, 64 lanes, 8 elements]."""
    if _MAPS:
        return _MAPS["m"]
    lane = np.arange(64)
    r, g = (lane & 15)[:, None], (lane >> 4)[:, None]
    j = np.arange(8)[None, :]
    ch = lambda c: 16 * (2 * c + (j >> 2)) + 4 * g + (j & 3)
    st = [np.where(8 * g + j < 18, ((16 * o + r) * 18 + 8 * g + j) * 9 + t, -1)
          for t in range(9) for o in range(4)]
    cv = [((16 * o + r) * 64 + ch(c)) * 9 + t for t in range(9) for o in range(4) for c in range(2)]
    hd = [np.where(r < 4, r * 1024 + 64 * p + ch(c), -1) for p in range(16) for c in range(2)]
    _MAPS["m"] = tuple(np.stack(m).astype(np.int64) for m in (st, cv, hd))
    return _MAPS["m"]


_DEV_MAPS = {}


def _dev_index(idx, dev):
    """Device copy of an index map, made once per (map, device); -1 entries stay -1."""
    key = (id(idx), str(dev))
    if key not in _DEV_MAPS:
        _DEV_MAPS[key] = torch.as_tensor(np.ascontiguousarray(idx).reshape(-1), device=dev)
    return _DEV_MAPS[key]


def _gather(flat, idx, dev):
    """flat[idx] with idx < 0 -> 0 (bf16 out)."""
    ext = torch.cat([flat, torch.zeros(1, dtype=flat.dtype, device=dev)])
    it = _dev_index(idx, dev)
    return ext[torch.where(it < 0, ext.numel() - 1, it)].to(torch.bfloat16)


def _bias_frag(b, dev):
    f = torch.zeros(256, dtype=torch.float32, device=dev)
    f[:b.numel()] = b
    return f.view(torch.bfloat16)           # 1 KiB


def _check_net(net):
    if net.channels != 64 or net.n_blocks != 4:
        raise ValueError("the fused kernel is built for ResNet10Q(channels=64, blocks=4)")


@torch.no_grad()
def pack_resnet(net):
    """Host (PyTorch gather) packing -> blob bf16 [frags * 512] on the net's device; the
    reference that r48_resnet_pack is tested against."""
    _check_net(net)
    dev = net.head.weight.device
    convs, (hw, hb) = net.folded()
    st, cv, hd = _maps()
    parts = []
    w, b = convs[0]
    parts += [_gather(w.reshape(-1), st, dev).reshape(-1), _bias_frag(b, dev)]
    for w, b in convs[1:]:
        parts += [_gather(w.reshape(-1), cv, dev).reshape(-1), _bias_frag(b, dev)]
    parts += [_gather(hw.reshape(-1), hd, dev).reshape(-1), _bias_frag(hb, dev)]
    blob = torch.cat(parts).contiguous()
    assert blob.numel() * 2 == _lib.load().r48_resnet_q_blob_bytes()
    return blob


_PTRS = {}


def _param_ptrs(net, dev):
    """Device array of the 56 parameter pointers r48_resnet_pack reads (uploaded once per set of
    parameter storages: they are stable between updates)."""
    tensors = []
    for k, conv in enumerate(net.conv_layers()):
        bn = net.bns[k] if net.use_bn else None
        tensors += [conv.weight, conv.bias] + ([bn.weight, bn.bias, bn.running_mean, bn.running_var] if bn is not None
                                               else [None] * 4)
    tensors += [net.head.weight, net.head.bias]
    for t in tensors:
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous() or t.device != dev):
            raise ValueError("pack_resnet_gpu needs contiguous fp32 parameters on the net's device")
    addrs = tuple(0 if t is None else t.data_ptr() for t in tensors)
    key = (str(dev), addrs)
    if key not in _PTRS:
        _PTRS.clear() if len(_PTRS) > 16 else None
        _PTRS[key] = torch.tensor(addrs, dtype=torch.int64, device=dev)
    return _PTRS[key]


@torch.no_grad()
def pack_resnet_gpu(net, out=None):
    """pack_resnet in one HIP launch (r48_resnet_pack): same layout, BN scale correctly rounded
    in f32 (PyTorch's may differ in the last ulp); `out` (a previous blob for the same net) is
    overwritten in place."""
    _check_net(net)
    dev = net.head.weight.device
    ptrs = _param_ptrs(net, dev)
    blob = torch.empty(_lib.load().r48_resnet_q_blob_bytes() // 2, dtype=torch.bfloat16, device=dev) \
        if out is None else out
    eps = float(net.bns[0].eps) if net.use_bn else 1e-5
    check(_lib.load().r48_resnet_pack(ptr(ptrs), C.c_float(eps), ptr(blob),
                                      C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
    return blob


def resnet_q_forward(boards, blob, q=True, actions=False, eps=0.0, seed=0, ctr=0, gid0=0):
    """Fused ResNet-10 inference over int8 boards [n, 16] (contiguous, on the GPU) with packed
    weights `blob` -> (Q [n, 4] or None, epsilon-greedy actions [n] or None)."""
    if not boards.is_cuda or boards.dtype != torch.int8 or not boards.is_contiguous():
        raise ValueError("boards must be a contiguous int8 GPU tensor")
    n = boards.numel() // 16
    dev = boards.device
    qt = torch.empty((n, 4), dtype=torch.float32, device=dev) if q else None
    at = torch.empty(n, dtype=torch.int8, device=dev) if actions else None
    if n == 0:                               # empty tensors may have NULL data pointers
        return qt, at
    check(_lib.load().r48_resnet_q_forward(ptr(boards), n, ptr(blob), ptr(qt), ptr(at), float(eps),
                                           int(seed) & (2 ** 64 - 1), int(gid0), int(ctr) & 0xFFFFFFFF,
                                           C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
    return qt, at
