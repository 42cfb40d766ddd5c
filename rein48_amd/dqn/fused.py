"""Host side of the fused ResNet-10 inference kernel (r48_resnet_q_forward, csrc/r48_resnet.hip).

pack_resnet(net) folds eval-mode BatchNorm into each conv (ResNet10Q.folded) and lays the
weights out as the kernel's v_mfma_f32_32x32x16_bf16 A-operand fragments (lane l, row
r = l & 31, half h = l >> 5, element j):
  stem fragment (tap t, k-chunk s, row tile m):  W[32m + r][16s + 8h + j][t // 3][t % 3]   (planes >= 18: 0)
  conv fragment (tap t, k-chunk s, row tile m):  W[32m + r][16s + 8(j>>2) + 4h + (j&3)][t // 3][t % 3]
each layer's fragments followed by one bias fragment (64 floats, zero padded to 1 KiB):
  blob = stem (36 + 1 fragments) | conv1 .. conv8 (72 + 1 each), bf16 fragments of 1 KiB.
The head weight is packed per lane: head_w[cell][h][a][2k + e] (bf16) = Wh[a][64 cell + ci]
with ci the channel of the lane's packed activation register k, element e (k = 4s + q:
row tile m = s >> 1, accumulator register i = 8(s & 1) + 2q + e, ci = 32m + 8(i>>2) + 4h + (i&3)).
"""
import ctypes as C

import numpy as np
import torch

from .. import _lib
from .._lib import check, ptr

_MAPS = {}


def _lane_maps():
    lane = np.arange(64)
    r, h = lane & 31, lane >> 5
    j = np.arange(8)
    stem_plane = lambda s: 16 * s + 8 * h[:, None] + j[None, :]                              # [64, 8]
    conv_ci = lambda s: 16 * s + 8 * (j[None, :] >> 2) + 4 * h[:, None] + (j[None, :] & 3)  # [64, 8]
    return r, stem_plane, conv_ci


def _maps(channels, planes=18):
    key = (channels, planes)
    if key in _MAPS:
        return _MAPS[key]
    C_ = channels
    r, stem_plane, conv_ci = _lane_maps()
    # stem: indices into w.reshape(-1) of shape [C, planes, 3, 3]; -1 = zero
    st = []
    for t in range(9):
        for s in range(2):
            for m in range(2):
                co = (32 * m + r)[:, None].repeat(8, 1)
                pl = stem_plane(s)
                idx = ((co * planes + pl) * 3 + t // 3) * 3 + t % 3
                st.append(np.where(pl < planes, idx, -1))
    cv = []
    for t in range(9):
        for s in range(4):
            for m in range(2):
                co = (32 * m + r)[:, None].repeat(8, 1)
                ci = conv_ci(s)
                cv.append(((co * C_ + ci) * 3 + t // 3) * 3 + t % 3)
    # head: [cell][h][a][32] -> index into Wh.reshape(-1) of shape [4, 16 * C]
    hd = np.zeros((16, 2, 4, 32), np.int64)
    for cell in range(16):
        for hh in range(2):
            for k in range(16):
                s, q = k >> 2, k & 3
                m = s >> 1
                for e in range(2):
                    i = 8 * (s & 1) + 2 * q + e
                    ci = 32 * m + 8 * (i >> 2) + 4 * hh + (i & 3)
                    for a in range(4):
                        hd[cell, hh, a, 2 * k + e] = a * 16 * C_ + cell * C_ + ci
    _MAPS[key] = (np.stack(st), np.stack(cv), hd)
    return _MAPS[key]


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


@torch.no_grad()
def pack_resnet(net):
    """-> (blob bf16 [frags * 512], head_w bf16 [4096], head_b f32 [4]) on the net's device."""
    if net.channels != 64 or net.n_blocks != 4:
        raise ValueError("the fused kernel is built for ResNet10Q(channels=64, blocks=4)")
    dev = net.head.weight.device
    convs, (hw, hb) = net.folded()
    st, cv, hd = _maps(net.channels)
    parts = []
    w, b = convs[0]
    parts += [_gather(w.reshape(-1), st, dev).reshape(-1), _bias_frag(b, dev)]
    for w, b in convs[1:]:
        parts += [_gather(w.reshape(-1), cv, dev).reshape(-1), _bias_frag(b, dev)]
    blob = torch.cat(parts).contiguous()
    assert blob.numel() * 2 == _lib.load().r48_resnet_q_blob_bytes()
    head_w = _gather(hw.reshape(-1), hd, dev).contiguous()
    return blob, head_w, hb.float().contiguous()


_PTRS = {}


@torch.no_grad()
def pack_resnet_gpu(net, out=None):
    """pack_resnet in one HIP launch (r48_resnet_pack): same layout, BN scale correctly rounded
    in f32 (PyTorch's may differ in the last ulp); `out` (a previous result for the same net) is
    overwritten in place."""
    if net.channels != 64 or net.n_blocks != 4:
        raise ValueError("the fused kernel is built for ResNet10Q(channels=64, blocks=4)")
    dev = net.head.weight.device
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
    if key not in _PTRS:                     # parameter storage is stable between updates: upload once
        _PTRS.clear() if len(_PTRS) > 16 else None
        _PTRS[key] = torch.tensor(addrs, dtype=torch.int64, device=dev)
    ptrs = _PTRS[key]
    if out is None:
        blob = torch.empty(_lib.load().r48_resnet_q_blob_bytes() // 2, dtype=torch.bfloat16, device=dev)
        head_w = torch.empty(16 * 2 * 4 * 32, dtype=torch.bfloat16, device=dev)
        head_b = torch.empty(4, dtype=torch.float32, device=dev)
    else:
        blob, head_w, head_b = out
    eps = float(net.bns[0].eps) if net.use_bn else 1e-5
    check(_lib.load().r48_resnet_pack(ptr(ptrs), C.c_float(eps), ptr(blob), ptr(head_w), ptr(head_b),
                                      C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
    return blob, head_w, head_b


def resnet_q_forward(boards, packed, q=True, actions=False, eps=0.0, seed=0, ctr=0, gid0=0):
    """Fused ResNet-10 inference over int8 boards [n, 16] -> (Q [n, 4] or None, actions [n] or None)."""
    if not boards.is_cuda or boards.dtype != torch.int8 or not boards.is_contiguous():
        raise ValueError("boards must be a contiguous int8 GPU tensor")
    blob, head_w, head_b = packed
    n = boards.numel() // 16
    dev = boards.device
    qt = torch.empty((n, 4), dtype=torch.float32, device=dev) if q else None
    at = torch.empty(n, dtype=torch.int8, device=dev) if actions else None
    check(_lib.load().r48_resnet_q_forward(ptr(boards), n, ptr(blob), ptr(head_w), ptr(head_b), ptr(qt), ptr(at),
                                           float(eps), int(seed) & (2 ** 64 - 1), int(gid0), int(ctr) & 0xFFFFFFFF,
                                           C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
    return qt, at


# ---- cell-grouped kernel (r48_resnet2_*, csrc/r48_resnet2.hip) -------------------------------
# v_mfma_f32_16x16x32_bf16 A fragments, lane l: row r = l & 15, channel group g = l >> 4, element j;
# the k order of chunk c is channel 16(2c + (j >> 2)) + 4g + (j & 3) (the accumulator layout):
#   stem (tap t, row tile o):              W0[16o + r][8g + j][t]          (planes >= 18: 0)
#   conv (tap t, row tile o, k-chunk c):   W[16o + r][16(2c + (j>>2)) + 4g + (j&3)][t]
#   head (cell p, k-chunk c):              Wh[r][64 p + same channel]      (rows r >= 4: 0)
# blob = stem (36 + bias) | conv1..8 (72 + bias each) | head (32 + bias of 4 floats), 1 KiB fragments.
_MAPS2 = {}


def _maps2():
    if _MAPS2:
        return _MAPS2["m"]
    lane = np.arange(64)
    r, g = (lane & 15)[:, None], (lane >> 4)[:, None]
    j = np.arange(8)[None, :]
    ch = lambda c: 16 * (2 * c + (j >> 2)) + 4 * g + (j & 3)
    st = [np.where(8 * g + j < 18, ((16 * o + r) * 18 + 8 * g + j) * 9 + t, -1)
          for t in range(9) for o in range(4)]
    cv = [((16 * o + r) * 64 + ch(c)) * 9 + t for t in range(9) for o in range(4) for c in range(2)]
    hd = [np.where(r < 4, r * 1024 + 64 * p + ch(c), -1) for p in range(16) for c in range(2)]
    _MAPS2["m"] = tuple(np.stack(m).astype(np.int64) for m in (st, cv, hd))
    return _MAPS2["m"]


@torch.no_grad()
def pack_resnet2(net):
    """Host (PyTorch gather) packing for r48_resnet2_q_forward -> blob bf16 [frags * 512]; the
    reference that r48_resnet2_pack is tested against."""
    if net.channels != 64 or net.n_blocks != 4:
        raise ValueError("the fused kernel is built for ResNet10Q(channels=64, blocks=4)")
    dev = net.head.weight.device
    convs, (hw, hb) = net.folded()
    st, cv, hd = _maps2()
    parts = []
    w, b = convs[0]
    parts += [_gather(w.reshape(-1), st, dev).reshape(-1), _bias_frag(b, dev)]
    for w, b in convs[1:]:
        parts += [_gather(w.reshape(-1), cv, dev).reshape(-1), _bias_frag(b, dev)]
    parts += [_gather(hw.reshape(-1), hd, dev).reshape(-1), _bias_frag(hb, dev)]
    blob = torch.cat(parts).contiguous()
    assert blob.numel() * 2 == _lib.load().r48_resnet2_q_blob_bytes()
    return blob


def _param_ptrs(net, dev):
    tensors = []
    for k, conv in enumerate(net.conv_layers()):
        bn = net.bns[k] if net.use_bn else None
        tensors += [conv.weight, conv.bias] + ([bn.weight, bn.bias, bn.running_mean, bn.running_var] if bn is not None
                                               else [None] * 4)
    tensors += [net.head.weight, net.head.bias]
    for t in tensors:
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous() or t.device != dev):
            raise ValueError("packing on the GPU needs contiguous fp32 parameters on the net's device")
    addrs = tuple(0 if t is None else t.data_ptr() for t in tensors)
    key = (str(dev), addrs)
    if key not in _PTRS:                     # parameter storage is stable between updates: upload once
        _PTRS.clear() if len(_PTRS) > 16 else None
        _PTRS[key] = torch.tensor(addrs, dtype=torch.int64, device=dev)
    return _PTRS[key]


@torch.no_grad()
def pack_resnet2_gpu(net, out=None):
    """pack_resnet2 in one HIP launch (r48_resnet2_pack); `out` is overwritten in place."""
    if net.channels != 64 or net.n_blocks != 4:
        raise ValueError("the fused kernel is built for ResNet10Q(channels=64, blocks=4)")
    dev = net.head.weight.device
    ptrs = _param_ptrs(net, dev)
    blob = torch.empty(_lib.load().r48_resnet2_q_blob_bytes() // 2, dtype=torch.bfloat16, device=dev) \
        if out is None else out
    eps = float(net.bns[0].eps) if net.use_bn else 1e-5
    check(_lib.load().r48_resnet2_pack(ptr(ptrs), C.c_float(eps), ptr(blob),
                                       C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
    return blob


def resnet2_q_forward(boards, blob, q=True, actions=False, eps=0.0, seed=0, ctr=0, gid0=0):
    """Cell-grouped fused ResNet-10 inference over int8 boards [n, 16] -> (Q [n, 4] or None,
    actions [n] or None)."""
    if not boards.is_cuda or boards.dtype != torch.int8 or not boards.is_contiguous():
        raise ValueError("boards must be a contiguous int8 GPU tensor")
    n = boards.numel() // 16
    dev = boards.device
    qt = torch.empty((n, 4), dtype=torch.float32, device=dev) if q else None
    at = torch.empty(n, dtype=torch.int8, device=dev) if actions else None
    check(_lib.load().r48_resnet2_q_forward(ptr(boards), n, ptr(blob), ptr(qt), ptr(at), float(eps),
                                            int(seed) & (2 ** 64 - 1), int(gid0), int(ctr) & 0xFFFFFFFF,
                                            C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
    return qt, at
