"""Host side of the fused CNN policy kernel (r48_cnn_policy_forward, rein48_amd/csrc/r48_policy.hip).

pack_cnn(net) lays out ActorCriticCNN's weights as the kernel's MFMA A-operand fragments
(v_mfma_f32_32x32x16_bf16: lane l, r = l & 31, h = l >> 5, element j):
  W1 fragment R (9, conv1 output position R):     W1dense[32R + r][8h + j]
  W2 fragment (g, kk, s) (16):                     conv2.w[32g + r][32kk + f]
  Wh fragment (p, g, s) (16):                      heads.w[r][64p + 32g + f]   (rows r >= 5 zero)
with f = 16s + 8(j>>2) + 4h + (j&3), the row order in which a 32x32 accumulator feeds the next
MFMA as its B operand. Biases: b1[32], b2[64], bh[5] padded to 104 floats.
"""
import ctypes as C

import numpy as np
import torch

from .. import _lib
from .._lib import check, ptr


def _index_maps():
    lane = np.arange(64)
    r, h = lane & 31, lane >> 5
    j = np.arange(8)
    f_perm = lambda s: 16 * s + 8 * (j[None, :] >> 2) + 4 * h[:, None] + (j[None, :] & 3)   # [64, 8]
    w1 = np.stack([(32 * R + r)[:, None] * 16 + (8 * h[:, None] + j[None, :]) for R in range(9)])  # into W1dense[288,16]
    w2 = np.stack([(32 * g + r)[:, None] * 128 + 32 * kk + f_perm(s)
                   for g in range(2) for kk in range(4) for s in range(2)])                     # into conv2.w[64,128]
    wh = np.stack([np.where((r < 5)[:, None], r[:, None] * 256 + 64 * p + 32 * g + f_perm(s), -1)
                   for p in range(4) for g in range(2) for s in range(2)])                      # into heads.w[5,256]
    return w1, w2, wh


_MAPS = None


@torch.no_grad()
def pack_cnn(net):
    """-> (wfrag bf16 [41, 64, 8], bias f32 [104]) on the net's device."""
    global _MAPS
    if _MAPS is None:
        _MAPS = _index_maps()
    dev = net.conv1.weight.device
    w1_idx, w2_idx, wh_idx = (torch.as_tensor(m, device=dev) for m in _MAPS)
    w1_dense, _, _, _ = net.dense_weights()
    f1 = w1_dense.reshape(-1)[w1_idx]
    f2 = net.conv2.weight.reshape(-1)[w2_idx]
    hw = torch.cat([net.heads.weight.reshape(-1), torch.zeros(1, device=dev)])
    fh = hw[torch.where(wh_idx < 0, hw.numel() - 1, wh_idx)]
    wfrag = torch.cat([f1, f2, fh]).to(torch.bfloat16).contiguous()
    bias = torch.zeros(104, dtype=torch.float32, device=dev)
    bias[:32] = net.conv1.bias
    bias[32:96] = net.conv2.bias
    bias[96:101] = net.heads.bias
    return wfrag, bias


def cnn_forward(boards, wfrag, bias, exponents=False, logits=True, value=True, actions=False, seed=0, ctr=0,
                gid0=0):
    """Fused CNN inference over int8 boards [n, 16]. Returns (logits [n,4], value [n], actions [n])
    with the unrequested ones None."""
    if not boards.is_cuda or boards.dtype != torch.int8 or not boards.is_contiguous():
        raise ValueError("boards must be a contiguous int8 GPU tensor")
    n = boards.numel() // 16
    dev = boards.device
    lg = torch.empty((n, 4), dtype=torch.float32, device=dev) if logits else None
    v = torch.empty(n, dtype=torch.float32, device=dev) if value else None
    a = torch.empty(n, dtype=torch.int8, device=dev) if actions else None
    check(_lib.load().r48_cnn_policy_forward(ptr(boards), n, ptr(wfrag), ptr(bias),
                                             _lib.FEAT_EXPONENTS if exponents else _lib.FEAT_VALUES,
                                             ptr(lg), ptr(v), ptr(a), int(seed) & (2 ** 64 - 1), int(gid0),
                                             int(ctr) & 0xFFFFFFFF,
                                             C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
    return lg, v, a
