"""Host side of the fused CNN policy kernel (r48_cnn_policy_forward, rein48_amd/csrc/r48_policy.hip).

pack_cnn(net) lays out ActorCriticCNN's weights as the policy kernels' MFMA A-operand fragments
(v_mfma_f32_32x32x16_bf16: lane l, r = l & 31, h = l >> 5, element j):
  W1 fragment R (9, conv1 output position R):     W1dense[32R + r][8h + j]
  W2 fragment (g, kk, s) (16):                     conv2.w[32g + r][32kk + f]
with f = 16s + 8(j>>2) + 4h + (j&3), the row order in which a 32x32 accumulator feeds the next
MFMA as its B operand; then the heads on v_mfma_f32_16x16x32_bf16 (lane l: m = l & 15, q = l >> 4):
  H16 fragment (p, g) (8):                         heads.w[m][64p + 32g + e]   (rows m >= 5 zero)
with e = 16(q & 1) + 4(q >> 1) + 8(j>>2) + (j&3), the feature order of a block's two 32x32-layout
fragments after their v_permlane16_swap (r48_cnn_common.h cnn_conv2_heads16). 33 fragments.
pack_cnn_train(net) is the fused update's blob: the 32x32 heads Wh fragment (p, g, s) (16):
heads.w[r][64p + 32g + f] (rows r >= 5 zero) after W1 / W2 (41 forward fragments), then Wh^T / W2^T.
Biases: b1[32], b2[64], bh[5] padded to 104 floats.
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
    m, q = lane & 15, lane >> 4
    e = 16 * (q[:, None] & 1) + 4 * (q[:, None] >> 1) + 8 * (j[None, :] >> 2) + (j[None, :] & 3)    # [64, 8]
    wh16 = np.stack([np.where((m < 5)[:, None], m[:, None] * 256 + 64 * p + 32 * g + e, -1)
                     for p in range(4) for g in range(2)])                                      # into heads.w[5,256]
    return w1, w2, wh, wh16


def _index_maps_backward():
    """A fragments of the fused update's backward-data GEMMs (r48_a3c_train.hip):
    Wh^T fragment (p, g) (8):       heads.w[o = 8h + j][64p + 32g + r]          (o >= 5: 0)
    W2^T fragment (kk, g, s) (16):  conv2.w[32g + f(s, j, h)][32kk + r]"""
    lane = np.arange(64)
    r, h = lane & 31, lane >> 5
    j = np.arange(8)
    f_perm = lambda s: 16 * s + 8 * (j[None, :] >> 2) + 4 * h[:, None] + (j[None, :] & 3)   # [64, 8]
    o = 8 * h[:, None] + j[None, :]
    wht = np.stack([np.where(o < 5, o * 256 + 64 * p + 32 * g + r[:, None], -1)
                    for p in range(4) for g in range(2)])
    w2t = np.stack([(32 * g + f_perm(s)) * 128 + 32 * kk + r[:, None]
                    for kk in range(4) for g in range(2) for s in range(2)])
    return wht, w2t


_MAPS = None
_MAPS_BWD = None


_DEV_MAPS = {}


def _on_device(name, maps, dev):
    """The index maps on `dev`, uploaded once (a host-to-device copy per pack stalls the stream)."""
    key = (name, str(dev))
    if key not in _DEV_MAPS:
        _DEV_MAPS[key] = tuple(torch.as_tensor(m, device=dev) for m in maps)
    return _DEV_MAPS[key]


def _pack_parts(net):
    """(W1 fragments, W2 fragments, bias) shared by both blobs, and the padded heads.w gather source."""
    global _MAPS
    if _MAPS is None:
        _MAPS = _index_maps()
    dev = net.conv1.weight.device
    w1_idx, w2_idx, _, _ = _on_device("fwd", _MAPS, dev)
    w1_dense, _, _, _ = net.dense_weights()
    f1 = w1_dense.reshape(-1)[w1_idx]
    f2 = net.conv2.weight.reshape(-1)[w2_idx]
    hw = torch.cat([net.heads.weight.reshape(-1), torch.zeros(1, device=dev)])
    bias = torch.zeros(104, dtype=torch.float32, device=dev)
    bias[:32] = net.conv1.bias
    bias[32:96] = net.conv2.bias
    bias[96:101] = net.heads.bias
    return f1, f2, hw, bias


def _gather_heads(hw, idx):
    return hw[torch.where(idx < 0, hw.numel() - 1, idx)]


@torch.no_grad()
def pack_cnn(net):
    """-> (wfrag bf16 [33, 64, 8], bias f32 [104]) on the net's device: the policy kernels' blob."""
    f1, f2, hw, bias = _pack_parts(net)
    wh16_idx = _on_device("fwd", _MAPS, net.conv1.weight.device)[3]
    return torch.cat([f1, f2, _gather_heads(hw, wh16_idx)]).to(torch.bfloat16).contiguous(), bias


@torch.no_grad()
def pack_cnn_train(net, fwd=None):
    """-> (wfrag bf16 [65, 64, 8], bias f32 [104]): the fused update's 41 forward fragments (W1, W2,
    the 32x32 heads) followed by its 8 Wh^T and 16 W2^T fragments. fwd: accepted for compatibility
    (the policy blob's heads are laid out for 16x16 MFMAs, so the update packs its own)."""
    global _MAPS_BWD
    if _MAPS_BWD is None:
        _MAPS_BWD = _index_maps_backward()
    f1, f2, hw, bias = _pack_parts(net)
    dev = net.conv1.weight.device
    wh_idx = _on_device("fwd", _MAPS, dev)[2]
    wht_idx, w2t_idx = _on_device("bwd", _MAPS_BWD, dev)
    fw2t = net.conv2.weight.reshape(-1)[w2t_idx]
    return torch.cat([f1, f2, _gather_heads(hw, wh_idx), _gather_heads(hw, wht_idx),
                      fw2t]).to(torch.bfloat16).contiguous(), bias


GRAD_FLOATS = 9703   # r48_cnn_train_grad's record: dW2 [64][128] | db2 [64] | dW1 [32][5] | dWh [5][257] | losses [2]


def _check_weights(wn, cm, counts, seg, rows, n_boards):
    """wn [+ cm + counts] per row, or seg [+ counts] per board (r48_a3c_segments). The kernels read
    seg[row % n_boards] and counts[board] as float4, so both are checked against n_boards here (a
    mismatch would be an out-of-bounds read, not an error). Returns n_boards."""
    if n_boards is None:
        if seg is not None or counts is not None:
            raise ValueError("per-board weights (seg / counts) need n_boards")
        n_boards = rows
    n_boards = int(n_boards)
    if n_boards < 1 or rows % n_boards:
        raise ValueError("rows (%d) must be a multiple of n_boards (%d)" % (rows, n_boards))
    for name, t in (("seg", seg), ("counts", counts)):
        if t is not None and (not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous()
                              or tuple(t.shape) != (n_boards, 4)):
            raise ValueError("%s must be a contiguous float32 GPU tensor [n_boards=%d, 4]" % (name, n_boards))
    if seg is not None:
        if wn is not None or cm is not None:
            raise ValueError("per-board weights (seg) replace wn / cm")
        return n_boards
    for name, t in (("wn", wn), ("cm", cm)):
        if t is not None and (not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != rows):
            raise ValueError("%s must be a contiguous float32 GPU tensor of %d rows" % (name, rows))
    if wn is None:
        raise ValueError("wn (or seg) is required")
    if (cm is None) != (counts is None):
        raise ValueError("reference mode needs both cm and counts")
    return n_boards


def cnn_train_grad(net, boards, actions, targets, wn=None, cm=None, counts=None, beta=0.001, exponents=False,
                   n_boards=None, packed=None, workspace=None, seg=None):
    """Gradient of the A3C loss (rein48_amd/a3c/losses.py) over `rows` training states in ONE fused
    pass (r48_cnn_train_grad). boards int8 [rows, 16]; actions int8 [rows]; targets, wn (= mask /
    (B * n)) f32 [rows]; reference mode: cm (= coef * mask / n) f32 [rows] and counts f32
    [n_boards, 4] (row r belongs to board r % n_boards). Or, instead of wn / cm, the per-board
    weights seg f32 [n_boards, 4] of kernels.segments (r48_cnn_train_grad_seg; reference mode iff
    counts is given). Returns (grads in net.parameters() order, actor loss, critic loss)."""
    L = _lib.load()
    rows = boards.numel() // 16
    dev = boards.device
    for name, t, dt in (("boards", boards, torch.int8), ("actions", actions, torch.int8),
                        ("targets", targets, torch.float32)):
        if not t.is_cuda or t.dtype != dt or not t.is_contiguous():
            raise ValueError("%s must be a contiguous %s GPU tensor" % (name, dt))
    n_boards = _check_weights(wn, cm, counts, seg, rows, n_boards)
    wfrag, bias = packed if packed is not None else pack_cnn_train(net)
    if workspace is None:
        workspace = torch.empty(L.r48_cnn_train_workspace_floats(), dtype=torch.float32, device=dev)
    elif (not workspace.is_cuda or workspace.dtype != torch.float32 or not workspace.is_contiguous()
          or workspace.numel() < L.r48_cnn_train_workspace_floats()):
        raise ValueError("workspace must be a contiguous float32 GPU tensor of >= %d floats"
                         % L.r48_cnn_train_workspace_floats())
    out = torch.empty(GRAD_FLOATS, dtype=torch.float32, device=dev)
    mode = _lib.FEAT_EXPONENTS if exponents else _lib.FEAT_VALUES
    stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    if seg is not None:
        check(L.r48_cnn_train_grad_seg(ptr(boards), rows, n_boards, ptr(actions), ptr(targets), ptr(seg),
                                       ptr(counts), float(beta), mode, ptr(wfrag), ptr(bias), ptr(workspace), ptr(out),
                                       stream))
    else:
        check(L.r48_cnn_train_grad(ptr(boards), rows, n_boards, ptr(actions), ptr(targets), ptr(wn),
                                   ptr(cm), ptr(counts), float(beta), mode, ptr(wfrag), ptr(bias), ptr(workspace),
                                   ptr(out), stream))
    dw2 = out[:64 * 128].view(64, 128)
    db2 = out[8192:8256]
    dw1 = out[8256:8416].view(32, 5)
    dwh = out[8416:8416 + 5 * 257].view(5, 257)
    grads = [dw1[:, :4].contiguous(), dw1[:, 4].contiguous(), dw2, db2, dwh[:, :256].contiguous(),
             dwh[:, 256].contiguous()]
    return grads, out[-2], out[-1]


def cnn_forward(boards, wfrag, bias, exponents=False, logits=True, value=True, actions=False, seed=0, ctr=0,
                gid0=0, actions_out=None, boards_out=None):
    """Fused CNN inference over int8 boards [n, 16]. Returns (logits [n,4], value [n], actions [n])
    with the unrequested ones None. actions_out: int8 [n] to draw into (implies actions);
    boards_out: int8 [n, 16] that receives a copy of the boards (the rollout's snapshot)."""
    if not boards.is_cuda or boards.dtype != torch.int8 or not boards.is_contiguous():
        raise ValueError("boards must be a contiguous int8 GPU tensor")
    n = boards.numel() // 16
    dev = boards.device
    for t, name, numel in ((actions_out, "actions_out", n), (boards_out, "boards_out", 16 * n)):
        if t is not None and (not t.is_cuda or t.dtype != torch.int8 or not t.is_contiguous() or t.numel() != numel):
            raise ValueError("%s must be a contiguous int8 GPU tensor of %d elements" % (name, numel))
    lg = torch.empty((n, 4), dtype=torch.float32, device=dev) if logits else None
    v = torch.empty(n, dtype=torch.float32, device=dev) if value else None
    a = actions_out if actions_out is not None else (torch.empty(n, dtype=torch.int8, device=dev) if actions else None)
    check(_lib.load().r48_cnn_policy_forward(ptr(boards), n, ptr(wfrag), ptr(bias),
                                             _lib.FEAT_EXPONENTS if exponents else _lib.FEAT_VALUES,
                                             ptr(lg), ptr(v), ptr(a), ptr(boards_out), int(seed) & (2 ** 64 - 1),
                                             int(gid0),
                                             int(ctr) & 0xFFFFFFFF,
                                             C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
    return lg, v, a


# ---------------------------------------------------------------- the reference MLP (r48_mlp.hip)
@torch.no_grad()
def pack_mlp(net, out=None):
    """ActorCriticMLP -> fp32 weight blob [2504] for r48_mlp_*, grouped by hidden-unit pair p (units
    2p, 2p + 1): a1 [32][16 in][2] | a1.b | a2 [32][4 out][2] | a2.b | c1 [32][16 in][2] | c1.b |
    c2 [64] | c2.b | 3 pad."""
    dev = net.a1.weight.device
    if out is None:
        out = torch.zeros(int(_lib.load().r48_mlp_weight_floats()), dtype=torch.float32, device=dev)
    by_pair = lambda w: w.reshape(32, 2, -1).permute(0, 2, 1)                # [64, in] -> [32, in, 2]  # noqa: E731
    parts = (by_pair(net.a1.weight), net.a1.bias, by_pair(net.a2.weight.t()), net.a2.bias, by_pair(net.c1.weight),
             net.c1.bias, net.c2.weight, net.c2.bias)
    off = 0
    for p in parts:
        k = p.numel()
        out[off:off + k].copy_(p.reshape(-1))
        off += k
    return out


def mlp_forward(boards, w, exponents=False, logits=True, value=True, actions=False, seed=0, ctr=0, gid0=0):
    """Fused fp32 MLP inference over int8 boards [n, 16] (r48_mlp_policy_forward) -> (logits [n, 4]
    post-ReLU, value [n], actions [n]) with the unrequested ones None."""
    if not boards.is_cuda or boards.dtype != torch.int8 or not boards.is_contiguous():
        raise ValueError("boards must be a contiguous int8 GPU tensor")
    n = boards.numel() // 16
    dev = boards.device
    lg = torch.empty((n, 4), dtype=torch.float32, device=dev) if logits else None
    v = torch.empty(n, dtype=torch.float32, device=dev) if value else None
    a = torch.empty(n, dtype=torch.int8, device=dev) if actions else None
    check(_lib.load().r48_mlp_policy_forward(ptr(boards), n, ptr(w), _lib.FEAT_EXPONENTS if exponents else _lib.FEAT_VALUES,
                                             ptr(lg), ptr(v), ptr(a), int(seed) & (2 ** 64 - 1), int(gid0),
                                             int(ctr) & 0xFFFFFFFF,
                                             C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
    return lg, v, a


MLP_GRAD_FLOATS = 2501   # r48_mlp_train_grad's gradient (FlatParams order), then actor + critic loss


def mlp_train_grad(net, boards, actions, targets, wn=None, cm=None, counts=None, beta=0.001, exponents=False,
                   n_boards=None, w=None, workspace=None, seg=None):
    """r48_mlp_train_grad: the A3C loss gradient (losses.chunk_loss's per-row weights wn / cm /
    counts, or the per-board seg, as cnn_train_grad) of every ActorCriticMLP parameter over `rows`
    training states in one fp32 pass -> (flat gradient [2501] in parameters() order, actor loss,
    critic loss) as device tensors (0-d for the losses)."""
    rows = boards.numel() // 16
    dev = boards.device
    for t, name in ((boards, "boards"), (actions, "actions"), (targets, "targets")):
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("%s must be a contiguous GPU tensor" % name)
    n_boards = _check_weights(wn, cm, counts, seg, rows, n_boards)
    if w is None:
        w = pack_mlp(net)
    L = _lib.load()
    need = int(L.r48_mlp_train_workspace_floats(rows))   # grows with rows: the hot pass's flagged-tile lists
    if workspace is None:
        workspace = torch.empty(need, dtype=torch.float32, device=dev)
    elif (not workspace.is_cuda or workspace.dtype != torch.float32 or not workspace.is_contiguous()
          or workspace.numel() < need):
        raise ValueError("workspace must be a contiguous float32 GPU tensor of >= %d floats for %d rows" % (need, rows))
    out = torch.empty(2504, dtype=torch.float32, device=dev)
    mode = _lib.FEAT_EXPONENTS if exponents else _lib.FEAT_VALUES
    stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    if seg is not None:
        check(L.r48_mlp_train_grad_seg(ptr(boards), rows, n_boards, ptr(actions), ptr(targets), ptr(seg),
                                       ptr(counts), float(beta), mode, ptr(w), ptr(workspace), ptr(out), stream))
    else:
        check(L.r48_mlp_train_grad(ptr(boards), rows, n_boards, ptr(actions), ptr(targets), ptr(wn),
                                   ptr(cm), ptr(counts), float(beta), mode, ptr(w), ptr(workspace), ptr(out), stream))
    return out[:MLP_GRAD_FLOATS], out[MLP_GRAD_FLOATS], out[MLP_GRAD_FLOATS + 1]
