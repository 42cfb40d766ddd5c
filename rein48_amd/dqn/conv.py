"""Host side of the ResNet-10 update's 3x3 convolutions on the 4x4 grid (csrc/r48_conv.hip).

ResNet10Q (nets.py) trains with channels-last bf16 activations [B, 16 cells, C]. On the GPU its
convolutions run as three hand-written MFMA kernels instead of the structured dense GEMMs
(hipBLASLt) of the portable path, and only the 100 in-grid (cell, tap) pairs are computed:
    forward      r48_conv3x3 with pack_conv(w)           (bias added in the kernel)
    data grad    r48_conv3x3 with pack_conv_dgrad(w)     (taps flipped, in/out channels swapped)
    weight grad  r48_conv3x3_wgrad                        (fp32, summed in a fixed order)
The stem's 18 one-hot planes are padded to one 32-channel k-chunk (board_onehot32). The Q head
Linear(1024 -> 4) runs as r48_q_head_forward / _backward (QHead) instead of three hipBLASLt GEMMs.

Fragment layout (v_mfma_f32_16x16x32_bf16 A operand), fragment (tap t, row tile O, k-chunk c) of
1 KiB: lane l, element j = W[16 O + (l & 15)][32 c + 8 (l >> 4) + j][t // 3][t % 3] (zero past the
real input channels).
"""
import torch

from .. import _lib
from .._lib import check, ptr
from ..a3c.kernels import _dev, _stream

_IDX = {}


def _frag_index(cin_pad, device):
    """Index into a [64, cin_pad, 9] weight of every fragment element, [9 * 4 * nc, 64, 8]."""
    key = (cin_pad, str(device))
    if key not in _IDX:
        nc = cin_pad // 32
        lane = torch.arange(64)
        j = torch.arange(8)
        idx = torch.empty(9, 4, nc, 64, 8, dtype=torch.long)
        for t in range(9):
            for O in range(4):
                for c in range(nc):
                    co = 16 * O + (lane & 15)
                    ci = 32 * c + 8 * (lane >> 4)
                    idx[t, O, c] = (co[:, None] * cin_pad + ci[:, None] + j[None, :]) * 9 + t
        _IDX[key] = idx.view(9 * 4 * nc, 64, 8).to(device)
    return _IDX[key]


def _pack(w9, cin_pad):
    """w9 [64, ci, 9] (any float dtype) -> bf16 fragments [9 * 4 * nc, 64, 8]."""
    co, ci = w9.shape[:2]
    if co != 64 or ci > cin_pad:
        raise ValueError("r48_conv3x3 needs 64 output channels and <= %d input channels" % cin_pad)
    wp = w9.float()
    if ci < cin_pad:
        wp = torch.cat([wp, wp.new_zeros(co, cin_pad - ci, 9)], 1)
    return wp.reshape(-1)[_frag_index(cin_pad, w9.device)].to(torch.bfloat16).contiguous()


def pack_conv(w, cin_pad):
    """Forward fragments of a Conv2d(ci, 64, 3, padding=1) weight [64, ci, 3, 3]."""
    return _pack(w.detach().reshape(w.shape[0], w.shape[1], 9), cin_pad)


def pack_conv_dgrad(w):
    """Data-gradient fragments: W'[ci][co][t] = W[co][ci][8 - t] (64 -> 64 channels)."""
    w9 = w.detach().reshape(w.shape[0], w.shape[1], 9).flip(2).transpose(0, 1)
    return _pack(w9, 64)


def board_onehot32(boards, out=None):
    """int8 boards [n, 16] -> bf16 one-hot [n, 16, 32] (planes 18..31 zero)."""
    _dev(boards, "boards", torch.int8)
    n = boards.numel() // 16
    if out is None:
        out = torch.empty((n, 16, 32), dtype=torch.bfloat16, device=boards.device)
    check(_lib.load().r48_board_onehot32(ptr(boards), n, ptr(out), _stream(boards)))
    return out


def conv3x3(x, frags, bias=None, add=None, out=None, stats=None):
    """x bf16 [B, 16, cin] (cin 32 or 64) -> y bf16 [B, 16, 64] (+ add, bf16 [B, 16, 64]); stats: a
    float[r48_conv_stats_floats()] buffer that receives the per-CU [S1 64][S2 64] sums of y."""
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and x.dim() == 3 and x.shape[1] == 16):
        raise ValueError("x must be a contiguous bf16 CUDA tensor [B, 16, cin]")
    B, _, cin = x.shape
    if add is not None and not (add.dtype == torch.bfloat16 and add.is_contiguous() and add.numel() == B * 1024):
        raise ValueError("add must be a contiguous bf16 tensor of B x 16 x 64")
    y = torch.empty((B, 16, 64), dtype=torch.bfloat16, device=x.device) if out is None else out
    b = None if bias is None else bias.detach().float().contiguous()
    check(_lib.load().r48_conv3x3(ptr(x), B, cin, ptr(frags), ptr(b), ptr(add), ptr(y), ptr(stats), _stream(x)))
    return y


_WS = {}


def conv3x3_wgrad(dy, x, out=None):
    """dw fp32 [64, cin, 3, 3] = sum over boards and in-grid cells of dy[b, p, co] x[b, p + off(t), ci]
    (into `out` when given: a contiguous fp32 tensor of that shape, e.g. a parameter's .grad)."""
    for t, name in ((dy, "dy"), (x, "x")):
        if not (t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous() and t.dim() == 3):
            raise ValueError("%s must be a contiguous bf16 CUDA tensor [B, 16, C]" % name)
    B, _, cin = x.shape
    L = _lib.load()
    key = (cin, str(x.device))
    if key not in _WS:
        _WS[key] = torch.empty(L.r48_conv_wgrad_workspace_floats(cin), dtype=torch.float32, device=x.device)
    dw = torch.empty((64, cin, 3, 3), dtype=torch.float32, device=x.device) if out is None else out
    if not (dw.dtype == torch.float32 and dw.is_contiguous() and dw.numel() == 64 * cin * 9):
        raise ValueError("out must be a contiguous fp32 tensor of 64 x cin x 9")
    check(L.r48_conv3x3_wgrad(ptr(dy), ptr(x), B, cin, ptr(_WS[key]), ptr(dw), _stream(x)))
    return dw


class Conv3x3Train(torch.autograd.Function):
    """y = conv3x3(x, w) + bias on the 4x4 grid for channels-last bf16 x [B, 16, cin_pad]; the
    weight's real input channels may be fewer than cin_pad (the stem). bias is a constant."""

    @staticmethod
    def forward(ctx, x, w, bias):
        cin_pad = x.shape[2]
        y = conv3x3(x, pack_conv(w, cin_pad), bias)
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gy = gy.to(torch.bfloat16).contiguous()
        dx = conv3x3(gy, pack_conv_dgrad(w)) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            dw = conv3x3_wgrad(gy, x)[:, :w.shape[1]].to(w.dtype)
        return dx, dw, None


def conv3x3_train(x, conv):
    """Conv2d(ci, 64, 3, padding=1) `conv` on channels-last bf16 x [B, 16, cin_pad] (training)."""
    return Conv3x3Train.apply(x, conv.weight, conv.bias)


_HEAD_WS = {}


def q_head_forward(h, w, b):
    """h bf16 [B, 1024], w [4, 1024], b [4] -> q fp32 [B, 4] (bf16-rounded values)."""
    if not (h.is_cuda and h.dtype == torch.bfloat16 and h.is_contiguous() and h.dim() == 2 and h.shape[1] == 1024):
        raise ValueError("h must be a contiguous bf16 CUDA tensor [B, 1024]")
    wb = w.detach().to(torch.bfloat16).contiguous()
    bf = b.detach().float().contiguous()
    q = torch.empty((h.shape[0], 4), dtype=torch.float32, device=h.device)
    check(_lib.load().r48_q_head_forward(ptr(h), h.shape[0], ptr(wb), ptr(bf), ptr(q), _stream(h)))
    return q


def q_head_backward(dq, h, w, out=None):
    """-> (dh bf16 [B, 1024], dw fp32 [4, 1024], db fp32 [4]); parameter gradients bf16-rounded,
    written to `out` when given (fp32 storage of 4 * 1024 + 4 floats from its first element: the
    weight rows, then the bias)."""
    L = _lib.load()
    key = str(h.device)
    if key not in _HEAD_WS:
        _HEAD_WS[key] = torch.empty(L.r48_q_head_workspace_floats(), dtype=torch.float32, device=h.device)
    dq = dq.float().contiguous()
    wb = w.detach().to(torch.bfloat16).contiguous()
    dh = torch.empty_like(h)
    if out is None:
        g = torch.empty(4 * 1024 + 4, dtype=torch.float32, device=h.device)
    else:
        if not (out.dtype == torch.float32 and out.is_contiguous() and out.data_ptr() % 16 == 0):
            raise ValueError("out must be contiguous 16-byte aligned fp32 storage")
        g = torch.as_strided(out, (4 * 1024 + 4,), (1,))
    check(L.r48_q_head_backward(ptr(dq), ptr(h), h.shape[0], ptr(wb), ptr(dh), ptr(_HEAD_WS[key]), ptr(g),
                                _stream(h)))
    return dh, g[:4096].view(4, 1024), g[4096:]


class QHead(torch.autograd.Function):
    """q = float(bf16(h @ bf16(w)^T + bf16(b))) -- nets.py's linear(h, w, b, bf16).float() -- with
    the gradients of that path (bf16 output gradient, bf16-rounded parameter gradients)."""

    @staticmethod
    def forward(ctx, h, w, b):
        ctx.save_for_backward(h, w)
        ctx.w_dtype, ctx.b_dtype = w.dtype, b.dtype
        return q_head_forward(h, w, b)

    @staticmethod
    def backward(ctx, dq):
        h, w = ctx.saved_tensors
        dh, dw, db = q_head_backward(dq, h, w)
        return dh, dw.to(ctx.w_dtype), db.to(ctx.b_dtype)


def q_head(h, head):
    """The head Linear(16 C -> 4) `head` on bf16 activations h [B, 1024] (training)."""
    return QHead.apply(h.contiguous(), head.weight, head.bias)


_PACK = {}


def pack_resnet_train(convs):
    """Forward fragments of the 9 convs (stem, conv1..8) and data-gradient fragments of conv1..8 in
    one launch (r48_conv_pack_resnet) -> (fwd list of 9, dgrad list of 9 with None for the stem),
    views of two blobs reused across calls (same layouts as pack_conv / pack_conv_dgrad)."""
    ws = [c.weight for c in convs]
    dev = ws[0].device
    if len(ws) != 9 or ws[0].shape != (64, 18, 3, 3) or any(w.shape != (64, 64, 3, 3) for w in ws[1:]) or \
            any(w.dtype != torch.float32 or not w.is_contiguous() for w in ws):
        raise ValueError("pack_resnet_train needs the 9 contiguous fp32 conv weights of ResNet10Q (C = 64)")
    key = (str(dev), tuple(w.data_ptr() for w in ws))
    if key not in _PACK:
        _PACK.clear()
        fwd = torch.empty((36 + 8 * 72) * 512, dtype=torch.bfloat16, device=dev)
        dg = torch.empty(8 * 72 * 512, dtype=torch.bfloat16, device=dev)
        tab = torch.tensor([w.data_ptr() for w in ws], dtype=torch.int64, device=dev)
        fv = [fwd[:36 * 512].view(36, 64, 8)] + [fwd[(36 + 72 * i) * 512:(36 + 72 * (i + 1)) * 512].view(72, 64, 8)
                                                 for i in range(8)]
        dv = [None] + [dg[72 * i * 512:72 * (i + 1) * 512].view(72, 64, 8) for i in range(8)]
        _PACK[key] = (tab, fwd, dg, fv, dv)
    tab, fwd, dg, fv, dv = _PACK[key]
    check(_lib.load().r48_conv_pack_resnet(ptr(tab), ptr(fwd), ptr(dg), _stream(fwd)))
    return fv, dv
