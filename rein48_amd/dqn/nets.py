"""ResNet-10 Q-network for 4x4 boards (BASELINE config 5), PyTorch-ROCm.

No reference code exists for it: README.md:15-17 proposes a ResNet with ReLU and Batch
Normalization as the 2048 feature extractor, and BASELINE config 5 names "ResNet-10 policy bf16".
Architecture (10 weight layers):
    input  18 one-hot exponent planes on the 4x4 grid (r48_board_onehot)
    stem   conv3x3 (pad 1) 18 -> C, BN, ReLU
    4 x BasicBlock: conv3x3 C -> C, BN, ReLU, conv3x3 C -> C, BN, + identity, ReLU
    head   Linear(16 C -> 4): one Q-value per action (0 UP, 1 DOWN, 2 LEFT, 3 RIGHT)
with C = 64 and no downsampling (the grid is only 4x4).

MI355X layout: activations are [B, 16 * C] (position-major, channel-minor) and every 3x3
convolution on the 4x4 grid is ONE structured dense GEMM [B, 16 C_in] x [16 C_in, 16 C_out]^T
whose weight is scattered (differentiably) from the conv kernel: 100 of the 144 (position,
tap) pairs are inside the grid, so the dense GEMM does 2.56x the useful FLOPs but runs as one
large hipBLASLt bf16 MFMA GEMM per layer with M = boards. At 2^21 boards it measured 2x
MIOpen's channels-last conv (tools/exp_resnet.py; MIOpen also rejects batches >= 2^18 on 4x4
inputs). BatchNorm is per channel over (boards x positions), computed in fp32.
forward(x [B, 16*18]) -> Q [B, 4] (fp32).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..a3c.nets import linear
from .kernels import PLANES

_BLOCKS = {}


def _tap_blocks(device):
    """The 100 in-grid (cell p, tap t) pairs of a pad-1 3x3 conv on the 4x4 grid as index
    tensors P (output cell), Q (input cell p + 4dr + dc) and T (tap (dr+1)*3 + (dc+1))."""
    key = str(device)
    if key not in _BLOCKS:
        P, Q, T = [], [], []
        for p in range(16):
            r, c = divmod(p, 4)
            for dr in (-1, 0, 1):
                for dc in (-1, 0, 1):
                    if 0 <= r + dr < 4 and 0 <= c + dc < 4:
                        P.append(p)
                        Q.append(4 * (r + dr) + c + dc)
                        T.append((dr + 1) * 3 + dc + 1)
        _BLOCKS[key] = tuple(torch.tensor(v, dtype=torch.long, device=device) for v in (P, Q, T))
    return _BLOCKS[key]


class _StructuredConvWeight(torch.autograd.Function):
    """w [co, ci, 3, 3] -> the [16 co, 16 ci] matrix of the conv on the 4x4 grid (block
    (p, q) = w[:, :, dr + 1, dc + 1] for every in-grid pair), in `dtype`. On the GPU one HIP pass
    each way (r48_struct_conv_weight / _grad: zeros, scatter and cast fused; the gradient sums
    each tap's blocks in a fixed order); on the CPU the same map as an index_put and a backward
    index_add over the 100 in-grid blocks."""

    @staticmethod
    def forward(ctx, w, dtype):
        co, ci = w.shape[:2]
        ctx.shape = (co, ci)
        if w.is_cuda and dtype in (torch.float32, torch.bfloat16):
            from .. import _lib
            from .._lib import check, ptr
            wf = w.detach().float().contiguous()
            d = torch.empty(16 * co, 16 * ci, dtype=dtype, device=w.device)
            check(_lib.load().r48_struct_conv_weight(ptr(wf), co, ci, _lib.BF16 if dtype == torch.bfloat16 else _lib.F32,
                                                     ptr(d), torch.cuda.current_stream(w.device).cuda_stream))
            ctx.w_dtype = w.dtype
            return d
        P, Q, T = _tap_blocks(w.device)
        taps = w.permute(2, 3, 0, 1).reshape(9, co, ci)
        d = torch.zeros(16, co, 16, ci, dtype=w.dtype, device=w.device)
        d[P, :, Q, :] = taps[T]
        ctx.w_dtype = w.dtype
        return d.view(16 * co, 16 * ci).to(dtype)

    @staticmethod
    def backward(ctx, gd):
        co, ci = ctx.shape
        if gd.is_cuda and gd.dtype in (torch.float32, torch.bfloat16):
            from .. import _lib
            from .._lib import check, ptr
            gd = gd.contiguous()
            gw = torch.empty(co, ci, 3, 3, dtype=torch.float32, device=gd.device)
            check(_lib.load().r48_struct_conv_weight_grad(ptr(gd), co, ci,
                                                          _lib.BF16 if gd.dtype == torch.bfloat16 else _lib.F32,
                                                          ptr(gw), torch.cuda.current_stream(gd.device).cuda_stream))
            return gw.to(ctx.w_dtype), None
        P, Q, T = _tap_blocks(gd.device)
        gd = gd.to(ctx.w_dtype)
        blocks = gd.reshape(16, co, 16, ci)[P, :, Q, :]                       # [100, co, ci]
        g9 = torch.zeros(9, co, ci, dtype=gd.dtype, device=gd.device).index_add_(0, T, blocks)
        return g9.view(3, 3, co, ci).permute(2, 3, 0, 1).contiguous(), None


def dense_conv_weight(conv, dtype=None):
    """[16 co, 16 ci] structured matrix of a Conv2d(ci, co, 3, padding=1) on the 4x4 grid, in
    `dtype` (default: the weight's)."""
    return _StructuredConvWeight.apply(conv.weight, conv.weight.dtype if dtype is None else dtype)


class ResNet10Q(nn.Module):
    def __init__(self, channels=64, blocks=4, bn=True, dtype=torch.float32):
        super().__init__()
        self.dtype = dtype
        self.channels, self.n_blocks, self.use_bn = channels, blocks, bn
        self.fused_bn = True          # training-mode BN + ReLU (+ add) via r48_bn_* on bf16 GPU tensors
        self.custom_conv = True       # bf16 GPU convs via r48_conv3x3 / _wgrad (conv.py) instead of dense GEMMs
        C = channels
        self.stem = nn.Conv2d(PLANES, C, 3, padding=1)
        self.convs = nn.ModuleList([nn.Conv2d(C, C, 3, padding=1) for _ in range(2 * blocks)])
        self.bns = nn.ModuleList([nn.BatchNorm1d(C) for _ in range(1 + 2 * blocks)]) if bn else None
        self.head = nn.Linear(16 * C, 4)
        for m in [self.stem, *self.convs]:
            nn.init.kaiming_normal_(m.weight, nonlinearity="relu")
            nn.init.zeros_(m.bias)
        nn.init.normal_(self.head.weight, std=1e-2)
        nn.init.zeros_(self.head.bias)

    def conv_layers(self):
        return [self.stem, *self.convs]

    def _bn(self, k, h):
        """BatchNorm per channel over (boards x cells): statistics and affine in the BN
        parameters' dtype (fp32), activations stay in their own dtype (bf16 on the GPU path)."""
        if not self.use_bn:
            return h
        B = h.shape[0]
        bn = self.bns[k]
        x = h.reshape(B * 16, self.channels)
        if x.dtype != bn.weight.dtype and not x.is_cuda:
            x = x.to(bn.weight.dtype)                   # CPU batch_norm needs matching dtypes
        return bn(x).view(B, 16 * self.channels)

    def wants_onehot32(self, device, dtype):
        """True when the input planes should come padded to 32 (board_onehot32): the custom convs."""
        return (self.custom_conv and self.use_bn and torch.device(device).type == "cuda" and dtype == torch.bfloat16
                and self.channels == 64)

    def _custom_conv(self, h):
        return (self.custom_conv and self.use_bn and h.is_cuda and h.dtype == torch.bfloat16
                and self.channels == 64)

    def _conv(self, conv, h):
        if self._custom_conv(h):
            # channels-last [B, 16, cin] through the hand-written block-sparse MFMA convs; the
            # bias is a constant before training-mode BN (see below), added in the kernel
            from .conv import conv3x3_train
            B = h.shape[0]
            x = h.reshape(B, 16, -1)
            if x.shape[2] not in (32, 64):        # the stem's 18 one-hot planes -> one 32-channel chunk
                x = F.pad(x, (0, 32 - x.shape[2]))
            return conv3x3_train(x.contiguous(), conv).view(B, 16 * 64)
        b = conv.bias.repeat(16)
        if self.use_bn:
            # every conv feeds a training-mode BN, which subtracts the batch mean: the conv bias has
            # no effect on the output and an exactly zero gradient, so it is a constant here (no
            # 65536 x 1024 bias-gradient reduction per layer); it still shifts the running mean
            # like before, which the eval-mode fold (folded()) accounts for
            b = b.detach()
        return linear(h, dense_conv_weight(conv, self.dtype), b, self.dtype)

    def _fused_bn(self, h):
        return (self.use_bn and self.fused_bn and self.training and h.is_cuda and h.dtype == torch.bfloat16
                and self.channels in (32, 64, 128))

    def _bn_relu(self, k, h, residual=None):
        """relu(BN_k(h) (+ residual)): on bf16 GPU activations in training mode one fused HIP pass
        forward and backward (bn.py), else torch's BatchNorm1d + ReLU."""
        if self._fused_bn(h):
            from .bn import bn_act
            B = h.shape[0]
            r = None if residual is None else residual.reshape(B * 16, self.channels)
            return bn_act(h.reshape(B * 16, self.channels), self.bns[k], r).view(B, 16 * self.channels)
        z = self._bn(k, h)
        if residual is not None:
            z = z + residual.to(z.dtype)
        return F.relu(z).to(self.dtype)

    def forward(self, x):
        d = self.dtype
        h = self._bn_relu(0, self._conv(self.stem, x))
        for b in range(self.n_blocks):
            c1, c2 = self.convs[2 * b], self.convs[2 * b + 1]
            y = self._bn_relu(1 + 2 * b, self._conv(c1, h))
            h = self._bn_relu(2 + 2 * b, self._conv(c2, y), residual=h)
        if self._custom_conv(h):
            from .conv import q_head
            return q_head(h, self.head)
        return linear(h, self.head.weight, self.head.bias, d).float()

    @torch.no_grad()
    def folded(self):
        """Inference weights with eval-mode BN folded into each conv: list of (w [co, ci, 3, 3],
        b [co]) for the 9 convs, plus (head w [4, 16 C], head b [4]); fp32."""
        out = []
        for k, conv in enumerate(self.conv_layers()):
            w, b = conv.weight.float(), conv.bias.float()
            if self.use_bn:
                bn = self.bns[k]
                s = bn.weight.float() / torch.sqrt(bn.running_var.float() + bn.eps)
                w = w * s.view(-1, 1, 1, 1)
                b = (b - bn.running_mean.float()) * s + bn.bias.float()
            out.append((w.contiguous(), b.contiguous()))
        return out, (self.head.weight.float().contiguous(), self.head.bias.float().contiguous())
