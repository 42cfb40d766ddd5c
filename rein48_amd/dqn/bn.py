"""Training-mode BatchNorm + ReLU (+ identity add) as one autograd Function over the HIP kernels
of rein48_amd/csrc/r48_bn.hip (r48_bn_forward / r48_bn_backward).

Used by ResNet10Q (nets.py) in training mode on bf16 GPU activations, where every BN is followed by
a ReLU and the second BN of a basic block by the identity add first:
    y = relu(BN(x) (+ residual))
Semantics of torch.nn.BatchNorm1d in training mode over the channels-last rows (batch statistics
with the biased variance for the normalisation; running_mean / running_var updated with momentum
and the unbiased variance; num_batches_tracked incremented), ReLU's gradient taken where y > 0.
There is no CPU path here: nets.py uses torch's BatchNorm1d for CPU tensors and eval mode.
"""
import torch

from .. import _lib
from .._lib import check, ptr
from ..a3c.kernels import _stream

_WS = {}


def _workspace(rows, C, device):
    n = int(_lib.load().r48_bn_workspace_floats(rows, C))
    key = (device, n)
    if key not in _WS:
        _WS[key] = torch.empty(n, dtype=torch.float32, device=device)
    return _WS[key]


def _need(t, name):
    if not (t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous() and t.data_ptr() % 16 == 0):
        raise ValueError("%s must be a contiguous 16-byte aligned bf16 CUDA tensor" % name)


class _BNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, residual, running_mean, running_var, momentum, eps, relu):
        rows, C = x.shape
        _need(x, "x")
        if residual is not None:
            _need(residual, "residual")
        y = torch.empty_like(x)
        save = torch.empty(2 * C, dtype=torch.float32, device=x.device)
        ws = _workspace(rows, C, x.device)
        g, b = gamma.detach().float().contiguous(), beta.detach().float().contiguous()
        check(_lib.load().r48_bn_forward(ptr(x), ptr(residual), rows, C, ptr(g), ptr(b), ptr(running_mean),
                                         ptr(running_var), float(momentum), float(eps), int(bool(relu)),
                                         ptr(save), ptr(ws), ptr(y), None, _stream(x)))
        ctx.save_for_backward(x, y, g, save)
        ctx.relu, ctx.has_res = bool(relu), residual is not None
        ctx.param_dtype = gamma.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, g, save = ctx.saved_tensors
        rows, C = x.shape
        dy = dy.contiguous()
        if dy.dtype != torch.bfloat16:
            dy = dy.to(torch.bfloat16)
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if ctx.has_res else None
        dgamma = torch.empty(C, dtype=torch.float32, device=x.device)
        dbeta = torch.empty(C, dtype=torch.float32, device=x.device)
        ws = _workspace(rows, C, x.device)
        check(_lib.load().r48_bn_backward(ptr(dy), ptr(y), None, ptr(x), rows, C, ptr(g), ptr(save), int(ctx.relu),
                                          ptr(ws), ptr(dx), ptr(dres), ptr(dgamma), ptr(dbeta), _stream(x)))
        return (dx, dgamma.to(ctx.param_dtype), dbeta.to(ctx.param_dtype), dres, None, None, None, None, None)


def bn_act(x, bn, residual=None, relu=True):
    """relu(bn(x) (+ residual)) for x bf16 [rows, C] on the GPU, bn a torch.nn.BatchNorm1d in
    training mode (its running statistics are updated in place)."""
    if bn.training and bn.track_running_stats:
        bn.num_batches_tracked.add_(1)
        rm, rv = bn.running_mean, bn.running_var
    else:
        rm = rv = None
    mom = bn.momentum if bn.momentum is not None else 0.1
    return _BNAct.apply(x.contiguous(), bn.weight, bn.bias, None if residual is None else residual.contiguous(),
                        rm, rv, mom, bn.eps, relu)
