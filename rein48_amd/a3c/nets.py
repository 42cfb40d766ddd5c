"""Policy/value networks (PyTorch-ROCm).

ActorCriticMLP  -- the reference network, algorithm/a3c/a3c.py:136-169:
    actor:  Dense 16->64 ReLU6 -> Dropout(0.4) -> Dense 64->4 ReLU -> softmax
    critic: Dense 16->64 ReLU6 -> Dropout(0.4) -> Dense 64->1
    tf.layers.dropout defaults to training=False, so the dropout is the identity; kernels
    xavier-uniform (a3c.py:138), biases zero (TF default). Input = the 16 raw tile values.
ActorCriticCNN  -- BASELINE config 3's "2-layer CNN policy", the trunk of the reference's only CNN
    (algorithm/ddpg/actor.py:51-85: conv 2x2 valid x32 ReLU -> conv 2x2 valid x64 ReLU -> 256),
    with an actor head (256->4, softmax) and a critic head (256->1). Xavier init as in a3c.py
    (the DDPG actor's N(1, 2) init saturates on raw tile values).

MI355X layout: a board is only 4x4, so each convolution is ONE dense GEMM over the whole batch
with a structured weight assembled (differentiably) from the small conv kernel: conv1 is
16 -> 9x32 = 288 and conv2 is 288 -> 4x64 = 256. That trades ~2x dense FLOPs for zero gathers
(a patch-gather formulation spent most of its update time in the gather's scatter-add
backward), and every layer lands on hipBLASLt bf16 MFMA tiles with M = boards.
The weight gradient of every layer is a reduction over millions of rows into a few thousand
outputs; SplitKLinear computes it as a batched GEMM over row chunks followed by a sum, instead
of one GEMM with K = rows that cannot fill the chip.
forward(x[B,16]) returns (logits[B,4], value[B]); logits are what the softmax / the sampling
kernel consume (for the MLP already through the ReLU of a3c.py:153).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

SPLITK_MIN_ROWS = 1 << 16


def splitk_weight_grad(gy, x):
    """gy^T x (the weight gradient of y = x w^T) in fp32 (fp64 for fp64 inputs): for >= 2^16 rows
    a batched GEMM over row chunks then a sum. bf16 on the GPU: the per-chunk partial products come
    out of hipBLASLt in fp32 (bmm out_dtype), so no bf16 rounding of partials and no cast pass."""
    acc = torch.float64 if x.dtype == torch.float64 else torch.float32
    rows = x.shape[0]
    f32_out = gy.is_cuda and gy.dtype == torch.bfloat16
    if rows >= SPLITK_MIN_ROWS:
        s = min(1024, rows // 8192)
        main = (rows // s) * s
        a, b = gy[:main].view(s, -1, gy.shape[1]).transpose(1, 2), x[:main].view(s, -1, x.shape[1])
        gw = (torch.bmm(a, b, out_dtype=acc) if f32_out else torch.bmm(a, b).to(acc)).sum(0)
        if main < rows:
            gw += (gy[main:].t() @ x[main:]).to(acc)
        return gw
    if f32_out:
        return torch.bmm(gy.t()[None], x[None], out_dtype=acc)[0]
    return (gy.t() @ x).to(acc)


class _SplitKLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        acc = torch.float64 if x.dtype == torch.float64 else torch.float32  # bf16 partials sum in fp32
        gx = gy @ w
        gw = splitk_weight_grad(gy, x)
        # fp32 accumulation, no cast copy; skipped when the bias is a constant (needs no grad)
        gb = gy.sum(0, dtype=acc) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return gx, gw.to(w.dtype), (gb.to(w.dtype) if gb is not None else None)


def linear(x, w, b, dtype):
    """x @ w^T + b computed in `dtype` (bf16 -> MFMA) with the split-K weight gradient."""
    if x.dim() != 2:
        shp = x.shape
        return linear(x.reshape(-1, shp[-1]), w, b, dtype).view(*shp[:-1], w.shape[0])
    return _SplitKLinear.apply(x.to(dtype), w.to(dtype), None if b is None else b.to(dtype))


def _xavier_(layer):
    nn.init.xavier_uniform_(layer.weight)
    nn.init.zeros_(layer.bias)
    return layer


class ActorCriticMLP(nn.Module):
    def __init__(self, dtype=torch.float32):
        super().__init__()
        self.dtype = dtype
        self.a1 = _xavier_(nn.Linear(16, 64))
        self.a2 = _xavier_(nn.Linear(64, 4))
        self.c1 = _xavier_(nn.Linear(16, 64))
        self.c2 = _xavier_(nn.Linear(64, 1))

    def forward(self, x):
        d = self.dtype
        h = F.relu6(linear(x, self.a1.weight, self.a1.bias, d))
        logits = F.relu(linear(h, self.a2.weight, self.a2.bias, d))
        v = linear(F.relu6(linear(x, self.c1.weight, self.c1.bias, d)), self.c2.weight, self.c2.bias, d)[..., 0]
        return logits.float(), v.float()

    @torch.no_grad()
    def load_reference_params(self, p):
        """p: oracle/a3c_ref.py layout (kernels [in, out], TF style)."""
        for name, lay in (("a_w1", self.a1), ("a_w2", self.a2), ("c_w1", self.c1), ("c_w2", self.c2)):
            lay.weight.copy_(torch.as_tensor(p[name]).t())
            lay.bias.copy_(torch.as_tensor(p[name.replace("w", "b")]))

    def reference_params(self):
        out = {}
        for name, lay in (("a_w1", self.a1), ("a_w2", self.a2), ("c_w1", self.c1), ("c_w2", self.c2)):
            out[name] = lay.weight.detach().t().double().cpu().numpy()
            out[name.replace("w", "b")] = lay.bias.detach().double().cpu().numpy()
        return out


def _patches(h, k):
    """patch index lists of a k x k valid convolution over an h x h grid (row-major)."""
    out = h - k + 1
    return [[(r + dr) * h + (c + dc) for dr in range(k) for dc in range(k)] for r in range(out) for c in range(out)]


class ActorCriticCNN(nn.Module):
    def __init__(self, dtype=torch.float32):
        super().__init__()
        self.dtype = dtype
        self.conv1 = nn.Linear(4, 32)       # 2x2x1 kernel, flattened (dr, dc)
        self.conv2 = nn.Linear(4 * 32, 64)  # 2x2x32 kernel, flattened (patch position, channel)
        self.heads = nn.Linear(4 * 64, 5)   # actor 4 + critic 1
        for lay in (self.conv1, self.conv2, self.heads):
            _xavier_(lay)
        # scatter maps from the conv kernels into the dense structured weights
        p1, p2 = _patches(4, 2), _patches(3, 2)
        r1, c1, k1 = [], [], []
        for pos, cells in enumerate(p1):                 # 9 output positions
            for f in range(32):
                for k, cell in enumerate(cells):
                    r1.append(pos * 32 + f)
                    c1.append(cell)
                    k1.append(f * 4 + k)                 # index into conv1.weight.view(-1)
        r2, c2, k2 = [], [], []
        for pos, cells in enumerate(p2):                 # 4 output positions over the 3x3 grid
            for g in range(64):
                for kk, cell in enumerate(cells):
                    for f in range(32):
                        r2.append(pos * 64 + g)
                        c2.append(cell * 32 + f)
                        k2.append(g * 128 + kk * 32 + f)
        for name, v in (("r1", r1), ("c1", c1), ("k1", k1), ("r2", r2), ("c2", c2), ("k2", k2)):
            self.register_buffer(name, torch.tensor(v, dtype=torch.long), persistent=False)

    def dense_weights(self):
        w1 = torch.zeros(9 * 32, 16, dtype=self.conv1.weight.dtype, device=self.conv1.weight.device)
        w1 = w1.index_put((self.r1, self.c1), self.conv1.weight.reshape(-1)[self.k1])
        w2 = torch.zeros(4 * 64, 9 * 32, dtype=self.conv2.weight.dtype, device=self.conv2.weight.device)
        w2 = w2.index_put((self.r2, self.c2), self.conv2.weight.reshape(-1)[self.k2])
        return w1, self.conv1.bias.repeat(9), w2, self.conv2.bias.repeat(4)

    def forward(self, x):
        d = self.dtype
        w1, b1, w2, b2 = self.dense_weights()
        h1 = F.relu(linear(x, w1, b1, d))               # [B, 9*32]  = conv 2x2 valid, 32 filters
        h2 = F.relu(linear(h1, w2, b2, d))              # [B, 4*64]  = conv 2x2 valid, 64 filters
        out = linear(h2, self.heads.weight, self.heads.bias, d).float()
        return out[:, :4], out[:, 4]


def make_net(kind, bf16=False):
    dt = torch.bfloat16 if bf16 else torch.float32
    return {"mlp": ActorCriticMLP, "cnn": ActorCriticCNN}[kind](dtype=dt)
