"""One training step of ResNet10Q (BASELINE config 5) with an explicit forward and backward on the
GPU -- the same arithmetic as `loss.backward()` through nets.py's custom-conv path, without
autograd's bookkeeping, and with the fusions it cannot express:

  * every conv of the forward sums its bf16 outputs per channel in its epilogue (r48_conv3x3
    `stats`), and the workgroup that writes the last per-CU record also FINISHES the BN (batch mean,
    invstd, apply coefficients, running statistics: r48_conv3x3_stats_finish, r48_bn_finish_args), so
    BN's forward is one apply pass (r48_bn_apply) with no statistics pass and no finish launch;
  * (fold_bn=True, opt-in) the apply of every BN but the last runs inside the NEXT conv's operand
    load (r48_conv3x3_bn_in): that conv reads the previous conv's output, forms relu(a x + b
    (+ identity)) per row as it loads it, and writes the result and its ReLU mask for the backward
    -- no separate apply pass and no re-read of z by the conv. Bit-identical, but measured 3 %
    SLOWER at the 64K minibatch (3.88 vs 3.76 ms per forward + backward, profiles/r04/dqn/bnfold.txt:
    the transform's VALU and the side-output stores sit on the conv's exposed load path), so the
    default keeps the separate apply passes;
  * every BN+ReLU forward writes a ReLU mask (1 bit per activation, r48_bn_forward `mask`), and
    its backward reads the mask instead of the 16x larger BN output;
  * every data-gradient conv reduces the BN backward of the layer below in its epilogue and finishes
    it in its last workgroup (r48_conv3x3_bn_grad with `fin`): its output IS that BN's output
    gradient, so BN's backward is one apply pass (r48_bn_backward_apply) with no reduction pass and
    no finish launch (only the last BN, fed by the head, reduces and finishes on its own);
  * a basic block's input gradient (first conv's data gradient + the identity path's gradient)
    is summed in the data-gradient conv's epilogue (r48_conv3x3_bn_grad `add`), not by a separate
    add -- and the identity path's gradient (the block output's gradient through its ReLU) is formed
    there from that gradient and the ReLU mask (`add_mask`), so the BN backward writes no masked
    copy of it (134 MB written and read back per block at the 64K minibatch);
  * parameter gradients are written straight into their .grad views of the flat gradient buffer
    (FlatParams): the convs' weight-gradient reduction, BN's dgamma/dbeta, the head's weight and
    bias gradient (one record);
  * activations live in buffers allocated once per batch size (9 conv outputs, 9 BN outputs).

Semantics = DQNLearner.learn's autograd path: Huber (smooth L1, beta 1) loss of Q(x)[action]
against the TD target, mean over the batch; BatchNorm in training mode (batch statistics, running
statistics updated with momentum, num_batches_tracked + 1); conv biases are constants (every conv
feeds a training-mode BN: their gradient is exactly zero). Differences from the autograd path are
summation order and bf16 rounding only (BN statistics summed unshifted in the conv epilogue, the
fused residual sum rounded once instead of twice): tests/test_dqn_gpu.py::
test_resnet_train_step_matches_autograd.
"""
import torch

from .. import _lib
from .._lib import check, ptr
from ..a3c.kernels import _stream
from .bn import _workspace
from .conv import conv3x3_wgrad, pack_resnet_train, q_head_backward, q_head_forward


def supported(net):
    """The fused step covers ResNet10Q with 64 channels, 4 blocks, BN, bf16 on the GPU."""
    return (getattr(net, "channels", None) == 64 and getattr(net, "n_blocks", None) == 4 and net.use_bn
            and net.dtype == torch.bfloat16 and next(net.parameters()).is_cuda)


class ResNetTrainStep:
    def __init__(self, net, fold_bn=False):
        if not supported(net):
            raise ValueError("ResNetTrainStep needs a bf16 CUDA ResNet10Q with 64 channels, 4 blocks and BN")
        self.net = net
        self.fold_bn = fold_bn
        self._bufs = {}

    def _buffers(self, B, dev):
        key = (B, str(dev))
        if key not in self._bufs:
            act = lambda: torch.empty((B, 16, 64), dtype=torch.bfloat16, device=dev)   # noqa: E731
            self._bufs.clear()            # one batch size at a time: the activations are large
            self._bufs[key] = {
                "y": [act() for _ in range(9)],                 # conv outputs (BN inputs)
                "z": [act() for _ in range(9)],                 # BN+ReLU outputs (next conv inputs)
                "m": [torch.empty((B * 16, 8), dtype=torch.uint8, device=dev) for _ in range(9)],
                "save": [torch.empty(128, dtype=torch.float32, device=dev) for _ in range(9)],
                "coef": [torch.empty(128, dtype=torch.float32, device=dev) for _ in range(9)],
                "bcoef": [torch.empty(192, dtype=torch.float32, device=dev) for _ in range(9)],
                "g": [act() for _ in range(5)],                 # gradient scratch
                "stem_dw": torch.empty((64, 32, 3, 3), dtype=torch.float32, device=dev),
                "loss": torch.empty(2, dtype=torch.float32, device=dev),        # mean loss, mean Q(s, a)
                # (zeroed: its last float is the finishing convs' arrival counter, reset by each finish)
                "stats": torch.zeros(int(_lib.load().r48_conv_stats_floats()), dtype=torch.float32, device=dev),
                "huber_ws": torch.empty(512, dtype=torch.float32, device=dev),
            }
        return self._bufs[key]

    def _fin_fwd(self, k, rows, save, coef):
        """r48_bn_finish_args of BN k's forward finish (kept alive until the launch has read it)."""
        bn = self.net.bns[k]
        mom = bn.momentum if bn.momentum is not None else 0.1
        self._fin = _lib.BnFinishArgs(bn.weight.data_ptr(), bn.bias.data_ptr(), bn.running_mean.data_ptr(),
                                      bn.running_var.data_ptr(), save.data_ptr(), coef.data_ptr(), None, None, rows,
                                      float(mom), float(bn.eps))
        return _lib.C.byref(self._fin)

    def _fin_bwd(self, k, rows, save, coef):
        """r48_bn_finish_args of BN k's backward finish: dgamma / dbeta into the flat gradient."""
        bn = self.net.bns[k]
        self._fin = _lib.BnFinishArgs(bn.weight.data_ptr(), None, None, None, save.data_ptr(), coef.data_ptr(),
                                      bn.weight.grad.data_ptr(), bn.bias.grad.data_ptr(), rows, 0.0, 0.0)
        return _lib.C.byref(self._fin)

    def _conv_finish(self, k, x, frags, bias, y, stats):
        """Forward conv into y (BN k's input) with BN k's finish in its last workgroup."""
        B, _, cin = x.shape
        check(_lib.load().r48_conv3x3_stats_finish(ptr(x), B, cin, ptr(frags), ptr(bias), ptr(y), ptr(stats),
                                                   self._fin_fwd(k, B * 16, self._S[k], self._CF[k]), _stream(x)))

    def _bn_apply(self, k, y, z, mask, residual=None):
        check(_lib.load().r48_bn_apply(ptr(y), ptr(residual), y.numel() // 64, 64, ptr(self._CF[k]), 1, ptr(z),
                                       ptr(mask), _stream(y)))

    def _bn_backward_apply(self, k, dz, dy):
        check(_lib.load().r48_bn_backward_apply(ptr(dz), ptr(self._M[k]), ptr(self._Y[k]), dz.numel() // 64, 64,
                                                ptr(self._BC[k]), ptr(dy), _stream(dz)))

    def _conv_bn_in(self, y_prev, coef, res, z_out, m_out, frags, bias, y, stats, fin=None):
        check(_lib.load().r48_conv3x3_bn_in(ptr(y_prev), y_prev.shape[0], ptr(frags), ptr(bias), ptr(coef), ptr(res),
                                            ptr(z_out), ptr(m_out), ptr(y), ptr(stats), fin, _stream(y_prev)))

    def _conv_bn_grad(self, dy, frags, out, k, add=None, add_mask=None, part=None):
        """out = data gradient conv of dy (+ add . [add_mask]) -- the gradient reaching BN k's output --
        with BN k's backward reduction summed into `part` and finished (coefficients into bcoef[k],
        dgamma / dbeta) in the same launch."""
        fin = self._fin_bwd(k, dy.shape[0] * 16, self._S[k], self._BC[k])
        check(_lib.load().r48_conv3x3_bn_grad(ptr(dy), dy.shape[0], ptr(frags), ptr(add), ptr(add_mask), ptr(out),
                                              ptr(self._Y[k]), ptr(self._M[k]), ptr(self._S[k]), ptr(part), fin,
                                              _stream(dy)))
        return out

    def _bn_backward(self, k, dz, mask, y, save, dy, dres=None):
        bn = self.net.bns[k]
        rows = y.numel() // 64
        check(_lib.load().r48_bn_backward(ptr(dz), None, ptr(mask), ptr(y), rows, 64, ptr(bn.weight), ptr(save), 1,
                                          ptr(_workspace(rows, 64, y.device)), ptr(dy), ptr(dres),
                                          ptr(bn.weight.grad), ptr(bn.bias.grad), _stream(y)))

    def __call__(self, x, action, target):
        """x bf16 [B, 16 * 32] (board_onehot32 planes), action [B] (int), target fp32 [B] ->
        (loss, mean Q(x)[action]) as 0-d tensors; gradients written into the parameters' .grad
        (conv biases untouched: their gradient is zero)."""
        net = self.net
        B = x.shape[0]
        x = x.reshape(B, 16, 32)
        buf = self._buffers(B, x.device)
        Y, Z, M, S, G = buf["y"], buf["z"], buf["m"], buf["save"], buf["g"]
        convs = net.conv_layers()
        fwd, dgrad = pack_resnet_train(convs)             # one launch, all 17 fragment sets
        # ---- forward
        torch._foreach_add_([m.num_batches_tracked for m in net.bns], 1)   # one launch for the 9 BNs
        st = buf["stats"]                                  # the conv epilogues' BN sums
        self._Y, self._M, self._S, self._CF, self._BC = Y, M, S, buf["coef"], buf["bcoef"]
        rows = B * 16
        self._conv_finish(0, x, fwd[0], convs[0].bias, Y[0], st)
        if self.fold_bn:
            # conv k applies BN k - 1 (+ the block's identity for k - 1 = 2, 4, 6) to its input rows
            # and writes Z[k - 1], M[k - 1], and finishes BN k; the last BN (into the head) is applied
            # on its own
            CF = self._CF
            for k in range(1, 9):
                res = Z[k - 3] if (k - 1) % 2 == 0 and k - 1 >= 2 else None
                self._conv_bn_in(Y[k - 1], CF[k - 1], res, Z[k - 1], M[k - 1], fwd[k], convs[k].bias, Y[k], st,
                                 fin=self._fin_fwd(k, rows, S[k], CF[k]))
            self._bn_apply(8, Y[8], Z[8], M[8], residual=Z[6])
        else:
            self._bn_apply(0, Y[0], Z[0], M[0])
            for b in range(4):
                i1, i2 = 1 + 2 * b, 2 + 2 * b
                h = Z[i1 - 1]
                self._conv_finish(i1, h, fwd[i1], convs[i1].bias, Y[i1], st)
                self._bn_apply(i1, Y[i1], Z[i1], M[i1])
                self._conv_finish(i2, Z[i1], fwd[i2], convs[i2].bias, Y[i2], st)
                self._bn_apply(i2, Y[i2], Z[i2], M[i2], residual=h)
        h = Z[8].view(B, 1024)
        hw_bf16 = net.head.weight.detach().to(torch.bfloat16)      # one cast for the head's two kernels
        q = q_head_forward(h, hw_bf16, net.head.bias)
        # ---- Huber loss of Q(x)[action] and its gradient (d loss / d q): one kernel + one finish
        a8 = action if action.dtype == torch.int8 else action.to(torch.int8)
        dq = torch.empty_like(q)
        stats = buf["loss"]
        check(_lib.load().r48_huber_grad(ptr(q), ptr(a8.contiguous()), ptr(target.float().contiguous()), B, ptr(dq),
                                         ptr(stats), ptr(buf["huber_ws"]), _stream(q)))
        # ---- backward
        hw, hb = net.head.weight.grad, net.head.bias.grad
        fused_head = hb.data_ptr() == hw.data_ptr() + 4 * hw.numel()        # one record: weight rows, bias
        dh, dw, db = q_head_backward(dq, h, hw_bf16, out=hw if fused_head else None)
        if not fused_head:
            hw.copy_(dw)
            hb.copy_(db)
        # per block, backwards: BN2 (+ identity) -> conv2 data/weight gradients -> BN1 -> conv1
        # data gradient + identity gradient (one epilogue: cur . [M[i2]]) and weight gradient. The
        # incoming gradient alternates between g[0] and g[4] (cur stays intact until the block's
        # last conv has read it); g[1..3] hold the block's temporaries.
        # Every data-gradient conv also reduces and finishes the BN backward of the layer below (its
        # output is that BN's output gradient); only BN 8's (the head's gradient) runs on its own.
        part = buf["stats"]
        cur = dh.view(B, 16, 64)
        for b in range(3, -1, -1):
            i1, i2 = 1 + 2 * b, 2 + 2 * b
            h_in = Z[i1 - 1]
            dy2, dz1, dy1 = G[1], G[2], G[3]
            if b == 3:
                self._bn_backward(i2, cur, M[i2], Y[i2], S[i2], dy2)
            else:
                self._bn_backward_apply(i2, cur, dy2)
            self._conv_bn_grad(dy2, dgrad[i2], dz1, i1, part=part)
            conv3x3_wgrad(dy2, Z[i1], out=convs[i2].weight.grad)
            self._bn_backward_apply(i1, dz1, dy1)
            nxt = G[4] if cur is G[0] else G[0]
            self._conv_bn_grad(dy1, dgrad[i1], nxt, i1 - 1, add=cur, add_mask=M[i2], part=part)
            conv3x3_wgrad(dy1, h_in, out=convs[i1].weight.grad)
            cur = nxt
        dy0 = G[1]
        self._bn_backward_apply(0, cur, dy0)
        conv3x3_wgrad(dy0, x, out=buf["stem_dw"])
        convs[0].weight.grad.copy_(buf["stem_dw"][:, :convs[0].weight.shape[1]])
        return stats[0], stats[1]
