"""TF1 RMSProp over a flat parameter buffer + synchronous gradient all-reduce.

The reference applies each worker's gradients to the shared global net with
tf.train.RMSPropOptimizer(1e-3) (a3c.py:79-80, 264-265) -- Hogwild, asynchronous. Here every
replica (one per GPU) holds the net, gradients are averaged with ONE all-reduce of one flat fp32
buffer per update (RCCL over xGMI on GPUs; the net is ~2.5 k (MLP) / ~38 k (CNN) parameters, so
the message is latency-bound, never link-bound), and every replica applies the same update.

FlatParams re-points every parameter and its .grad at views of two contiguous buffers, so the
all-reduce and the optimizer are one call each. On GPU tensors the TF1 update is the fused HIP
kernel r48_rmsprop_tf1 (one launch for all parameters); on CPU tensors (the CPU test-suite)
the same arithmetic runs as torch ops.
"""
import torch
import torch.distributed as dist


def _staged(collective, t, group, **kw):
    """Run `collective` on t. gloo has no device path on every build, so a GPU tensor under
    gloo (the two-ranks-on-one-GPU tests) goes through a host copy; RCCL takes it in place."""
    if t.is_cuda and dist.get_backend(group) == "gloo":
        h = t.cpu()
        collective(h, group=group, **kw)
        t.copy_(h)
    else:
        collective(t, group=group, **kw)


class FlatParams:
    EXTRA = 8

    def __init__(self, module):
        params = [p for p in module.parameters() if p.requires_grad]
        self.params = params
        dev, dt = params[0].device, params[0].dtype
        total = sum(p.numel() for p in params)
        self.data = torch.zeros(total, dtype=dt, device=dev)
        # the gradient is the head of the all-reduce message; its tail carries up to EXTRA reported
        # scalars (losses, ...) so they are averaged by the same collective
        self._msg = torch.zeros(total + self.EXTRA, dtype=dt, device=dev)
        self.grad = self._msg[:total]
        off = 0
        for p in params:
            k = p.numel()
            self.data[off:off + k].copy_(p.data.view(-1))
            p.data = self.data[off:off + k].view_as(p)
            p.grad = self.grad[off:off + k].view_as(p)
            off += k

    def zero_grad(self):
        self.grad.zero_()

    def allreduce_grad(self, group=None, extras=None):
        """Average the gradient over the process group (one collective). `extras` (a 1-d tensor of
        at most EXTRA scalars, e.g. the losses) is averaged by the same all-reduce; returns it
        (averaged; unchanged on one rank), or None."""
        total, k = self.grad.numel(), 0
        if extras is not None:
            extras = extras.reshape(-1)
            k = extras.numel()
            if k > self.EXTRA:
                raise ValueError("at most %d extra scalars ride the gradient all-reduce" % self.EXTRA)
        if dist.is_available() and dist.is_initialized():
            world = dist.get_world_size(group)
            if world > 1:
                msg = self._msg[:total + k]
                if k:
                    msg[total:].copy_(extras)
                _staged(dist.all_reduce, msg, group, op=dist.ReduceOp.SUM)
                msg.div_(world)
                return msg[total:].clone() if k else None
        return extras

    def broadcast_(self, src=0, group=None):
        """Start every replica from rank src's parameters."""
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
            _staged(dist.broadcast, self.data, group, src=src)


class FlatBuffers:
    """The floating-point buffers of a module (BatchNorm running_mean / running_var) re-pointed at
    views of ONE contiguous buffer. Each replica updates them from its own minibatch; averaging
    them over the group after every update (one all-reduce) keeps the replicas identical -- the
    running statistics are a linear function of the batch statistics, so the average equals what
    one replica would hold after the same update on the union of the minibatches' means. Integer
    buffers (num_batches_tracked) advance identically on every replica and are left alone."""

    def __init__(self, module):
        bufs = [b for b in module.buffers() if b.is_floating_point()]
        self.buffers = bufs
        if not bufs:
            self.data = torch.zeros(0)
            return
        dev, dt = bufs[0].device, bufs[0].dtype
        self.data = torch.zeros(sum(b.numel() for b in bufs), dtype=dt, device=dev)
        off = 0
        for b in bufs:
            k = b.numel()
            self.data[off:off + k].copy_(b.data.view(-1))
            b.data = self.data[off:off + k].view_as(b)
            off += k

    def allreduce_mean_(self, group=None):
        if self.data.numel() and dist.is_available() and dist.is_initialized():
            world = dist.get_world_size(group)
            if world > 1:
                _staged(dist.all_reduce, self.data, group, op=dist.ReduceOp.SUM)
                self.data.div_(world)

    def broadcast_(self, src=0, group=None):
        if self.data.numel() and dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
            _staged(dist.broadcast, self.data, group, src=src)


class RMSPropTF1:
    """tf.train.RMSPropOptimizer semantics: ms slot initialised to ONES, eps inside the sqrt,
    decay 0.9, momentum 0 (a3c.py:264-265 uses the defaults with lr 1e-3)."""

    def __init__(self, flat, lr=1e-3, decay=0.9, momentum=0.0, eps=1e-10):
        self.flat = flat
        self.lr, self.decay, self.momentum, self.eps = lr, decay, momentum, eps
        self.ms = torch.ones_like(flat.data)
        self.mom = torch.zeros_like(flat.data)

    @torch.no_grad()
    def step(self):
        d, g = self.flat.data, self.flat.grad
        if d.is_cuda:
            from .kernels import rmsprop_tf1_
            rmsprop_tf1_(d, g, self.ms, self.mom, self.lr, self.decay, self.momentum, self.eps)
        else:
            self.ms.mul_(self.decay).addcmul_(g, g, value=1.0 - self.decay)
            self.mom.mul_(self.momentum).addcdiv_(g, (self.ms + self.eps).sqrt(), value=self.lr)
            d.sub_(self.mom)
