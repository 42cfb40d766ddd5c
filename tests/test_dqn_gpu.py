"""Config-5 kernels and trainer on the GPU vs the float64 oracle (oracle/dqn_ref.py).

One-hot planes (exact), epsilon-greedy (exact given the Philox draw), TD target (fp32 vs f64),
ResNet-10 forward in fp32 (vs f64) and bf16 (vs f64, bounded by PyTorch's own bf16 rounding),
and one DQN update whose loss equals the oracle's recomputation from the sampled minibatch and
the pre-update weights.
"""
import numpy as np
import pytest
import torch

from oracle import dqn_ref as R
from oracle import native as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_onehot_exact():
    from rein48_amd.dqn.kernels import board_onehot
    b = np.random.default_rng(0).integers(0, 18, size=(10_001, 16)).astype(np.int8)
    t = torch.from_numpy(b).to(DEV)
    want = R.onehot(b).reshape(-1, 16 * 18)
    np.testing.assert_array_equal(board_onehot(t, dtype=torch.float32).cpu().numpy(), want)
    np.testing.assert_array_equal(board_onehot(t, dtype=torch.bfloat16).float().cpu().numpy(), want)


def test_egreedy_exact():
    from rein48_amd.dqn.kernels import egreedy_actions
    rng = np.random.default_rng(1)
    n, seed, ctr, gid0, eps = 100_000, 5, 9, 300, 0.3
    q = rng.normal(size=(n, 4)).astype(np.float32)
    q[::7, 1] = q[::7, 0]                                          # ties -> first argmax
    got = egreedy_actions(torch.from_numpy(q).to(DEV), eps, seed, ctr, gid0=gid0).cpu().numpy()
    idx = np.arange(0, n, 53)
    w = np.array([O.philox([(gid0 + i) & 0xFFFFFFFF, (gid0 + i) >> 32, ctr, 0xD0E], [seed, 0]) for i in idx],
                 np.uint64)
    u = (w[:, 0] >> 8).astype(np.float64) / 16777216.0
    want = R.egreedy(q[idx], u, (w[:, 1] >> 30).astype(np.int64), eps)
    np.testing.assert_array_equal(got[idx], want)
    assert abs((got != q.argmax(1)).mean() - eps * 0.75) < 0.01    # 3/4 of random picks differ


@pytest.mark.parametrize("double", [False, True])
def test_td_target_matches_oracle(double):
    from rein48_amd.dqn.kernels import td_target
    rng = np.random.default_rng(2)
    n = 50_001
    r = rng.normal(size=n).astype(np.float32)
    d = (rng.random(n) < 0.2).astype(np.uint8)
    qt, qo = (rng.normal(size=(n, 4)).astype(np.float32) for _ in range(2))
    T = lambda a: torch.from_numpy(a).to(DEV)
    y = td_target(T(r), T(d), T(qt), T(qo) if double else None, 0.97).cpu().numpy()
    np.testing.assert_allclose(y, R.td_target(r, d, qt, qo if double else None, 0.97), rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("double", [False, True])
def test_td_target_log2_reward_equals_torch_transform(double):
    """log2_reward folds the trainer's reward transform (torch.log2(1.0 + r), trainer.py _reward) into
    the TD-target launch: bit-equal to the kernel on the transformed rewards, on merge rewards (0 and
    sums of tiles up to 2^17) and on arbitrary non-negative floats."""
    from rein48_amd.dqn.kernels import td_target
    rng = np.random.default_rng(3)
    n = 40_003
    r = np.where(rng.random(n) < 0.5, 0.0, 2.0 ** rng.integers(1, 18, n) * rng.integers(1, 4, n)).astype(np.float32)
    r[: n // 4] = rng.random(n // 4).astype(np.float32) * 1e3
    d = (rng.random(n) < 0.2).astype(np.uint8)
    qt, qo = (rng.normal(size=(n, 4)).astype(np.float32) for _ in range(2))
    T = lambda a: torch.from_numpy(a).to(DEV)
    rt = T(r)
    got = td_target(rt, T(d), T(qt), T(qo) if double else None, 0.97, log2_reward=True)
    want = td_target(torch.log2(1.0 + rt), T(d), T(qt), T(qo) if double else None, 0.97)
    assert torch.equal(got, want)


def _params(net):
    return {"convs": [(c.weight.detach().double().cpu().numpy(), c.bias.detach().double().cpu().numpy())
                      for c in net.conv_layers()],
            "bns": [dict(mean=m.running_mean.double().cpu().numpy(), var=m.running_var.double().cpu().numpy(),
                         gamma=m.weight.detach().double().cpu().numpy(), beta=m.bias.detach().double().cpu().numpy())
                    for m in net.bns] if net.use_bn else None,
            "head": (net.head.weight.detach().double().cpu().numpy(), net.head.bias.detach().double().cpu().numpy())}


def test_resnet10_gpu_matches_oracle():
    """fp32 forward vs f64 within 1e-4 and the bf16 forward within 5e-2, both as max |error|
    relative to mean |Q| (bf16 rounds inputs, weights and activations; fp32 accumulation)."""
    from rein48_amd.dqn.kernels import board_onehot
    from rein48_amd.dqn.nets import ResNet10Q
    torch.manual_seed(0)
    net = ResNet10Q().to(DEV).eval()
    with torch.no_grad():
        for m in net.bns:
            m.running_mean.uniform_(-0.2, 0.2)
            m.running_var.uniform_(0.5, 2.0)
        net.head.weight.normal_(std=0.05)
    b = np.random.default_rng(3).integers(0, 12, size=(512, 16)).astype(np.int8)
    bt = torch.from_numpy(b).to(DEV)
    want = R.resnet10_q(_params(net), b)
    scale = np.abs(want).mean()
    with torch.no_grad():
        q32 = net(board_onehot(bt, dtype=torch.float32)).cpu().numpy()
        net.dtype = torch.bfloat16
        q16 = net(board_onehot(bt, dtype=torch.bfloat16)).cpu().numpy()
    e32 = np.abs(q32 - want).max() / scale
    e16 = np.abs(q16 - want).max() / scale
    assert e32 < 1e-4, e32
    assert e16 < 5e-2, e16


def test_dqn_update_loss_matches_oracle():
    """fp32, no BN (train-mode BN would use batch statistics the eval-mode oracle does not
    model): the reported Huber loss of one update equals the oracle's recomputation from the
    sampled minibatch with the pre-update online and target weights (double DQN)."""
    from rein48_amd.dqn import DQNConfig, DQNTrainer
    cfg = DQNConfig(n_boards=2048, replay_capacity=1 << 16, batch=1024, learn_start=1 << 30, bn=False, bf16=False,
                    channels=16, blocks=2, seed=7, double=True, gamma=0.95)
    tr = DQNTrainer(cfg, device=DEV)
    for _ in range(6):
        tr.train_step()
    assert len(tr.replay) == 6 * 2048
    with torch.no_grad():                                            # make target != online
        for p in tr.target.parameters():
            p.add_(0.01 * torch.randn_like(p))
    p_on, p_tg = _params(tr.net), _params(tr.target)
    out = tr.update(sync=False)                                      # the loss as a 0-d GPU tensor
    assert torch.is_tensor(out["loss"]) and out["loss"].is_cuda
    out["loss"] = float(out["loss"])
    b = {k: v.cpu().numpy() for k, v in out["batch"].items()}
    q = R.resnet10_q(p_on, b["state"])[np.arange(len(b["action"])), b["action"].astype(np.int64)]
    y = R.td_target(np.log2(1.0 + b["reward"].astype(np.float64)), b["done"], R.resnet10_q(p_tg, b["next_state"]),
                    R.resnet10_q(p_on, b["next_state"]), 0.95)
    np.testing.assert_allclose(out["loss"], R.huber(q, y), rtol=1e-4, atol=1e-6)
    assert any(not np.allclose(a, c) for a, c in zip(p_on["convs"][0], _params(tr.net)["convs"][0]))


def test_dqn_bf16_resnet10_trains():
    from rein48_amd.dqn import DQNConfig, DQNTrainer
    cfg = DQNConfig(n_boards=4096, replay_capacity=1 << 17, batch=2048, learn_start=8192, seed=1, target_sync=2)
    tr = DQNTrainer(cfg, device=DEV)
    outs = [tr.train_step() for _ in range(5)]
    assert np.isnan(outs[0]["loss"]) and all(np.isfinite(o["loss"]) for o in outs[1:])
    assert tr.updates == 4 and len(tr.replay) == 5 * 4096          # learn_start reached at step 2
    assert tr.epsilon() < 1.0
    for a, b in zip(tr.target.state_dict().values(), tr.net.state_dict().values()):
        assert torch.equal(a, b)                                     # synced after update 4


@pytest.mark.parametrize("pack", ["host", "gpu"])
@pytest.mark.parametrize("empty_frac", [0.4, 0.9])
def test_fused_resnet_matches_torch(empty_frac, pack):
    """r48_resnet_q_forward (bf16 16x16x32 MFMA, columns = 16 boards of one cell, in-grid taps
    only, activations in registers, eval-mode BN folded; weights packed by pack_resnet or
    r48_resnet_pack) vs the PyTorch ResNet10Q. Error metric: max |got - ref| / (|ref| +
    mean|ref|). Against fp32 the kernel's error is within 1.5x (+1e-3) of PyTorch's own bf16
    forward's error and below 5e-2; the fused epsilon-greedy draw equals r48_egreedy_actions on
    the kernel's own Q."""
    from rein48_amd.dqn.fused import pack_resnet, pack_resnet_gpu, resnet_q_forward
    from rein48_amd.dqn.kernels import board_onehot, egreedy_actions
    from rein48_amd.dqn.nets import ResNet10Q
    torch.manual_seed(5)
    net = ResNet10Q().to(DEV).eval()
    with torch.no_grad():
        for m in net.bns:
            m.running_mean.uniform_(-0.3, 0.3)
            m.running_var.uniform_(0.5, 2.0)
            m.weight.uniform_(0.5, 1.5)
            m.bias.uniform_(-0.2, 0.2)
        for c in net.conv_layers():
            c.bias.uniform_(-0.2, 0.2)
        net.head.weight.normal_(std=0.05)
        net.head.bias.uniform_(-1, 1)
    rng = np.random.default_rng(6)
    n = 100_003                                    # a partial last tile
    b = rng.integers(1, 16, size=(n, 16)).astype(np.int8)
    b[rng.random((n, 16)) < empty_frac] = 0
    b[:5] = np.arange(16, dtype=np.int8)[None] % 18  # every plane incl. 15, and one 17-tile board
    b[5, 3] = 17
    bt = torch.from_numpy(b).to(DEV)
    packed = pack_resnet(net) if pack == "host" else pack_resnet_gpu(net)
    fwd = resnet_q_forward
    q, _ = fwd(bt, packed)
    with torch.no_grad():
        ref32 = net(board_onehot(bt, dtype=torch.float32))
        net.dtype = torch.bfloat16
        ref16 = net(board_onehot(bt, dtype=torch.bfloat16))

    def worst(a, r):
        return float(((a - r).abs() / (r.abs() + r.abs().mean())).max())

    e_k, e_t = worst(q, ref32), worst(ref16, ref32)
    assert e_k <= 1.5 * e_t + 1e-3 and e_k <= 5e-2, (e_k, e_t)
    _, act = fwd(bt, packed, q=False, actions=True, eps=0.25, seed=11, ctr=3, gid0=40)
    assert torch.equal(act, egreedy_actions(q, 0.25, 11, 3, gid0=40))


def _bn_case(rows, C, res, relu, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(rows, C, generator=g) * (torch.rand(C, generator=g) * 2 + 0.5) + torch.randn(C, generator=g) * 3
    r = torch.randn(rows, C, generator=g) if res else None
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g) * 0.3
    dy = torch.randn(rows, C, generator=g).to(torch.bfloat16).float()
    return x, r, gamma, beta, dy


def _torch_bn_act(x, r, gamma, beta, rm, rv, relu, dtype):
    """torch.nn.functional reference in `dtype` (fp32: the reference; bf16: torch's own rounding)."""
    xs = x.to(DEV, dtype).requires_grad_(True)
    gs, bs = gamma.to(DEV).requires_grad_(True), beta.to(DEV).requires_grad_(True)
    z = torch.nn.functional.batch_norm(xs, rm, rv, gs, bs, training=True, momentum=0.1, eps=1e-5)
    rs = None
    if r is not None:
        rs = r.to(DEV, dtype).requires_grad_(True)
        z = z + rs
    y = torch.relu(z) if relu else z
    return xs, rs, gs, bs, y


@pytest.mark.parametrize("rows,C,res,relu", [(1 << 16, 64, False, True), (1 << 16, 64, True, True),
                                             (100_003, 64, True, False), (4099, 32, False, True),
                                             (20_000, 128, True, True)])
def test_fused_bn_act_matches_torch(rows, C, res, relu):
    """r48_bn_forward / r48_bn_backward (bn.py) vs F.batch_norm (+ add, ReLU) in training mode.
    Forward y and backward dx / d(residual) are bf16: their error vs the fp32 reference is within
    1.5x (+1e-3) of PyTorch's own bf16 path's error; so are dgamma / dbeta (fp32 sums over all
    rows; + 1e-3 of their mean magnitude); running statistics (fp32) within 1e-4. All paths see
    the same bf16-representable x, residual and dy. Channel means are offset by up to ~3
    std-devs (the shifted sums must not cancel)."""
    from rein48_amd.dqn.bn import bn_act
    x, r, gamma, beta, dy = _bn_case(rows, C, res, relu, seed=rows + C)
    ref_rm, ref_rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    x = x.to(torch.bfloat16).float()             # every path sees the same (bf16-representable) input
    if res:
        r = r.to(torch.bfloat16).float()
    xs, rs, gs, bs, y32 = _torch_bn_act(x, r, gamma, beta, ref_rm, ref_rv, relu, torch.float32)
    y32.backward(dy.to(DEV))
    t_rm, t_rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    xt, rt, gt, bt, y16 = _torch_bn_act(x, r, gamma, beta, t_rm, t_rv, relu, torch.bfloat16)
    y16.backward(dy.to(DEV, torch.bfloat16))

    bn = torch.nn.BatchNorm1d(C).to(DEV).train()
    with torch.no_grad():
        bn.weight.copy_(gamma)
        bn.bias.copy_(beta)
    xk = x.to(DEV, torch.bfloat16).requires_grad_(True)
    rk = r.to(DEV, torch.bfloat16).requires_grad_(True) if res else None
    yk = bn_act(xk, bn, rk, relu=relu)
    yk.backward(dy.to(DEV, torch.bfloat16))

    def worst(a, ref):
        a, ref = a.detach().float(), ref.detach().float()
        return float(((a - ref).abs() / (ref.abs() + ref.abs().mean())).max())

    for got, torch16, ref in ((yk, y16, y32), (xk.grad, xt.grad, xs.grad)) + \
            (((rk.grad, rt.grad, rs.grad),) if res else ()):
        e_k, e_t = worst(got, ref), worst(torch16, ref)
        assert e_k <= 1.5 * e_t + 1e-3, (e_k, e_t)
    for got, torch16, ref in ((bn.weight.grad, gt.grad, gs.grad), (bn.bias.grad, bt.grad, bs.grad)):
        e_k, e_t = float((got - ref).abs().max()), float((torch16 - ref).abs().max())
        assert e_k <= 1.5 * e_t + 1e-3 * float(ref.abs().mean()), (e_k, e_t)
    torch.testing.assert_close(bn.running_mean, ref_rm, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bn.running_var, ref_rv, rtol=1e-4, atol=1e-4)
    assert int(bn.num_batches_tracked) == 1
    yk2 = bn_act(xk.detach(), bn, None if rk is None else rk.detach(), relu=relu)   # deterministic
    assert torch.equal(bn_act(xk.detach(), bn, None if rk is None else rk.detach(), relu=relu), yk2)


def test_resnet_update_fused_bn_matches_torch_bn():
    """One training forward/backward of the bf16 ResNet10Q with the fused BN path vs the same
    net through torch's BatchNorm1d: losses agree to bf16 precision and every parameter gradient
    is close in relative norm (both are bf16 computations of the same fp32 function)."""
    from rein48_amd.dqn.kernels import board_onehot
    from rein48_amd.dqn.nets import ResNet10Q
    torch.manual_seed(9)
    net = ResNet10Q(dtype=torch.bfloat16).to(DEV).train()
    with torch.no_grad():
        net.head.weight.normal_(std=0.05)
    b = torch.from_numpy(np.random.default_rng(9).integers(0, 12, size=(8192, 16)).astype(np.int8)).to(DEV)
    x = board_onehot(b, dtype=torch.bfloat16)
    tgt = torch.randn(8192, 4, device=DEV)
    grads, losses, stats = [], [], []
    for fused in (True, False):
        net.fused_bn = fused
        net.zero_grad()
        for m in net.bns:
            m.reset_running_stats()
        loss = torch.nn.functional.smooth_l1_loss(net(x), tgt)
        loss.backward()
        losses.append(float(loss.detach()))
        # conv biases feed a BN, which removes them: their exact gradient is 0 and both paths
        # return rounding noise, so they are not compared
        grads.append([p.grad.detach().float().clone() for k, p in net.named_parameters()
                      if not (k.endswith(".bias") and (k.startswith("stem") or k.startswith("convs")))])
        stats.append([m.running_var.clone() for m in net.bns])
    assert abs(losses[0] - losses[1]) <= 1e-2 * abs(losses[1])
    for ga, gb in zip(*grads):
        assert float((ga - gb).norm()) <= 5e-2 * float(gb.norm()) + 1e-6
    for sa, sb in zip(*stats):
        torch.testing.assert_close(sa, sb, rtol=1e-2, atol=1e-3)


@pytest.mark.parametrize("ci", [18, 64])
def test_structured_conv_weight_kernels_match_cpu_map(ci):
    """r48_struct_conv_weight / _grad (one HIP pass each way) == the CPU index_put / index_add
    map of nets._StructuredConvWeight: forward exact in fp32 and equal to the rounded fp32 matrix
    in bf16; gradient within fp32 summation-order error, for the stem (ci = 18) and a block conv."""
    from rein48_amd.dqn.nets import _StructuredConvWeight
    torch.manual_seed(ci)
    co = 64
    w = torch.randn(co, ci, 3, 3, dtype=torch.float32)
    want = _StructuredConvWeight.apply(w, torch.float32)
    got32 = _StructuredConvWeight.apply(w.to(DEV), torch.float32)
    got16 = _StructuredConvWeight.apply(w.to(DEV), torch.bfloat16)
    assert torch.equal(got32.cpu(), want)
    assert torch.equal(got16.cpu(), want.to(torch.bfloat16))
    gd = torch.randn(16 * co, 16 * ci, dtype=torch.float32)
    wc = w.clone().requires_grad_(True)
    _StructuredConvWeight.apply(wc, torch.float32).backward(gd)
    for dt in (torch.float32, torch.bfloat16):
        wg = w.to(DEV).requires_grad_(True)
        _StructuredConvWeight.apply(wg, dt).backward(gd.to(DEV, dt))
        ref = wc.grad if dt == torch.float32 else None
        if ref is None:                                   # bf16 gradient input: the CPU map of the rounded gd
            wr = w.clone().requires_grad_(True)
            _StructuredConvWeight.apply(wr, torch.float32).backward(gd.to(torch.bfloat16).float())
            ref = wr.grad
        torch.testing.assert_close(wg.grad.cpu(), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("bn", [True, False])
def test_gpu_weight_packing_equals_pack_resnet(bn):
    """r48_resnet_pack (one launch: BN fold, 16x16x32 fragments incl. the head) == the PyTorch
    pack_resnet. The layout is exact (without BN: bit for bit); with BN the scale gamma /
    sqrt(var + eps) may differ from PyTorch's in the last f32 ulp (its division / sqrt kernels
    are not guaranteed correctly rounded), so the folded f32 biases agree to 1e-6 relative and the
    bf16 weights to one bf16 ulp on < 0.1 % of elements. Repacking into the same buffer after a
    weight change tracks it."""
    from rein48_amd.dqn.fused import pack_resnet, pack_resnet_gpu
    from rein48_amd.dqn.nets import ResNet10Q
    torch.manual_seed(12)
    net = ResNet10Q(bn=bn).to(DEV).eval()
    with torch.no_grad():
        if bn:
            for m in net.bns:
                m.running_mean.uniform_(-0.3, 0.3)
                m.running_var.uniform_(0.5, 2.0)
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
        for c in net.conv_layers():
            c.bias.uniform_(-0.2, 0.2)
        net.head.bias.uniform_(-1, 1)
    stem, conv, head = 37, 73, 33
    bias_rows = [stem - 1] + [stem + conv * L + conv - 1 for L in range(8)] + [stem + 8 * conv + head - 1]

    def check(got, want):
        frags, wf = got.view(torch.int16).long().view(-1, 512), want.view(torch.int16).long().view(-1, 512)
        assert frags.shape[0] == stem + 8 * conv + head
        is_bias = torch.zeros(frags.shape[0], dtype=torch.bool, device=DEV)
        is_bias[bias_rows] = True
        diff = (frags[~is_bias] - wf[~is_bias]).abs()
        if not bn:
            assert int(diff.max()) == 0
        else:
            assert int(diff.max()) <= 1 and float((diff > 0).float().mean()) < 1e-3
        gb = got.view(-1, 512)[is_bias].contiguous().view(torch.float32)
        wb = want.view(-1, 512)[is_bias].contiguous().view(torch.float32)
        torch.testing.assert_close(gb, wb, rtol=1e-6, atol=1e-7)

    got = pack_resnet_gpu(net)
    check(got, pack_resnet(net))
    with torch.no_grad():
        net.convs[3].weight.mul_(1.5)
    got = pack_resnet_gpu(net, out=got)
    check(got, pack_resnet(net))


def test_fused_resnet_tile_edges_bit_identical():
    """Every board's Q is computed in its own MFMA column with a fixed summation order, so the
    result must not depend on n or on where the board sits in its 64-board tile / persistent
    loop: Q(boards[:n]) equals Q(boards)[:n] bit for bit at the tile edges (1, 15, 16, 17, 63, 64,
    65, 257 boards and 256 CUs' worth + 1), and n = 0 launches nothing."""
    from rein48_amd.dqn.fused import pack_resnet_gpu, resnet_q_forward
    from rein48_amd.dqn.nets import ResNet10Q
    torch.manual_seed(31)
    net = ResNet10Q().to(DEV).eval()
    with torch.no_grad():
        net.head.weight.normal_(std=0.05)
    blob = pack_resnet_gpu(net)
    b = torch.from_numpy(np.random.default_rng(31).integers(0, 14, size=(40_000, 16)).astype(np.int8)).to(DEV)
    full, _ = resnet_q_forward(b, blob)
    for n in (1, 15, 16, 17, 63, 64, 65, 257, 256 * 64 + 1):
        q, _ = resnet_q_forward(b[:n].contiguous(), blob)
        assert torch.equal(q.view(torch.int32), full[:n].view(torch.int32)), n
    q0, a0 = resnet_q_forward(b[:0].contiguous(), blob, actions=True)
    assert q0.shape == (0, 4) and a0.shape == (0,)


# ---------------------------------------------------------------- the update's 3x3 conv kernels
def _rel(a, b):
    return float((a.float() - b.float()).abs().max()) / max(float(b.float().abs().max()), 1e-30)


@pytest.mark.parametrize("ci,B", [(64, 4099), (18, 1037), (64, 16)])
def test_conv3x3_kernels_match_torch_conv2d(ci, B):
    """r48_conv3x3 (forward and, with the flipped transposed taps, the data gradient) and
    r48_conv3x3_wgrad vs torch.nn.functional.conv2d (padding 1) in fp32 on the same bf16-rounded
    inputs: the kernels accumulate in fp32 over bf16 products like the reference computation, so
    the only differences are summation order and the bf16 rounding of the kernel outputs (forward,
    data gradient: <= 1e-2 relative to the largest value; weight gradient, fp32 out: <= 2e-3).
    Ragged board counts (tails of a 16-board tile and of a 4-board staging step) included."""
    import torch.nn.functional as F
    from rein48_amd.dqn.conv import board_onehot32, conv3x3, conv3x3_wgrad, pack_conv, pack_conv_dgrad
    g = torch.Generator(device="cpu").manual_seed(ci * 7 + B)
    w = (torch.randn(64, ci, 3, 3, generator=g) * 0.1).to(DEV)
    bias = (torch.randn(64, generator=g) * 0.5).to(DEV)
    if ci == 18:   # the stem: one-hot planes of exponents, padded to 32 channels
        boards = torch.randint(0, 18, (B, 16), generator=g, dtype=torch.int8).to(DEV)
        x = board_onehot32(boards)
        x_ref = x[:, :, :18].float()
    else:
        x = torch.randn(B, 16, ci, generator=g).to(DEV).to(torch.bfloat16)
        x_ref = x.float()
    xi = x_ref.permute(0, 2, 1).reshape(B, ci, 4, 4).requires_grad_(True)
    wb = w.to(torch.bfloat16).float().requires_grad_(True)
    y_ref = F.conv2d(xi, wb, bias, padding=1)                            # [B, 64, 4, 4]
    y = conv3x3(x.contiguous(), pack_conv(w, x.shape[2]), bias)          # [B, 16, 64]
    assert _rel(y, y_ref.permute(0, 2, 3, 1).reshape(B, 16, 64)) < 1e-2
    gy = torch.randn(B, 16, 64, generator=g).to(DEV).to(torch.bfloat16)
    y_ref.backward(gy.float().reshape(B, 4, 4, 64).permute(0, 3, 1, 2))
    dw = conv3x3_wgrad(gy, x.contiguous())[:, :ci]
    assert _rel(dw, wb.grad) < 2e-3
    if ci == 64:
        dx = conv3x3(gy, pack_conv_dgrad(w))
        assert _rel(dx, xi.grad.reshape(B, ci, 16).permute(0, 2, 1)) < 1e-2
    # deterministic: fixed-order reductions
    assert torch.equal(conv3x3_wgrad(gy, x.contiguous())[:, :ci], dw)


@pytest.mark.parametrize("B", [4099, 5, 1])
def test_q_head_matches_linear(B):
    """QHead (r48_q_head_forward / _backward) vs the path it replaces, nets.py's
    linear(h, w, b, bf16).float() through hipBLASLt: the same bf16 products summed in fp32 in another
    order, outputs and parameter gradients rounded to bf16 -- q and dh agree within 1 bf16 ulp of
    the largest value (<= 1e-2 relative), dw and db within 1e-2 relative. Ragged B (not a multiple
    of the 4-board unroll) included; the fixed-order reductions make the backward deterministic."""
    from rein48_amd.a3c.nets import linear
    from rein48_amd.dqn.conv import QHead
    g = torch.Generator(device="cpu").manual_seed(B)
    h = torch.randn(B, 1024, generator=g).to(DEV).to(torch.bfloat16)
    w = (torch.randn(4, 1024, generator=g) * 0.05).to(DEV).requires_grad_(True)
    b = torch.randn(4, generator=g).to(DEV).requires_grad_(True)
    dq = torch.randn(B, 4, generator=g).to(DEV)
    outs = []
    for fn in (lambda hh: QHead.apply(hh, w, b), lambda hh: linear(hh, w, b, torch.bfloat16).float()):
        hh = h.clone().requires_grad_(True)
        w.grad = b.grad = None
        q = fn(hh)
        q.backward(dq)
        outs.append((q.detach(), hh.grad.detach(), w.grad.detach().clone(), b.grad.detach().clone()))
    (q, dh, dw, db), (q_r, dh_r, dw_r, db_r) = outs
    assert q.dtype == torch.float32 and torch.equal(q, q.to(torch.bfloat16).float())
    assert _rel(q, q_r) < 1e-2 and _rel(dh, dh_r) < 1e-2
    assert _rel(dw, dw_r) < 1e-2 and _rel(db, db_r) < 1e-2
    hh = h.clone().requires_grad_(True)
    w.grad = b.grad = None
    QHead.apply(hh, w, b).backward(dq)
    assert torch.equal(hh.grad, dh) and torch.equal(w.grad, dw) and torch.equal(b.grad, db)


@pytest.mark.parametrize("ci,B", [(64, 4099), (18, 1037)])
def test_conv3x3_stats_match_fp64_sums(ci, B):
    """r48_conv3x3's fused BN statistics: the per-CU records summed equal the fp64 per-channel sum
    and sum of squares of the bf16 outputs it wrote (fp32 partials: 1e-5 relative), and the
    outputs equal the stats-free launch's bit for bit."""
    from rein48_amd import _lib
    from rein48_amd.dqn.conv import board_onehot32, conv3x3, pack_conv
    g = torch.Generator(device="cpu").manual_seed(ci + B)
    w = (torch.randn(64, ci, 3, 3, generator=g) * 0.1).to(DEV)
    bias = (torch.randn(64, generator=g) * 0.5 + 2.0).to(DEV)          # means well away from 0
    if ci == 18:
        x = board_onehot32(torch.randint(0, 18, (B, 16), generator=g, dtype=torch.int8).to(DEV))
    else:
        x = torch.randn(B, 16, ci, generator=g).to(DEV).to(torch.bfloat16)
    st = torch.empty(int(_lib.load().r48_conv_stats_floats()), dtype=torch.float32, device=DEV)
    y = conv3x3(x.contiguous(), pack_conv(w, x.shape[2]), bias, stats=st)
    assert torch.equal(y, conv3x3(x.contiguous(), pack_conv(w, x.shape[2]), bias))
    rec = st[:-4].view(-1, 2, 64).double().sum(0)   # (the last 4 floats: the arrival counter)
    yd = y.reshape(-1, 64).double()
    for got, want in ((rec[0], yd.sum(0)), (rec[1], (yd * yd).sum(0))):
        assert float((got - want).abs().max()) <= 1e-5 * float(want.abs().max())


@pytest.mark.parametrize("B,with_add", [(4099, False), (4099, True), (1037, True), (4099, "mask"), (1037, "mask")])
def test_conv3x3_bn_grad_reduction_matches_fp64(B, with_add):
    """r48_conv3x3_bn_grad (the data-gradient conv with the BN-backward reduction of the layer
    below in its epilogue): its output equals the plain r48_conv3x3 launch's bit for bit, and its
    per-CU records summed equal the fp64 per-channel sums of g = out . [mask bit] and of
    g (bn_x - mean) (fp32 partials: within 1e-5 of the sum of the terms' magnitudes). Ragged board
    counts, with and without the residual add; "mask": the add masked by a ReLU mask in the kernel
    (add_mask) equals the plain launch with the masked add written out (zeros where a bit is 0)."""
    import ctypes
    from rein48_amd import _lib
    from rein48_amd.dqn.conv import conv3x3, pack_conv_dgrad
    g = torch.Generator(device="cpu").manual_seed(B + (2 if with_add == "mask" else int(with_add)))
    frags = pack_conv_dgrad((torch.randn(64, 64, 3, 3, generator=g) * 0.1).to(DEV))
    dy = torch.randn(B, 16, 64, generator=g).to(DEV).to(torch.bfloat16)
    add = torch.randn(B, 16, 64, generator=g).to(DEV).to(torch.bfloat16) if with_add else None
    bn_x = (torch.randn(B, 16, 64, generator=g) + 3.0).to(DEV).to(torch.bfloat16)
    mask = torch.randint(0, 256, (B * 16, 8), generator=g, dtype=torch.uint8).to(DEV)
    save = torch.cat([torch.randn(64, generator=g) + 3.0, torch.rand(64, generator=g) + 0.5]).to(DEV)
    add_mask = torch.randint(0, 256, (B * 16, 8), generator=g, dtype=torch.uint8).to(DEV) if with_add == "mask" else None
    L = _lib.load()
    part = torch.full((int(L.r48_conv_stats_floats()),), float("nan"), dtype=torch.float32, device=DEV)
    out = torch.empty_like(dy)
    _lib.check(L.r48_conv3x3_bn_grad(_lib.ptr(dy), B, _lib.ptr(frags), _lib.ptr(add), _lib.ptr(add_mask), _lib.ptr(out),
                                     _lib.ptr(bn_x), _lib.ptr(mask), _lib.ptr(save), _lib.ptr(part), None,
                                     ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    if add_mask is not None:
        abits = ((add_mask.long().unsqueeze(-1) >> torch.arange(8, device=DEV)) & 1).reshape(B, 16, 64).bool()
        add = torch.where(abits, add, torch.zeros((), dtype=add.dtype, device=DEV))
    assert torch.equal(out, conv3x3(dy, frags, add=add))
    bits = ((mask.long().unsqueeze(-1) >> torch.arange(8, device=DEV)) & 1).reshape(B * 16, 64).bool()
    gd = torch.where(bits, out.reshape(-1, 64).double(), torch.zeros((), dtype=torch.float64, device=DEV))
    xd = bn_x.reshape(-1, 64).double() - save[:64].double()
    rec = part[:-4].view(-1, 2, 64).double().sum(0)
    for got, terms in ((rec[0], gd), (rec[1], gd * xd)):
        err = (got - terms.sum(0)).abs()
        assert bool((err <= 1e-5 * terms.abs().sum(0) + 1e-30).all()), float(err.max())



def _fin_args(L, gamma, beta, rm, rv, save, coef, dgamma, dbeta, rows, mom, eps):
    from rein48_amd import _lib
    p = lambda t: None if t is None else t.data_ptr()   # noqa: E731
    return _lib.BnFinishArgs(p(gamma), p(beta), p(rm), p(rv), p(save), p(coef), p(dgamma), p(dbeta), rows, mom, eps)


@pytest.mark.parametrize("B,cin", [(4099, 64), (1 << 16, 64), (1037, 32)])
def test_conv_stats_finish_equals_conv_then_bn_finish(B, cin):
    """r48_conv3x3_stats_finish (the BN finish in the workgroup whose statistics record arrives last,
    r48_bn_finish_args) against r48_conv3x3 with stats + the standalone r48_bn_finish: the same conv
    output bit for bit; save (mean, invstd), coef and the running statistics equal to fp32 rounding of
    the same fp64 sums taken in another order (rel 1e-6); twice in a row (the arrival counter is reset)
    with bit-identical results; then r48_bn_apply from that coef == r48_bn_forward_stats' output."""
    import ctypes
    from rein48_amd import _lib
    from rein48_amd.dqn.conv import pack_conv
    g = torch.Generator(device="cpu").manual_seed(B + cin)
    L = _lib.load()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    w = (torch.randn(64, cin, 3, 3, generator=g) * 0.1).to(DEV)
    frags, bias = pack_conv(w, cin), (torch.randn(64, generator=g) * 0.3).to(DEV)
    x = torch.randn(B, 16, cin, generator=g).to(DEV).to(torch.bfloat16)
    gamma, beta = (torch.rand(64, generator=g) + 0.5).to(DEV), (torch.randn(64, generator=g) * 0.2).to(DEV)
    rm0, rv0 = (torch.randn(64, generator=g) * 0.1).to(DEV), (torch.rand(64, generator=g) + 0.5).to(DEV)
    n = int(L.r48_conv_stats_floats())
    # reference: conv with statistics records, then the standalone finish
    st = torch.zeros(n, dtype=torch.float32, device=DEV)
    y_ref = torch.empty(B, 16, 64, dtype=torch.bfloat16, device=DEV)
    _lib.check(L.r48_conv3x3(_lib.ptr(x), B, cin, _lib.ptr(frags), _lib.ptr(bias), None, _lib.ptr(y_ref), _lib.ptr(st), s))
    save_r, coef_r = torch.empty(128, device=DEV), torch.empty(128, device=DEV)
    rm_r, rv_r = rm0.clone(), rv0.clone()
    _lib.check(L.r48_bn_finish(_lib.ptr(st), 256, B * 16, 64, _lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(rm_r),
                               _lib.ptr(rv_r), 0.1, 1e-5, _lib.ptr(save_r), _lib.ptr(coef_r), s))
    outs = []
    st2 = torch.zeros(n, dtype=torch.float32, device=DEV)
    for _ in range(2):
        y = torch.empty_like(y_ref)
        save, coef = torch.empty(128, device=DEV), torch.empty(128, device=DEV)
        rm, rv = rm0.clone(), rv0.clone()
        fin = _fin_args(L, gamma, beta, rm, rv, save, coef, None, None, B * 16, 0.1, 1e-5)
        _lib.check(L.r48_conv3x3_stats_finish(_lib.ptr(x), B, cin, _lib.ptr(frags), _lib.ptr(bias), _lib.ptr(y),
                                              _lib.ptr(st2), ctypes.byref(fin), s))
        torch.cuda.synchronize()
        assert int(st2[-4:].view(torch.int32)[0]) == 0          # the arrival counter is back to 0
        outs.append((y, save, coef, rm, rv))
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    y, save, coef, rm, rv = outs[0]
    assert torch.equal(y, y_ref)
    for got, want in ((save, save_r), (coef, coef_r), (rm, rm_r), (rv, rv_r)):
        torch.testing.assert_close(got, want, rtol=1e-6, atol=1e-7)
    z, m = torch.empty_like(y), torch.empty(B * 16, 8, dtype=torch.uint8, device=DEV)
    _lib.check(L.r48_bn_apply(_lib.ptr(y), None, B * 16, 64, _lib.ptr(coef_r), 1, _lib.ptr(z), _lib.ptr(m), s))
    z_r, m_r = torch.empty_like(y), torch.empty_like(m)
    ws = torch.empty(int(L.r48_bn_workspace_floats(B * 16, 64)), device=DEV)
    _lib.check(L.r48_bn_forward_stats(_lib.ptr(st), 256, _lib.ptr(y), None, B * 16, 64, _lib.ptr(gamma), _lib.ptr(beta),
                                      None, None, 0.1, 1e-5, 1, _lib.ptr(torch.empty(128, device=DEV)), _lib.ptr(ws),
                                      _lib.ptr(z_r), _lib.ptr(m_r), s))
    assert torch.equal(z, z_r) and torch.equal(m, m_r)


@pytest.mark.parametrize("B,with_add", [(4099, "mask"), (1 << 16, False)])
def test_conv_bn_grad_finish_equals_backward_part(B, with_add):
    """r48_conv3x3_bn_grad with fin (the BN backward's finish in its last workgroup) against the same
    conv without it + r48_bn_backward_part's finish: the same dx bit for bit; dgamma, dbeta and the
    apply coefficients equal to fp32 rounding (rel 1e-6, other fp64 order); r48_bn_backward_apply
    from the standalone finish's coefficients == r48_bn_backward_part's input gradient bit for bit."""
    import ctypes
    from rein48_amd import _lib
    from rein48_amd.dqn.conv import pack_conv_dgrad
    g = torch.Generator(device="cpu").manual_seed(B + 11)
    L = _lib.load()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    frags = pack_conv_dgrad((torch.randn(64, 64, 3, 3, generator=g) * 0.1).to(DEV))
    dy = torch.randn(B, 16, 64, generator=g).to(DEV).to(torch.bfloat16)
    add = torch.randn(B, 16, 64, generator=g).to(DEV).to(torch.bfloat16) if with_add else None
    add_mask = torch.randint(0, 256, (B * 16, 8), generator=g, dtype=torch.uint8).to(DEV) if with_add == "mask" else None
    bn_x = (torch.randn(B, 16, 64, generator=g) + 3.0).to(DEV).to(torch.bfloat16)
    mask = torch.randint(0, 256, (B * 16, 8), generator=g, dtype=torch.uint8).to(DEV)
    save = torch.cat([torch.randn(64, generator=g) + 3.0, torch.rand(64, generator=g) + 0.5]).to(DEV)
    gamma = (torch.rand(64, generator=g) + 0.5).to(DEV)
    n = int(L.r48_conv_stats_floats())
    part = torch.zeros(n, dtype=torch.float32, device=DEV)
    out_r = torch.empty_like(dy)
    _lib.check(L.r48_conv3x3_bn_grad(_lib.ptr(dy), B, _lib.ptr(frags), _lib.ptr(add), _lib.ptr(add_mask), _lib.ptr(out_r),
                                     _lib.ptr(bn_x), _lib.ptr(mask), _lib.ptr(save), _lib.ptr(part), None, s))
    dz = torch.randn(B, 16, 64, generator=g).to(DEV).to(torch.bfloat16)    # the gradient the apply consumes
    ws = torch.empty(int(L.r48_bn_workspace_floats(B * 16, 64)), device=DEV)
    dx_r, dg_r, db_r = torch.empty_like(dz), torch.empty(64, device=DEV), torch.empty(64, device=DEV)
    _lib.check(L.r48_bn_backward_part(_lib.ptr(part), 256, _lib.ptr(dz), _lib.ptr(mask), _lib.ptr(bn_x), B * 16, 64,
                                      _lib.ptr(gamma), _lib.ptr(save), _lib.ptr(ws), _lib.ptr(dx_r), None, _lib.ptr(dg_r),
                                      _lib.ptr(db_r), s))
    coef_r = ws[-192:].clone()                               # the finish's coefficients (workspace tail)
    part2 = torch.zeros(n, dtype=torch.float32, device=DEV)
    out = torch.empty_like(dy)
    coef, dg, db = torch.empty(192, device=DEV), torch.empty(64, device=DEV), torch.empty(64, device=DEV)
    fin = _fin_args(L, gamma, None, None, None, save, coef, dg, db, B * 16, 0.0, 0.0)
    _lib.check(L.r48_conv3x3_bn_grad(_lib.ptr(dy), B, _lib.ptr(frags), _lib.ptr(add), _lib.ptr(add_mask), _lib.ptr(out),
                                     _lib.ptr(bn_x), _lib.ptr(mask), _lib.ptr(save), _lib.ptr(part2), ctypes.byref(fin), s))
    torch.cuda.synchronize()
    assert torch.equal(out, out_r)
    assert int(part2[-4:].view(torch.int32)[0]) == 0
    torch.testing.assert_close(dg, dg_r, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(db, db_r, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(coef, coef_r, rtol=1e-6, atol=1e-9)
    dx = torch.empty_like(dz)
    _lib.check(L.r48_bn_backward_apply(_lib.ptr(dz), _lib.ptr(mask), _lib.ptr(bn_x), B * 16, 64, _lib.ptr(coef_r),
                                       _lib.ptr(dx), s))
    assert torch.equal(dx, dx_r)

# ---------------------------------------------------------------- steady-state sizes (the bench's)
# The tests above run the conv kernels at <= 1 tile per wave and the wgrad ring at <= 3 steps per
# workgroup. At the bench's 64K-board minibatch k_conv3x3 runs 2 tiles per wave (the cross-tile row
# prefetch and the tile += stride loop) and k_conv_wgrad 32 128-row steps per workgroup (the 3-buffer
# LDS-DMA ring wraps ~10 times). These run those sizes (and a ragged one) against fp64 references.
def _shift_cells(x, dr, dc):
    """x [B, 16, C] (cell = 4 r + c) -> x at cell (r + dr, c + dc), zero outside the grid."""
    B, _, C = x.shape
    g = x.view(B, 4, 4, C)
    out = torch.zeros_like(g)
    r0, r1 = max(0, -dr), min(4, 4 - dr)
    c0, c1 = max(0, -dc), min(4, 4 - dc)
    out[:, r0:r1, c0:c1] = g[:, r0 + dr:r1 + dr, c0 + dc:c1 + dc]
    return out.view(B, 16, C)


def _conv_fp64(x, w, bias=None):
    """3x3 conv, padding 1, on [B, 16, Cin] -> [B, 16, 64] in float64 (9 shifted matmuls)."""
    xd = x.double()
    B = xd.shape[0]
    y = torch.zeros(B * 16, w.shape[0], dtype=torch.float64, device=x.device)
    wd = w.double()
    for kr in range(3):
        for kc in range(3):
            xs = _shift_cells(xd, kr - 1, kc - 1).reshape(B * 16, -1)
            y += xs @ wd[:, :, kr, kc].t()
    if bias is not None:
        y += bias.double()
    return y.view(B, 16, -1)


def _wgrad_fp64(gy, x):
    """dW[o, c, kr, kc] = sum over boards and cells of gy[b, p, o] * x[b, p + (kr-1, kc-1), c]."""
    B, _, C = x.shape
    gd = gy.double().reshape(B * 16, -1)
    xd = x.double()
    dw = torch.zeros(gd.shape[1], C, 3, 3, dtype=torch.float64, device=x.device)
    for kr in range(3):
        for kc in range(3):
            dw[:, :, kr, kc] = gd.t() @ _shift_cells(xd, kr - 1, kc - 1).reshape(B * 16, C)
    return dw


@pytest.mark.parametrize("B", [1 << 16, (1 << 16) + 5])
def test_conv3x3_kernels_at_bench_size_match_fp64(B):
    """k_conv3x3 forward, forward + BN statistics, data gradient + residual add, and k_conv_wgrad at
    the bench's 64K-board minibatch (2 tiles per wave, 32 ring steps per workgroup) and a ragged
    64K + 5, vs float64 on the same bf16 inputs: forward / data gradient within 1e-2 of the largest
    value (bf16 output rounding), every element; the statistics within 1e-5 of the fp64 sums of the
    written outputs; the weight gradient (fp32 out, summed over 2^20 rows) within 1e-4 of its largest
    entry -- one lost or doubled 128-row ring step moves entries by ~1e-2 of that."""
    from rein48_amd import _lib
    from rein48_amd.dqn.conv import conv3x3, conv3x3_wgrad, pack_conv, pack_conv_dgrad
    g = torch.Generator(device="cpu").manual_seed(B)
    w = (torch.randn(64, 64, 3, 3, generator=g) * 0.1).to(DEV).to(torch.bfloat16).float()
    bias = (torch.randn(64, generator=g) * 0.5 + 1.0).to(DEV)
    x = torch.randn(B, 16, 64, generator=g).to(DEV).to(torch.bfloat16)
    y_ref = _conv_fp64(x, w, bias)
    st = torch.empty(int(_lib.load().r48_conv_stats_floats()), dtype=torch.float32, device=DEV)
    y = conv3x3(x, pack_conv(w, 64), bias, stats=st)
    assert _rel(y, y_ref) < 1e-2
    assert torch.equal(y, conv3x3(x, pack_conv(w, 64), bias))
    rec = st[:-4].view(-1, 2, 64).double().sum(0)   # (the last 4 floats: the arrival counter)
    yd = y.reshape(-1, 64).double()
    for got, want in ((rec[0], yd.sum(0)), (rec[1], (yd * yd).sum(0))):
        assert float((got - want).abs().max()) <= 1e-5 * float(want.abs().max())
    del y_ref, yd
    gy = torch.randn(B, 16, 64, generator=g).to(DEV).to(torch.bfloat16)
    add = torch.randn(B, 16, 64, generator=g).to(DEV).to(torch.bfloat16)
    # data gradient = conv with the flipped, transposed taps
    wt = w.flip(2, 3).transpose(0, 1).contiguous()
    dx_ref = _conv_fp64(gy, wt) + add.double()
    dx = conv3x3(gy, pack_conv_dgrad(w), add=add)
    assert _rel(dx, dx_ref) < 1e-2
    del dx_ref
    dw_ref = _wgrad_fp64(gy, x)
    dw = conv3x3_wgrad(gy, x)
    assert _rel(dw, dw_ref) < 1e-4, _rel(dw, dw_ref)
    assert torch.equal(conv3x3_wgrad(gy, x), dw)


@pytest.mark.parametrize("B,with_add", [(1 << 16, True), ((1 << 16) + 5, False)])
def test_conv3x3_bn_grad_at_bench_size_matches_fp64(B, with_add):
    """r48_conv3x3_bn_grad at the bench's minibatch (2 tiles per wave, the cross-tile prefetch):
    output == the plain data-gradient launch bit for bit, BN-backward records == the fp64 sums
    within 1e-5 of the summed magnitudes (as test_conv3x3_bn_grad_reduction_matches_fp64)."""
    import ctypes
    from rein48_amd import _lib
    from rein48_amd.dqn.conv import conv3x3, pack_conv_dgrad
    g = torch.Generator(device="cpu").manual_seed(B + 3 * with_add)
    frags = pack_conv_dgrad((torch.randn(64, 64, 3, 3, generator=g) * 0.1).to(DEV))
    dy = torch.randn(B, 16, 64, generator=g).to(DEV).to(torch.bfloat16)
    add = torch.randn(B, 16, 64, generator=g).to(DEV).to(torch.bfloat16) if with_add else None
    bn_x = (torch.randn(B, 16, 64, generator=g) + 3.0).to(DEV).to(torch.bfloat16)
    mask = torch.randint(0, 256, (B * 16, 8), generator=g, dtype=torch.uint8).to(DEV)
    save = torch.cat([torch.randn(64, generator=g) + 3.0, torch.rand(64, generator=g) + 0.5]).to(DEV)
    L = _lib.load()
    part = torch.full((int(L.r48_conv_stats_floats()),), float("nan"), dtype=torch.float32, device=DEV)
    out = torch.empty_like(dy)
    _lib.check(L.r48_conv3x3_bn_grad(_lib.ptr(dy), B, _lib.ptr(frags), _lib.ptr(add), None, _lib.ptr(out),
                                     _lib.ptr(bn_x), _lib.ptr(mask), _lib.ptr(save), _lib.ptr(part), None,
                                     ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    assert torch.equal(out, conv3x3(dy, frags, add=add))
    bits = ((mask.long().unsqueeze(-1) >> torch.arange(8, device=DEV)) & 1).reshape(B * 16, 64).bool()
    gd = torch.where(bits, out.reshape(-1, 64).double(), torch.zeros((), dtype=torch.float64, device=DEV))
    xd = bn_x.reshape(-1, 64).double() - save[:64].double()
    rec = part[:-4].view(-1, 2, 64).double().sum(0)
    for got, terms in ((rec[0], gd), (rec[1], gd * xd)):
        err = (got - terms.sum(0)).abs()
        assert bool((err <= 1e-5 * terms.abs().sum(0) + 1e-30).all()), float(err.max())


def test_onehot32_exact():
    from rein48_amd.dqn.conv import board_onehot32
    b = np.random.default_rng(5).integers(0, 18, size=(3001, 16)).astype(np.int8)
    got = board_onehot32(torch.from_numpy(b).to(DEV)).float().cpu().numpy()
    want = np.zeros((3001, 16, 32), np.float32)
    want[:, :, :18] = R.onehot(b).reshape(3001, 16, 18)
    np.testing.assert_array_equal(got, want)


def test_resnet_update_custom_conv_matches_structured_gemm():
    """One training forward/backward of the bf16 ResNet10Q through the hand-written convolutions
    (r48_conv3x3 / _wgrad) vs through the structured dense GEMMs (hipBLASLt): both are bf16
    computations of the same fp32 function, so the losses agree to bf16 precision and every
    weight gradient is close in relative norm."""
    from rein48_amd.dqn.kernels import board_onehot
    from rein48_amd.dqn.nets import ResNet10Q
    torch.manual_seed(10)
    net = ResNet10Q(dtype=torch.bfloat16).to(DEV).train()
    with torch.no_grad():
        net.head.weight.normal_(std=0.05)
    b = torch.from_numpy(np.random.default_rng(10).integers(0, 12, size=(8200, 16)).astype(np.int8)).to(DEV)
    x = board_onehot(b, dtype=torch.bfloat16)
    tgt = torch.randn(8200, 4, device=DEV)
    grads, losses = [], []
    for custom in (True, False):
        net.custom_conv = custom
        net.zero_grad()
        for m in net.bns:
            m.reset_running_stats()
        loss = torch.nn.functional.smooth_l1_loss(net(x), tgt)
        loss.backward()
        losses.append(float(loss.detach()))
        grads.append([p.grad.detach().float().clone() for k, p in net.named_parameters()
                      if not (k.endswith(".bias") and (k.startswith("stem") or k.startswith("convs")))])
    assert abs(losses[0] - losses[1]) <= 1e-2 * abs(losses[1])
    for ga, gb in zip(*grads):
        assert float((ga - gb).norm()) <= 5e-2 * float(gb.norm()) + 1e-6


@pytest.mark.parametrize("B", [4096, 1000, 1 << 16])      # 1 << 16: the bench's minibatch
def test_resnet_train_step_matches_autograd(B):
    """train_step.ResNetTrainStep (explicit forward/backward: BN statistics summed in the conv
    epilogues, BN ReLU masks, the block-input gradient summed in the data-gradient conv's epilogue,
    gradients straight into the flat buffer) vs loss.backward() through nets.py's custom-conv
    autograd path on the same bf16 net, both against the same net in fp32 (structured GEMMs + torch
    BN). The two bf16 computations differ in summation order and rounding only (unshifted conv-fused
    statistics vs k_bn_stats; the residual sum rounded once instead of twice; a bf16 flip moves a
    value by 2^-8 and flips propagate through 9 layers), so: loss and mean Q agree to 5e-4, running
    statistics to 1e-4 relative, and every gradient's relative error against fp32 is within 1.5x
    (+ 2e-3) of the autograd path's own bf16 error; test_conv3x3_stats_match_fp64_sums pins the sums."""
    from rein48_amd.a3c.optim import FlatParams
    from rein48_amd.dqn.conv import board_onehot32
    from rein48_amd.dqn.kernels import board_onehot
    from rein48_amd.dqn.nets import ResNet10Q
    from rein48_amd.dqn.train_step import ResNetTrainStep
    torch.manual_seed(B)
    net = ResNet10Q(dtype=torch.bfloat16).to(DEV).train()
    with torch.no_grad():
        net.head.weight.normal_(std=0.05)
    flat = FlatParams(net)
    rng = np.random.default_rng(B)
    boards = torch.from_numpy(rng.integers(0, 14, size=(B, 16)).astype(np.int8)).to(DEV)
    x = board_onehot32(boards).view(B, 512)
    action = torch.from_numpy(rng.integers(0, 4, size=B).astype(np.int8)).to(DEV)
    target = torch.from_numpy(rng.normal(size=B).astype(np.float32)).to(DEV)
    stats0 = [(m.running_mean.clone(), m.running_var.clone()) for m in net.bns]
    out = []
    for mode in ("autograd", "fused", "fp32"):
        for m, (rm, rv) in zip(net.bns, stats0):
            m.running_mean.copy_(rm)
            m.running_var.copy_(rv)
        flat.zero_grad()
        net.dtype = torch.float32 if mode == "fp32" else torch.bfloat16
        if mode == "fused":
            loss, q_mean = ResNetTrainStep(net)(x, action, target)
        else:
            xin = board_onehot(boards, dtype=torch.float32) if mode == "fp32" else x
            q = net(xin)
            q_sa = q.gather(1, action.long().view(-1, 1)).squeeze(1)
            loss = torch.nn.functional.smooth_l1_loss(q_sa, target)
            loss.backward()
            q_mean = q_sa.detach().mean()
        out.append((float(loss), float(q_mean), [p.grad.detach().clone() for p in flat.params],
                    [(m.running_mean.clone(), m.running_var.clone()) for m in net.bns]))
    net.dtype = torch.bfloat16
    (la, qa, ga, sa), (lb, qb, gb, sb), (_, _, g32, _) = out
    assert abs(la - lb) <= 5e-4 * abs(la) and abs(qa - qb) <= 5e-4 * abs(qa) + 1e-6
    for (ra, va), (rb, vb) in zip(sa, sb):
        assert float((ra - rb).abs().max()) <= 1e-4 * float(ra.abs().max()) + 1e-6
        assert float((va - vb).abs().max()) <= 1e-4 * float(va.abs().max()) + 1e-6
    names = [n for n, p in net.named_parameters() if p.requires_grad]
    for n, a, b, r in zip(names, ga, gb, g32):
        if float(r.norm()) == 0.0:                  # conv biases: zero gradient on every path
            assert float(a.norm()) == 0.0 and float(b.norm()) == 0.0, n
            continue
        ea = float((a - r).norm()) / float(r.norm())
        eb = float((b - r).norm()) / float(r.norm())
        assert eb <= 1.5 * ea + 2e-3, (n, ea, eb)


def test_fused_train_step_writes_every_gradient_but_the_conv_biases():
    """DQNLearner.learn zeroes the flat gradient only before the first of consecutive fused steps:
    the step must WRITE (not accumulate into) every parameter gradient except the conv biases', which
    stay exactly zero. Flat gradient filled with NaN, conv-bias slots zeroed, one fused step: no NaN
    left, biases still zero; a second step without zeroing gives the same gradient bit for bit."""
    from rein48_amd.a3c.optim import FlatParams
    from rein48_amd.dqn.conv import board_onehot32
    from rein48_amd.dqn.nets import ResNet10Q
    from rein48_amd.dqn.train_step import ResNetTrainStep
    torch.manual_seed(5)
    B = 4099
    net = ResNet10Q(dtype=torch.bfloat16).to(DEV).train()
    flat = FlatParams(net)
    rng = np.random.default_rng(5)
    x = board_onehot32(torch.from_numpy(rng.integers(0, 14, size=(B, 16)).astype(np.int8)).to(DEV)).view(B, 512)
    action = torch.from_numpy(rng.integers(0, 4, size=B).astype(np.int8)).to(DEV)
    target = torch.from_numpy(rng.normal(size=B).astype(np.float32)).to(DEV)
    biases = [c.bias for c in net.conv_layers()]
    flat.grad.fill_(float("nan"))
    for bb in biases:
        bb.grad.zero_()
    step = ResNetTrainStep(net)
    stats0 = [(m.running_mean.clone(), m.running_var.clone()) for m in net.bns]
    step(x, action, target)
    g1 = flat.grad.clone()
    assert not bool(torch.isnan(g1).any())
    assert all(float(bb.grad.abs().max()) == 0.0 for bb in biases)
    for m, (rm, rv) in zip(net.bns, stats0):
        m.running_mean.copy_(rm)
        m.running_var.copy_(rv)
    step(x, action, target)
    assert torch.equal(flat.grad, g1)


def test_conv_pack_resnet_matches_host_packing():
    """r48_conv_pack_resnet (all 17 fragment sets of the update in one launch) is bit-identical to
    pack_conv / pack_conv_dgrad per layer."""
    from rein48_amd.dqn.conv import pack_conv, pack_conv_dgrad, pack_resnet_train
    from rein48_amd.dqn.nets import ResNet10Q
    torch.manual_seed(3)
    net = ResNet10Q(dtype=torch.bfloat16).to(DEV)
    convs = net.conv_layers()
    fwd, dg = pack_resnet_train(convs)
    for i, c in enumerate(convs):
        assert torch.equal(fwd[i].view(-1), pack_conv(c.weight, 32 if i == 0 else 64).view(-1)), i
        if i:
            assert torch.equal(dg[i].view(-1), pack_conv_dgrad(c.weight).view(-1)), i


def test_fused_adam_matches_torch_adam():
    """r48_adam (trainer.Adam on a GPU fp32 flat buffer: one launch) vs torch.optim.Adam over the same
    parameters and gradients for 6 steps: the same fp32 update formula, fused (contractions may round
    differently), so parameters agree to 1e-6 relative; the first step's update is exactly lr in
    size where the gradient is nonzero."""
    from rein48_amd.a3c.optim import FlatParams
    from rein48_amd.dqn.trainer import Adam
    torch.manual_seed(7)
    a = torch.nn.Linear(64, 36).to(DEV)                 # 64*36 + 36 = 2340 floats: a multiple of 4
    b = torch.nn.Linear(64, 36).to(DEV)
    b.load_state_dict(a.state_dict())
    flat = FlatParams(a)
    assert flat.data.numel() % 4 == 0
    mine = Adam(flat, lr=1e-3)
    ref = torch.optim.Adam(b.parameters(), lr=1e-3)
    for _ in range(6):
        x = torch.randn(32, 64, device=DEV)
        flat.zero_grad()
        a(x).square().sum().backward()
        mine.step()
        ref.zero_grad()
        b(x).square().sum().backward()
        ref.step()
    torch.testing.assert_close(a.weight, b.weight, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(a.bias, b.bias, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("B", [4099, 1 << 16])
def test_resnet_train_step_bn_fold_is_bit_identical(B):
    """ResNetTrainStep with every BN apply but the last folded into the next conv's operand load
    (r48_conv3x3_bn_in + r48_bn_finish) == the step with separate apply passes, bit for bit: the
    folded load forms relu(a x + b (+ identity)) with k_bn_apply's arithmetic and rounding, so every
    activation, ReLU mask, loss, gradient and running statistic is identical (ragged and bench-size
    minibatches)."""
    from rein48_amd.a3c.optim import FlatParams
    from rein48_amd.dqn.conv import board_onehot32
    from rein48_amd.dqn.nets import ResNet10Q
    from rein48_amd.dqn.train_step import ResNetTrainStep
    torch.manual_seed(B)
    net = ResNet10Q(dtype=torch.bfloat16).to(DEV).train()
    with torch.no_grad():
        net.head.weight.normal_(std=0.05)
        for m in net.bns:                                    # non-trivial affine parameters
            m.weight.uniform_(0.5, 1.5)
            m.bias.uniform_(-0.5, 0.5)
    flat = FlatParams(net)
    rng = np.random.default_rng(B + 1)
    boards = torch.from_numpy(rng.integers(0, 14, size=(B, 16)).astype(np.int8)).to(DEV)
    x = board_onehot32(boards).view(B, 512)
    action = torch.from_numpy(rng.integers(0, 4, size=B).astype(np.int8)).to(DEV)
    target = torch.from_numpy(rng.normal(size=B).astype(np.float32)).to(DEV)
    stats0 = [(m.running_mean.clone(), m.running_var.clone()) for m in net.bns]
    out = []
    for fold in (True, False):
        for m, (rm, rv) in zip(net.bns, stats0):
            m.running_mean.copy_(rm)
            m.running_var.copy_(rv)
        flat.zero_grad()
        step = ResNetTrainStep(net, fold_bn=fold)
        loss, q_mean = step(x, action, target)
        buf = next(iter(step._bufs.values()))
        out.append((loss.clone(), q_mean.clone(), flat.grad.clone(),
                    [torch.cat([m.running_mean, m.running_var]) for m in net.bns],
                    [z.clone() for z in buf["z"]], [m.clone() for m in buf["m"]]))
    (la, qa, ga, sa, za, ma), (lb, qb, gb, sb, zb, mb) = out
    assert torch.equal(la, lb) and torch.equal(qa, qb)
    for k, (u, v) in enumerate(zip(za, zb)):
        assert torch.equal(u, v), ("z", k)
    for k, (u, v) in enumerate(zip(ma, mb)):
        assert torch.equal(u, v), ("mask", k)
    for k, (u, v) in enumerate(zip(sa, sb)):
        assert torch.equal(u, v), ("running stats", k)
    assert torch.equal(ga, gb)


def test_dqn_trainer_at_the_config5_per_gpu_slice():
    """DQNTrainer at the bench's per-GPU slice of BASELINE config 5 (16M boards over 8 GPUs): 2^21
    boards acting, a 2^25-slot HBM ring, 64K-board minibatches, for three train steps.
      - acting: one fused launch over all 2^21 boards (the trainer's act) equals 2^18-board chunks
        keyed by their global board ids (Q bit-identical, epsilon-greedy actions identical);
      - the ring: sampled transitions are consistent with the oracle move (a not-done row's
        next_state is the moved state plus at most one spawned 2/4 in an empty cell; a done row's
        next_state is a reset board: exactly one tile, 2 or 4), actions in 0..3;
      - the updates' losses and the flat parameters stay finite."""
    from rein48_amd.dqn import DQNConfig, DQNTrainer
    from rein48_amd.dqn.fused import resnet_q_forward
    n, cap, B = 1 << 21, 1 << 25, 1 << 16
    tr = DQNTrainer(DQNConfig(n_boards=n, replay_capacity=cap, batch=B, learn_start=B, seed=7), device=DEV)
    assert tr.use_fused
    losses = [tr.train_step()["loss"] for _ in range(3)]
    assert len(tr.replay) == 3 * n and all(np.isfinite(losses)), losses
    assert bool(torch.isfinite(tr.flat.data).all())
    # acting: one launch == 2^18-board chunks (same Philox keys: global board id, step counter)
    blob = tr.packed(tr.net)
    eps, ctr = 0.3, 11
    q1, a1 = resnet_q_forward(tr.env.boards, blob, q=True, actions=True, eps=eps, seed=5, ctr=ctr, gid0=0)
    for s in range(0, n, 1 << 18):
        qc, ac = resnet_q_forward(tr.env.boards[s:s + (1 << 18)].contiguous(), blob, q=True, actions=True, eps=eps,
                                  seed=5, ctr=ctr, gid0=s)
        assert torch.equal(qc, q1[s:s + (1 << 18)]) and torch.equal(ac, a1[s:s + (1 << 18)]), s
    # the ring's rows: oracle move of (state, action) vs next_state
    out = tr.replay.sample(1 << 16)
    st, a, s2, d = (out[k][:6000].cpu().numpy() for k in ("state", "action", "next_state", "done"))
    assert ((a >= 0) & (a < 4)).all()
    for i in range(st.shape[0]):
        if d[i]:
            nz = s2[i][s2[i] != 0]
            assert nz.size == 1 and nz[0] in (1, 2), (i, s2[i])
            continue
        moved = O.move(st[i], int(a[i]))[0]
        diff = moved != s2[i]
        assert diff.sum() <= 1, i
        if diff.any():
            assert moved[diff][0] == 0 and s2[i][diff][0] in (1, 2), i
