"""Config-5 value-based pieces on the CPU (no GPU): the structured-GEMM ResNet-10 vs
F.conv2d and vs the float64 oracle (oracle/dqn_ref.py; parity UNPINNED against the reference,
which has no DQN/ResNet code), BN folding, the flat Adam vs torch.optim.Adam, and the oracle's
TD target / Huber against torch's definitions."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import dqn_ref as R


def _params(net):
    return {"convs": [(c.weight.detach().numpy(), c.bias.detach().numpy()) for c in net.conv_layers()],
            "bns": [dict(mean=m.running_mean.numpy(), var=m.running_var.numpy(), gamma=m.weight.detach().numpy(),
                         beta=m.bias.detach().numpy()) for m in net.bns] if net.use_bn else None,
            "head": (net.head.weight.detach().numpy(), net.head.bias.detach().numpy())}


def _net(bn=True, channels=8, blocks=2):
    from rein48_amd.dqn.nets import ResNet10Q
    torch.manual_seed(0)
    net = ResNet10Q(channels=channels, blocks=blocks, bn=bn, dtype=torch.float64).double()
    if bn:
        for m in net.bns:
            m.running_mean.uniform_(-0.3, 0.3)
            m.running_var.uniform_(0.5, 1.5)
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
    return net


@pytest.mark.parametrize("ci,co", [(18, 8), (8, 8)])
def test_structured_conv_equals_conv2d(ci, co):
    from rein48_amd.dqn.nets import dense_conv_weight
    torch.manual_seed(1)
    conv = torch.nn.Conv2d(ci, co, 3, padding=1).double()
    x = torch.randn(7, ci, 4, 4, dtype=torch.float64, requires_grad=True)
    ref = conv(x)                                                   # [7, co, 4, 4]
    xp = x.permute(0, 2, 3, 1).reshape(7, 16 * ci)                  # position-major, channel-minor
    got = F.linear(xp, dense_conv_weight(conv), conv.bias.repeat(16)).view(7, 4, 4, co).permute(0, 3, 1, 2)
    torch.testing.assert_close(got, ref, rtol=1e-12, atol=1e-12)
    g = torch.randn_like(ref)
    gw_ref, gx_ref = torch.autograd.grad(ref, (conv.weight, x), g)
    gw, gx = torch.autograd.grad(got, (conv.weight, x), g)
    torch.testing.assert_close(gw, gw_ref, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(gx, gx_ref, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("bn", [False, True])
def test_resnet10_matches_oracle(bn):
    net = _net(bn).eval()
    b = np.random.default_rng(0).integers(0, 18, size=(64, 16))
    q = net(torch.from_numpy(R.onehot(b).reshape(64, -1))).detach().numpy()
    np.testing.assert_allclose(q, R.resnet10_q(_params(net), b), rtol=1e-6, atol=1e-8)   # Q is returned in fp32


def test_full_size_net_shape_and_param_count():
    from rein48_amd.dqn.nets import ResNet10Q
    net = ResNet10Q()
    n_w = sum(m.weight.numel() for m in net.conv_layers()) + net.head.weight.numel()
    assert len(net.conv_layers()) + 1 == 10                                  # 10 weight layers
    assert n_w == 18 * 64 * 9 + 8 * 64 * 64 * 9 + 16 * 64 * 4
    assert net(torch.zeros(3, 16 * 18)).shape == (3, 4)


def test_bn_folding_matches_eval_forward():
    from rein48_amd.dqn.nets import ResNet10Q
    net = _net(True).eval()
    convs, head = net.folded()
    plain = ResNet10Q(channels=8, blocks=2, bn=False, dtype=torch.float64).double().eval()
    with torch.no_grad():
        for c, (w, b) in zip(plain.conv_layers(), convs):
            c.weight.copy_(w)
            c.bias.copy_(b)
        plain.head.weight.copy_(head[0])
        plain.head.bias.copy_(head[1])
    x = torch.from_numpy(R.onehot(np.random.default_rng(2).integers(0, 18, size=(40, 16))).reshape(40, -1))
    torch.testing.assert_close(plain(x), net(x), rtol=1e-5, atol=1e-6)     # folded weights are fp32


def test_flat_adam_matches_torch_adam():
    from rein48_amd.a3c.optim import FlatParams
    from rein48_amd.dqn.trainer import Adam
    torch.manual_seed(3)
    a = torch.nn.Linear(5, 3).double()
    b = torch.nn.Linear(5, 3).double()
    b.load_state_dict(a.state_dict())
    flat = FlatParams(a)
    mine = Adam(flat, lr=1e-2)
    ref = torch.optim.Adam(b.parameters(), lr=1e-2)
    for _ in range(5):
        x = torch.randn(8, 5, dtype=torch.float64)
        flat.zero_grad()
        a(x).square().sum().backward()
        mine.step()
        ref.zero_grad()
        b(x).square().sum().backward()
        ref.step()
    torch.testing.assert_close(a.weight, b.weight, rtol=1e-10, atol=1e-12)


def test_oracle_td_target_and_huber():
    rng = np.random.default_rng(4)
    qt, qo = rng.normal(size=(100, 4)), rng.normal(size=(100, 4))
    r, d = rng.normal(size=100), (rng.random(100) < 0.3)
    y = R.td_target(r, d, qt, None, 0.9)
    np.testing.assert_allclose(y, r + 0.9 * (1 - d) * qt.max(1))
    y2 = R.td_target(r, d, qt, qo, 0.9)
    np.testing.assert_allclose(y2, r + 0.9 * (1 - d) * qt[np.arange(100), qo.argmax(1)])
    x = rng.normal(size=100) * 3
    assert abs(R.huber(x, y) - float(F.smooth_l1_loss(torch.tensor(x), torch.tensor(y)))) < 1e-12


def test_fused_kernel_packing_layout_cpu():
    """pack_resnet (host packing of the fused inference kernel's blob, csrc/r48_resnet.hip) against
    an element-wise restatement of the 16x16x32 fragment layout: lane l = 16g + r, element j;
    stem (t, o): W0[16o + r][8g + j][t] (planes >= 18 zero); conv (t, o, c):
    W[16o + r][16(2c + (j >> 2)) + 4g + (j & 3)][t]; head (p, c): Wh[r][64p + same channel]
    (rows >= 4 zero); each block closed by its f32 bias fragment. Runs on the CPU."""
    from rein48_amd.dqn.fused import pack_resnet
    from rein48_amd.dqn.nets import ResNet10Q
    torch.manual_seed(3)
    net = ResNet10Q().eval()
    with torch.no_grad():
        for m in net.bns:
            m.running_mean.uniform_(-0.3, 0.3)
            m.running_var.uniform_(0.5, 2.0)
    convs, (hw, hb) = net.folded()
    blob = pack_resnet(net).view(torch.int16).numpy().reshape(-1, 64, 8)
    bf = lambda v: torch.tensor(float(v), dtype=torch.float32).to(torch.bfloat16).view(torch.int16).item()
    rng = np.random.default_rng(0)
    W0 = convs[0][0].detach().numpy()
    for _ in range(200):
        t, o, l, j = rng.integers(9), rng.integers(4), rng.integers(64), rng.integers(8)
        r, g = l & 15, l >> 4
        want = W0[16 * o + r, 8 * g + j, t // 3, t % 3] if 8 * g + j < 18 else 0.0
        assert blob[t * 4 + o, l, j] == bf(want)
    for L in (1, 5, 8):
        W = convs[L][0].detach().numpy()
        base = 37 + (L - 1) * 73
        for _ in range(200):
            t, o, c, l, j = rng.integers(9), rng.integers(4), rng.integers(2), rng.integers(64), rng.integers(8)
            r, g = l & 15, l >> 4
            ci = 16 * (2 * c + (j >> 2)) + 4 * g + (j & 3)
            assert blob[base + (t * 4 + o) * 2 + c, l, j] == bf(W[16 * o + r, ci, t // 3, t % 3])
        bias = pack_resnet(net).view(-1, 512)[base + 72].view(torch.float32)[:64]
        torch.testing.assert_close(bias, convs[L][1].detach(), rtol=0, atol=0)
    head = 37 + 8 * 73
    H = hw.detach().numpy()
    for _ in range(200):
        p, c, l, j = rng.integers(16), rng.integers(2), rng.integers(64), rng.integers(8)
        r, g = l & 15, l >> 4
        ci = 16 * (2 * c + (j >> 2)) + 4 * g + (j & 3)
        want = H[r, 64 * p + ci] if r < 4 else 0.0
        assert blob[head + 2 * p + c, l, j] == bf(want)
    torch.testing.assert_close(pack_resnet(net).view(-1, 512)[head + 32].view(torch.float32)[:4], hb.detach(), rtol=0, atol=0)


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dqn_learner_worker(rank, world, port, q):
    """One rank of the DQN learner (rein48_amd/dqn/trainer.py:DQNLearner) on the CPU over gloo."""
    import copy
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rein48_amd.dqn import DQNConfig, DQNLearner
        cfg = DQNConfig(channels=8, blocks=2, bf16=False, seed=100 + rank, target_sync=2, lr=1e-3)
        lr = DQNLearner(cfg, device="cpu")             # different seeds: the broadcast makes them equal
        init = lr.flat.data.numpy().copy()
        g = torch.Generator().manual_seed(7 + rank)     # each rank its own minibatch
        B = 32
        x = F.one_hot(torch.randint(0, 18, (B, 16), generator=g), 18).float().view(B, 16 * 18)
        a = torch.randint(0, 4, (B,), generator=g, dtype=torch.int8)
        y = torch.randn(B, generator=g)
        out1 = lr.learn(x, a, y)
        out2 = lr.learn(x, a, y)                        # second update: target sync (target_sync = 2)
        folded, head = lr.net.eval().folded()
        fold = np.concatenate([t.detach().numpy().ravel() for wb in folded for t in wb] + [t.detach().numpy().ravel() for t in head])
        tgt = torch.cat([p.detach().view(-1) for p in lr.target.parameters()]).numpy().copy()
        q.put((rank, init, None, None, lr.flat.grad.numpy().copy(), lr.flat.data.numpy().copy(),
               lr.bn_buffers.data.numpy().copy(), fold, tgt, out1["loss"], out2["loss"], lr.updates))
    finally:
        dist.destroy_process_group()


def test_two_rank_dqn_learner_gloo():
    """DQN's multi-rank sequence on two gloo ranks: rank 0's initial weights broadcast, ONE
    all-reduce of the flat gradient (= the mean of the ranks' local gradients), an identical Adam
    step, the BN running statistics averaged over the ranks, so the BN-folded eval weights (the
    fused acting kernel's input) and the target net are identical on every rank."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dqn_learner_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=90) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    r0, r1 = res
    np.testing.assert_array_equal(r0[1], r1[1])                           # broadcast initial weights
    np.testing.assert_array_equal(r0[5], r1[5])                           # parameters after 2 updates
    np.testing.assert_array_equal(r0[4], r1[4])                           # last averaged gradient
    np.testing.assert_array_equal(r0[6], r1[6])                           # BN running statistics
    np.testing.assert_array_equal(r0[7], r1[7])                           # folded eval weights
    np.testing.assert_array_equal(r0[8], r1[8])                           # target net (synced at update 2)
    np.testing.assert_array_equal(r0[8], r0[5])                           # target == online after the sync
    assert r0[11] == r1[11] == 2
    assert np.isfinite(r0[9]) and np.isfinite(r1[10])


def _dqn_first_update_worker(rank, world, port, q):
    import copy
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rein48_amd.dqn import DQNConfig, DQNLearner
        cfg = DQNConfig(channels=8, blocks=2, bf16=False, seed=100 + rank, lr=1e-3)
        lr = DQNLearner(cfg, device="cpu")
        g = torch.Generator().manual_seed(7 + rank)
        B = 32
        x = F.one_hot(torch.randint(0, 18, (B, 16), generator=g), 18).float().view(B, 16 * 18)
        a = torch.randint(0, 4, (B,), generator=g, dtype=torch.int8)
        y = torch.randn(B, generator=g)
        # what this rank alone would compute: local gradient (the conv biases feeding a BN get none,
        # like the flat buffer's zeros) and local BN running statistics
        twin = copy.deepcopy(lr.net).train()
        for p in twin.parameters():
            p.grad = None
        qs = twin(x).gather(1, a.long().view(-1, 1)).squeeze(1)
        F.smooth_l1_loss(qs, y).backward()
        local_g = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).view(-1)
                             for p in twin.parameters() if p.requires_grad]).numpy().copy()
        local_bn = torch.cat([b.view(-1) for b in twin.buffers() if b.is_floating_point()]).numpy().copy()
        lr.learn(x, a, y)
        q.put((rank, local_g, local_bn, lr.flat.grad.numpy().copy(), lr.bn_buffers.data.numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_two_rank_dqn_first_update_averages_gradient_and_bn_stats():
    """After one update on two gloo ranks: flat gradient == mean of the ranks' local gradients, BN
    running statistics == mean of what each rank's own forward would have left."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dqn_first_update_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=90) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, g0, b0, G0, B0), (_, g1, b1, G1, B1) = res
    np.testing.assert_allclose(G0, (g0 + g1) / 2, rtol=1e-5, atol=1e-7)
    np.testing.assert_array_equal(G0, G1)
    np.testing.assert_allclose(B0, (b0 + b1) / 2, rtol=1e-6, atol=1e-7)
    np.testing.assert_array_equal(B0, B1)
    assert not np.allclose(b0, b1)          # the ranks' own statistics did differ
