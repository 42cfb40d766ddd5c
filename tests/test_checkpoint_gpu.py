"""Checkpoint / resume of the GPU trainers (rein48_amd/checkpoint.py): a trainer restored from a
checkpoint continues bit-identically to one that never stopped -- same parameters, optimizer slots,
env boards and counters (hence the same Philox draws), and for DQN the same replay ring contents."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _a3c(net, bf16):
    from rein48_amd.a3c import A3CConfig, A3CTrainer
    cfg = A3CConfig(n_boards=4099, max_steps=20, mode="textbook", net=net, bf16=bf16, features="exponents", seed=9)
    return A3CTrainer(cfg, device=DEV)


@pytest.mark.parametrize("net,bf16", [("cnn", True), ("mlp", False)])
def test_a3c_resume_is_bit_identical(tmp_path, net, bf16):
    from rein48_amd import checkpoint
    a = _a3c(net, bf16)
    a.train_step()
    a.train_step()
    path = tmp_path / "a3c.pt"
    checkpoint.save(a, path)
    la = [a.train_step() for _ in range(2)]
    b = _a3c(net, bf16)
    b.train_step()                        # diverge first
    checkpoint.load(b, path)
    lb = [b.train_step() for _ in range(2)]
    torch.cuda.synchronize()
    assert la == lb
    assert torch.equal(a.flat.data, b.flat.data) and torch.equal(a.opt.ms, b.opt.ms)
    assert torch.equal(a.env.boards, b.env.boards) and a.env.counters == b.env.counters
    assert a.sample_ctr == b.sample_ctr and a.updates == b.updates == 4


def test_dqn_trainer_resume_is_bit_identical(tmp_path):
    from rein48_amd import checkpoint
    from rein48_amd.dqn import DQNConfig, DQNTrainer

    def make():
        return DQNTrainer(DQNConfig(n_boards=2048, replay_capacity=10_000, batch=1024, learn_start=4096,
                                    target_sync=3, seed=4), device=DEV)

    a = make()
    for _ in range(4):                    # 8192 transitions, two updates
        a.train_step()
    path = tmp_path / "dqn.pt"
    checkpoint.save(a, path)
    la = [a.train_step()["loss"] for _ in range(4)]   # the ring wraps (10,000 slots)
    b = make()
    b.train_step()
    checkpoint.load(b, path)
    assert len(b.replay) == 8192
    lb = [b.train_step()["loss"] for _ in range(4)]
    torch.cuda.synchronize()
    assert la == lb
    assert torch.equal(a.flat.data, b.flat.data) and torch.equal(a.bn_buffers.data, b.bn_buffers.data)
    assert torch.equal(a.env.boards, b.env.boards) and a.replay.counters == b.replay.counters
    idx = torch.arange(len(a.replay), device=DEV)
    ra, rb = a.replay.gather(idx), b.replay.gather(idx)
    for k in ("state", "action", "reward", "next_state", "done"):
        assert torch.equal(ra[k], rb[k]), k


def test_a3c_load_rejects_mismatched_draws_inputs_or_shard(tmp_path):
    """a checkpoint only loads where the resume is bit-identical -- another seed (other
    Philox draws), features (other network inputs), bf16, loss mode, rank shard or draw contract raise."""
    import dataclasses
    from rein48_amd import checkpoint
    from rein48_amd.a3c import A3CConfig, A3CTrainer
    base = A3CConfig(n_boards=512, max_steps=8, mode="textbook", net="cnn", bf16=True, features="exponents", seed=9)
    a = A3CTrainer(base, device=DEV)
    path = tmp_path / "a3c.pt"
    checkpoint.save(a, path)
    for change in (dict(seed=10), dict(features="values"), dict(mode="reference"), dict(bf16=False)):
        other = A3CTrainer(dataclasses.replace(base, **change), device=DEV)
        with pytest.raises(ValueError):
            checkpoint.load(other, path)
    b = A3CTrainer(base, device=DEV)
    b.gid0 = 512                              # what rank 1 of a 2-rank job would hold
    with pytest.raises(ValueError, match="shard"):
        checkpoint.load(b, path)
    st = torch.load(path, weights_only=True)
    st["draw_contract"] = 2
    torch.save(st, tmp_path / "old.pt")
    with pytest.raises(ValueError, match="draw contract"):
        checkpoint.load(A3CTrainer(base, device=DEV), tmp_path / "old.pt")
    checkpoint.load(A3CTrainer(base, device=DEV), path)   # the matching trainer loads


def test_dqn_resume_without_replay_contents_starts_an_empty_ring(tmp_path):
    """save(replay=False): the resumed ring is empty (size 0, head 0) with the sampling counter kept,
    so no zero / stale rows are sampled as transitions."""
    from rein48_amd import checkpoint
    from rein48_amd.dqn import DQNConfig, DQNTrainer

    def make():
        return DQNTrainer(DQNConfig(n_boards=1024, replay_capacity=8_000, batch=512, learn_start=2048, seed=4),
                          device=DEV)

    a = make()
    for _ in range(3):
        a.train_step()
    checkpoint.save(a, tmp_path / "dqn.pt", replay=False)
    b = make()
    for _ in range(2):
        b.train_step()                        # b's ring holds its own transitions
    checkpoint.load(b, tmp_path / "dqn.pt")
    size, head, ctr = b.replay.counters
    assert (size, head) == (0, 0) and ctr == a.replay.counters[2]
    b.train_step()                            # refills: below learn_start, no update
    assert len(b.replay) == 1024
