"""Checkpoint / resume (rein48_amd/checkpoint.py) of the device-agnostic DQN learner on the CPU:
updates after a save + load are bit-identical to updates that never stopped."""
import pytest
import torch


def _batches(k, B=64, seed=0):
    import torch.nn.functional as F
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(k):
        x = F.one_hot(torch.randint(0, 18, (B, 16), generator=g), 18).float().view(B, 16 * 18)
        out.append((x, torch.randint(0, 4, (B,), generator=g, dtype=torch.int8), torch.randn(B, generator=g)))
    return out


def _learner():
    from rein48_amd.dqn import DQNConfig, DQNLearner
    return DQNLearner(DQNConfig(channels=8, blocks=2, bf16=False, seed=3, target_sync=3, lr=1e-3), device="cpu")


def test_dqn_learner_resume_is_bit_identical(tmp_path):
    from rein48_amd import checkpoint
    data = _batches(6)
    a = _learner()
    for x, act, y in data[:3]:
        a.learn(x, act, y)
    path = tmp_path / "dqn.pt"
    checkpoint.save(a, path)
    for x, act, y in data[3:]:
        a.learn(x, act, y)
    b = _learner()
    b.learn(*data[5])                     # diverge first: the load must overwrite everything
    checkpoint.load(b, path)
    assert b.updates == 3 and b.opt.t == 3
    for x, act, y in data[3:]:
        b.learn(x, act, y)
    for (ka, va), (kb, vb) in zip(a.net.state_dict().items(), b.net.state_dict().items()):
        assert ka == kb and torch.equal(va, vb), ka
    for (ka, va), (kb, vb) in zip(a.target.state_dict().items(), b.target.state_dict().items()):
        assert torch.equal(va, vb), ka
    assert torch.equal(a.opt.m, b.opt.m) and torch.equal(a.opt.v, b.opt.v) and a.updates == b.updates


def test_checkpoint_rejects_a_mismatched_trainer(tmp_path):
    from rein48_amd import checkpoint
    from rein48_amd.dqn import DQNConfig, DQNLearner
    a = _learner()
    path = tmp_path / "dqn.pt"
    checkpoint.save(a, path)
    other = DQNLearner(DQNConfig(channels=16, blocks=2, bf16=False, seed=3), device="cpu")
    with pytest.raises(ValueError):
        checkpoint.load(other, path)
    with pytest.raises(TypeError):
        checkpoint.save(object(), path)


def test_checkpoint_rejects_another_seed_rank_or_contract(tmp_path):
    """seed, rank shard and draw contract must match (a resume under other draws is not
    bit-identical); hyper-parameters such as lr may differ."""
    from rein48_amd import checkpoint
    from rein48_amd.dqn import DQNConfig, DQNLearner
    a = _learner()
    path = tmp_path / "dqn.pt"
    checkpoint.save(a, path)
    with pytest.raises(ValueError, match="seed"):
        checkpoint.load(DQNLearner(DQNConfig(channels=8, blocks=2, bf16=False, seed=4), device="cpu"), path)
    b = _learner()
    b.rank = 1
    with pytest.raises(ValueError, match="shard"):
        checkpoint.load(b, path)
    st = torch.load(path, weights_only=True)
    st["draw_contract"] = 2
    torch.save(st, tmp_path / "old.pt")
    with pytest.raises(ValueError, match="draw contract"):
        checkpoint.load(_learner(), tmp_path / "old.pt")
    checkpoint.load(DQNLearner(DQNConfig(channels=8, blocks=2, bf16=False, seed=3, lr=5e-4), device="cpu"), path)


def test_checkpoint_reads_format_1_with_a_warning(tmp_path):
    """a format-1 file (no draw_contract / gid0 keys) still resumes -- contract 3 assumed,
    with a warning -- and resumes bit-identically; the config checks still apply."""
    from rein48_amd import checkpoint
    from rein48_amd.dqn import DQNConfig, DQNLearner
    data = _batches(4)
    a = _learner()
    for x, act, y in data[:2]:
        a.learn(x, act, y)
    checkpoint.save(a, tmp_path / "new.pt")
    st = torch.load(tmp_path / "new.pt", weights_only=True)
    st["format"] = 1
    del st["draw_contract"], st["gid0"]
    torch.save(st, tmp_path / "v1.pt")
    b = _learner()
    with pytest.warns(UserWarning, match="format 1"):
        checkpoint.load(b, tmp_path / "v1.pt")
    for x, act, y in data[2:]:
        a.learn(x, act, y)
        b.learn(x, act, y)
    assert torch.equal(a.flat.data, b.flat.data) and b.updates == a.updates == 4
    with pytest.raises(ValueError, match="seed"), pytest.warns(UserWarning):
        checkpoint.load(DQNLearner(DQNConfig(channels=8, blocks=2, bf16=False, seed=4), device="cpu"), tmp_path / "v1.pt")
    st["format"] = 0
    torch.save(st, tmp_path / "v0.pt")
    with pytest.raises(ValueError, match="format"):
        checkpoint.load(_learner(), tmp_path / "v0.pt")
