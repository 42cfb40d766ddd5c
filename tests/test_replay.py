"""Transition store (config 5): oracle pinned to the reference Replay, index generators.

CPU: oracle/replay_ref.py reproduces tests/golden/replay.json (generated from the reference's
algorithm/ddpg/replay.py) row for row; the Feistel sampler draws without replacement and the
ring sampler is uniform. GPU (tests/test_replay_gpu.py): the HIP store against both.
"""
import json
import os
import random

import numpy as np
import pytest

from oracle import native as O
from oracle.replay_ref import ReplayRef

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def replay_golden():
    with open(os.path.join(HERE, "golden", "replay.json")) as f:
        return json.load(f)


def test_replay_ref_matches_reference_fixture(replay_golden):
    for sc in replay_golden["scenarios"]:
        random.seed(sc["seed"])
        rep = ReplayRef(sc["replay_size"])
        for t in sc["transitions"]:
            rep.store(t)
        assert rep.filled() == sc["filled"] and rep.cur_size == sc["cur_size_before"], sc["name"]
        out = rep.sample() if sc["batch_size"] is None else rep.sample(sc["batch_size"])
        for k, v in sc["sample"].items():
            assert np.asarray(v).tolist() == out[k].tolist(), (sc["name"], k)
            assert list(out[k].shape) == sc["sample_shapes"][k]
        assert rep.cur_size == sc["cur_size_after"] == 0


def test_fixture_semantics(replay_golden):
    """What the fixture pins, spelled out: drop past max_size, whole buffer in order when
    batch > len, without replacement otherwise, clear after sample."""
    by = {s["name"]: s for s in replay_golden["scenarios"]}
    assert by["overflow_all"]["cur_size_before"] == 100 and by["overflow_all"]["picked"] == list(range(100))
    assert by["fewer"]["picked"] == [0, 1, 2]
    assert sorted(by["exact_perm"]["picked"]) == list(range(5)) and by["exact_perm"]["picked"] != list(range(5))
    sub = by["subset"]["picked"]
    assert len(sub) == 10 and len(set(sub)) == 10
    assert by["empty"]["sample_shapes"]["state"] == [0] and replay_golden["mini_batch_size"] == 10
    assert len(by["default_batch"]["picked"]) == 10


@pytest.mark.parametrize("size", [1, 2, 3, 5, 64, 1000, 1023, 1025, 65_537])
def test_feistel_sampler_is_without_replacement(size):
    for ctr in (0, 7):
        n = min(size, 4096)
        idx = O.replay_index(0xABCDEF, ctr, size, n, ring=False)
        assert idx.min() >= 0 and idx.max() < size
        assert len(np.unique(idx)) == n
    if size <= 4096:
        full = O.replay_index(0xABCDEF, 3, size, size, ring=False)
        assert sorted(full.tolist()) == list(range(size))       # batch == size: a permutation
        if size >= 5:
            assert full.tolist() != list(range(size))


def test_feistel_sampler_is_uniform_over_slots():
    size, trials = 37, 4000
    counts = np.zeros(size)
    for ctr in range(trials):
        counts[O.replay_index(99, ctr, size, 1, ring=False)[0]] += 1
    exp = trials / size
    chi2 = float(((counts - exp) ** 2 / exp).sum())
    assert chi2 < 80, chi2          # 36 dof, p ~ 5e-5


def test_ring_sampler_uniform_and_in_range():
    size = 1_000_003
    idx = O.replay_index(5, 0, size, 200_000, ring=True)
    assert idx.min() >= 0 and idx.max() < size
    counts = np.bincount(idx * 10 // size, minlength=10)
    exp = idx.size / 10
    assert float(((counts - exp) ** 2 / exp).sum()) < 35
    big = O.replay_index(5, 1, 6 << 30, 1000, ring=True)    # 64-bit sizes (> 2^32 slots)
    assert big.max() < (6 << 30) and big.max() > (1 << 32)
