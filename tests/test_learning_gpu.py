"""The textbook trainers learn: after a bounded amount of training, whole
episodes played with the trained policy (evaluate.play_episodes: main.py's play() loop, score =
tile sum at game over, main.py:48) score above the reference random policy -- measured in the same
test with the same evaluation, and pinned against the reference random-policy fingerprint
(tests/golden/fingerprint.json: 20,000 reference episodes, mean score 265.1). The reference's own
mode cannot learn (reward is always 0, GameClient.py:138); these use the opt-in merge reward."""
import json
import os

import pytest

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
HERE = os.path.dirname(os.path.abspath(__file__))


def _fingerprint():
    return json.load(open(os.path.join(HERE, "golden", "fingerprint.json")))


def test_random_policy_evaluation_matches_reference_fingerprint():
    """The evaluation loop itself: the uniform random policy's mean score over 8,192 GPU episodes is
    the reference's 265.1 within 4 standard errors (sd 83.4)."""
    from rein48_amd.evaluate import play_episodes, random_policy
    fp = _fingerprint()["score"]
    ev = play_episodes(random_policy(3), 8192, DEV, seed=21)
    assert ev["finished"] == 1.0
    se = fp["sd"] / 8192 ** 0.5
    assert abs(ev["mean_score"] - fp["mean"]) < 4 * se, (ev["mean_score"], fp["mean"])


def test_a3c_textbook_cnn_learns():
    """A3C, textbook loss with the merge reward, CNN bf16, 2^16 boards x 1,500 updates: the trained
    policy's mean whole-episode score exceeds the reference random policy's by >= 12 % (measured
    curve, profiles/r04/learning.json: 275 / 305 / 324 / 336 after 500 / 1000 / 1500 / 2000 updates)."""
    from rein48_amd.a3c import A3CConfig, A3CTrainer
    from rein48_amd.evaluate import play_episodes
    fp = _fingerprint()["score"]["mean"]
    tr = A3CTrainer(A3CConfig(n_boards=1 << 16, max_steps=100, mode="textbook", net="cnn", bf16=True,
                              features="exponents", seed=3), device=DEV)
    for _ in range(1500):
        tr.train_step()
    ev = play_episodes(tr.policy(), 4096, DEV, seed=12)
    assert ev["mean_score"] > 1.12 * fp, ev


def test_dqn_resnet_learns():
    """DQN (ResNet-10 bf16, merge reward, HBM replay ring), 4,096 boards x 1,500 env steps: the greedy
    policy (epsilon 0.01) scores >= 50 % above the reference random policy (measured curve,
    profiles/r04/learning.json: 437 / 515 / 561 / 587 after 750 / 1500 / 2250 / 3000 steps)."""
    from rein48_amd.dqn import DQNConfig, DQNTrainer
    from rein48_amd.evaluate import play_episodes
    fp = _fingerprint()["score"]["mean"]
    dq = DQNTrainer(DQNConfig(n_boards=4096, replay_capacity=1 << 21, batch=4096, learn_start=16384, seed=5,
                              eps_decay_steps=1500), device=DEV)
    for _ in range(1500):
        dq.train_step()
    ev = play_episodes(dq.policy(), 4096, DEV, seed=13)
    assert ev["mean_score"] > 1.5 * fp, ev
