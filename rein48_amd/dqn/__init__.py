"""Value-based training around the env (BASELINE config 5): ResNet-10 Q-network, DQN with an
HBM-resident replay ring (rein48_amd/replay.py)."""
from .nets import ResNet10Q
from .trainer import DQNConfig, DQNLearner, DQNTrainer

__all__ = ["ResNet10Q", "DQNConfig", "DQNLearner", "DQNTrainer"]
