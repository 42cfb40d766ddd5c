"""rein48_amd -- MI355X-native vectorized 2048 environment (nevertiree/Rein48's hot path).

  VecGame        batched env on one GPU (gfx950 kernels in librein48.so, C-ABI include/rein48.h)
  game.Game      drop-in for game/GameClient.py:Game
  control.Rand   drop-in for control/rand.py:Rand
"""
from .env import ACTIONS, VecGame  # noqa: F401

__version__ = "0.1.0"
