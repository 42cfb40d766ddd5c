"""Drop-in for nevertiree/Rein48 control/rand.py (class Rand).

Rand.random_action(*args) -> "UP" | "DOWN" | "LEFT" | "RIGHT", uniform, from Python's
global `random` exactly as control/rand.py:9-11 does (randint(0, 3)), so a seeded run
interleaves its draws with Game's spawn draws like the reference. The batched form of
this policy runs inside the env kernel (VecGame.step(actions=None): Philox, 2 bits per
board-step), which is the one the hot path uses.
"""
import random

_NAMES = {0: "UP", 1: "DOWN", 2: "LEFT", 3: "RIGHT"}


class Rand:

    @staticmethod
    def random_action(*args):
        return _NAMES[random.randint(0, 3)]
