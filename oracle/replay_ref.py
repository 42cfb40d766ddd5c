"""TEST INFRASTRUCTURE ONLY -- restatement of the reference transition buffer
(algorithm/ddpg/replay.py:8-47), pinned by tests/golden/replay.json (generated from the
reference itself by tests/golden/make_replay_golden.py).

  store   (:18-21)  append while cur_size < max_size, otherwise drop
  sample  (:23-27)  sub_list(buffer, batch) -> list_2_dict -> clear()
  sub_list (:29-34) the list itself when num > len, else random.sample(list, num)
  list_2_dict (:36-43) four numpy arrays: state, action, reward, next_state
Uses CPython's global `random`, exactly as the reference does, so under the same
random.seed it picks the same rows.
"""
import random

import numpy as np

MINI_BATCH_SIZE = 10   # replay.py:5


class ReplayRef:
    def __init__(self, replay_size=100):
        self.max_size = replay_size
        self.cur_size = 0
        self.buffer = []

    def filled(self):
        return self.max_size <= self.cur_size

    def store(self, trans):
        if self.cur_size < self.max_size:
            self.cur_size += 1
            self.buffer.append(trans)

    def sample(self, batch_size=MINI_BATCH_SIZE):
        rows = self.buffer if batch_size > len(self.buffer) else random.sample(self.buffer, batch_size)
        out = {"state": np.array([x[0] for x in rows]), "action": np.array([x[1] for x in rows]),
               "reward": np.array([x[2] for x in rows]), "next_state": np.array([x[3] for x in rows])}
        self.cur_size = 0
        self.buffer = []
        return out
