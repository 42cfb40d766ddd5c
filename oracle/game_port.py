"""Faithful pure-Python restatement of the reference env -- TEST/BASELINE INFRASTRUCTURE ONLY.

Restates nevertiree/Rein48 game/GameClient.py (Game) and control/rand.py (Rand) with the
reference's cost model -- list-of-lists boards of raw tile values, a deep copy per move
to detect change (GameClient.py:137, 180), the global `random` module for every draw
(:121, :125; rand.py:11) -- so that timing it on the GPU box's host stands in for timing
the reference itself, which cannot travel there (BASELINE.md "CPU-baseline plan").
bench.py's cpu_baseline leg runs it; tests pin it against tests/golden/ (same seeded
trajectories as the reference) and the calibration in BASELINE.md ties its speed to the
reference's.
"""
import copy
import random

ACTION_NAMES = ("UP", "DOWN", "LEFT", "RIGHT")
_ALIASES = (("UP", "Up", "U", "up", "u", 0), ("DOWN", "Down", "D", "down", "d", 1),
            ("LEFT", "Left", "L", "left", "l", 2), ("RIGHT", "Right", "R", "right", "r", 3))


def _direction(action):
    for d, names in enumerate(_ALIASES):
        if action in names:
            return d
    raise ValueError("bad action %r" % (action,))


def _slide(cells):
    """One line toward index 0: compact, then merge equal neighbours once (GameClient.py:141-179)."""
    tiles = [v for v in cells if v]
    out = []
    k = 0
    while k < len(tiles):
        if k + 1 < len(tiles) and tiles[k] == tiles[k + 1]:
            out.append(tiles[k] * 2)
            k += 2
        else:
            out.append(tiles[k])
            k += 1
    return out + [0] * (len(cells) - len(out))


class PortGame:
    def __init__(self, size=4):
        self.size = max(4, size)
        self.state_matrix = None
        self.reset()

    def reset(self):
        self.state_matrix = [[0] * self.size for _ in range(self.size)]
        self.state_matrix = self.fill(self.state_matrix)
        return self.state_matrix

    @staticmethod
    def move(matrix, action):
        d = _direction(action)
        before = copy.deepcopy(matrix)  # the reference's change test (GameClient.py:137)
        if d >= 2:
            for r, row in enumerate(matrix):
                if d == 2:
                    row[:] = _slide(row)
                else:
                    row[:] = _slide(row[::-1])[::-1]
        else:
            cols = [list(col) for col in zip(*matrix)]
            for c, col in enumerate(cols):
                new = _slide(col) if d == 0 else _slide(col[::-1])[::-1]
                for r, v in enumerate(new):
                    matrix[r][c] = v
        return matrix, 0, before != matrix

    @staticmethod
    def fill(matrix):
        n = len(matrix)
        blank = [(i, j) for i in range(n) for j in range(n) if matrix[i][j] == 0]
        if blank:
            i, j = blank[random.randint(0, len(blank) - 1)]
            matrix[i][j] = 2 if random.uniform(0, 1) > 0.1 else 4
        return matrix

    @staticmethod
    def over(matrix):
        n = len(matrix)
        for i in range(n):
            for j in range(n):
                v = matrix[i][j]
                if v == 0 or (i + 1 < n and matrix[i + 1][j] == v) or (j + 1 < n and matrix[i][j + 1] == v):
                    return False
        return True

    def step(self, action):
        self.state_matrix, reward, changed = self.move(self.state_matrix, action)
        if changed:
            self.state_matrix = self.fill(self.state_matrix)
        return self.state_matrix, reward, self.over(self.state_matrix)


def random_action(*args):
    return ACTION_NAMES[random.randint(0, 3)]


def run_steps(n_steps, seed=0):
    """main.py:36-42 loop with auto-restart (a fresh game on done) for n_steps steps;
    returns the number of finished episodes."""
    random.seed(seed)
    g = PortGame()
    episodes = 0
    for _ in range(n_steps):
        _, _, done = g.step(random_action(g.state_matrix))
        if done:
            episodes += 1
            g = PortGame()
    return episodes
