"""Drop-in replacement for nevertiree/Rein48 game/GameClient.py (class Game).

Same names, argument meaning, return shapes and errors as the reference:
  Game(table_matrix_size=4)            GameClient.py:19-29
  .reset(display=False) -> state       :33-38   (new list; ONE spawned tile)
  .step(action) -> (state, 0, done)    :40-51   (state mutated in place and aliased)
  .state_matrix / size attributes      :17, :21-27
  static create_matrix / has_game_over / has_table_filled / random_fill_grid /
  update_matrix / print_terminal       :55-269
Actions: "UP"/"Up"/"U"/"up"/"u"/0, ... /3 matched by equality like the reference
(:140, :182, :206, :230), so True means DOWN and 2.0 means LEFT; anything else raises
ValueError (:254).

Compute runs on the GPU through librein48.so: each 4x4 step is ONE r48_game_step1 launch that
moves the board and evaluates every spawn outcome (blank rank x tile) with its game over, then
the host's draw picks one. The spawn DRAWS are taken
from Python's global `random` exactly as the reference takes them (randint over the
row-major blank list, then uniform(0,1) > 0.1 -> 2 else 4, GameClient.py:121-125), so
`random.seed(s)` gives the reference's trajectory bit for bit. The batched VecGame draws
on device instead (Philox).

Board sizes: the exponent kernels are 4x4. Game(n) with n > 4 runs
on the value-domain grid kernels (r48_values_move_grid / r48_values_check_grid: any rows x
cols, one GPU thread per line of the move), composed like GameClient.py:45-51 with the spawn
drawn from the global `random` on the host, so it follows the reference's trajectories under
`random.seed` as well. The static helpers accept any integer tiles on any rectangular matrix
(the reference's own tests use 4x1 / 1x4 matrices and the value 1).
"""
import copy
import ctypes
import random
import weakref

import numpy as np
import torch

from .. import _lib
from .._lib import check, ptr

_UP = ["UP", "Up", "U", "up", "u", 0]
_DOWN = ["DOWN", "Down", "D", "down", "d", 1]
_LEFT = ["LEFT", "Left", "L", "left", "l", 2]
_RIGHT = ["RIGHT", "Right", "R", "right", "r", 3]
_BAD_ACTION = "Input action signal is wrong:\n You must input valid inputs, such as  [U] [D] [L] [R]... "


def action_code(action):
    """The reference's direction test (GameClient.py:140,182,206,230): `action in [...]`."""
    for code, names in enumerate((_UP, _DOWN, _LEFT, _RIGHT)):
        if action in names:
            return code
    raise ValueError(_BAD_ACTION)


def _exponent(v):
    """raw tile value -> exponent, or None if not 0 / 2^e with 1 <= e <= 30"""
    if v == 0:
        return 0
    if isinstance(v, bool) or v != int(v):
        return None
    v = int(v)
    if v < 2 or v & (v - 1) or v > (1 << 30):
        return None
    return v.bit_length() - 1


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("rein48 Game needs a ROCm GPU (torch.cuda.is_available() is False)")
    return torch.device("cuda", torch.cuda.current_device())


def _pad(matrix, code):
    """rows x cols (<= 4x4) -> 4x4 int32 board, anchored on the side the tiles move toward
    (zeros on the far side cannot change any line)."""
    rows, cols = len(matrix), len(matrix[0])
    if rows > 4 or cols > 4 or any(len(r) != cols for r in matrix):
        raise NotImplementedError("rein48 kernels handle rectangular matrices up to 4x4, got %dx%d"
                                  % (rows, max(len(r) for r in matrix)))
    r0 = 4 - rows if code == 1 else 0
    c0 = 4 - cols if code == 3 else 0
    board = [0] * 16
    for i in range(rows):
        for j in range(cols):
            board[4 * (r0 + i) + c0 + j] = int(matrix[i][j])
    return board, r0, c0


def _grid_tensor(matrix):
    rows, cols = len(matrix), len(matrix[0])
    if any(len(r) != cols for r in matrix):
        raise ValueError("rein48 kernels need a rectangular matrix")
    return torch.tensor(matrix, dtype=torch.int32, device=_device()).contiguous(), rows, cols


def _grid_move(matrix, code):
    """update_matrix on any rows x cols (r48_values_move_grid), written back in place."""
    b, rows, cols = _grid_tensor(matrix)
    a = torch.tensor([code], dtype=torch.int8, device=b.device)
    check(_lib.load().r48_values_move_grid(ptr(b), 1, rows, cols, ptr(a), None,
                                           torch.cuda.current_stream(b.device).cuda_stream))
    out = b.cpu().tolist()
    for i in range(rows):
        matrix[i][:] = out[i]


def _grid_check(matrix):
    b, rows, cols = _grid_tensor(matrix)
    out = torch.empty(2, dtype=torch.uint8, device=b.device)
    check(_lib.load().r48_values_check_grid(ptr(b), 1, rows, cols, ptr(out[0:1]), ptr(out[1:2]),
                                            torch.cuda.current_stream(b.device).cuda_stream))
    filled, over = out.cpu().tolist()
    return bool(filled), bool(over)


class Game:

    state_matrix, state_space_size = None, 0

    def __init__(self, table_matrix_size=4):
        self.reward_space_size = 1
        self.action_space_size = 4
        self.state_space_size = 4 if table_matrix_size < 4 else table_matrix_size
        dev = _device()
        # 4x4: one r48_game_step1 launch per step (the move and every spawn outcome with its game
        # over, k_game_step1), the board passed in the kernel arguments and the 520-byte result
        # written by the kernel straight into mapped, coherent host memory (r48_host_alloc): one
        # launch and one stream synchronisation per step. The spawn draw stays on the global
        # `random` (GameClient.py:121,125) and picks a candidate. Larger boards: the value-domain
        # grid kernels.
        self._small = self.state_space_size == 4
        if self._small:
            lib = self._lib = _lib.load()
            nb = int(lib.r48_game_step1_out_bytes())
            self._dev = torch.device(dev)
            dp = ctypes.c_void_p()
            with torch.cuda.device(self._dev):
                hp = lib.r48_host_alloc(nb, ctypes.byref(dp))
            if not hp:
                raise RuntimeError("r48_host_alloc failed: %s" % lib.r48_last_error().decode())
            weakref.finalize(self, lib.r48_host_free, hp)
            self._out = dp.value
            self._hn = np.ctypeslib.as_array((ctypes.c_uint8 * nb).from_address(hp))
            self._b = np.zeros(16, dtype=np.int8)
        self.reset()

    # ---------------------------------------------------------------- public (GameClient.py:33-51)
    def reset(self, display=False):
        self.state_matrix = self.create_matrix(self.state_space_size)
        self.state_matrix = self.random_fill_grid(self.state_matrix)
        if display:
            Game.print_terminal(self.state_matrix)
        return self.state_matrix

    def step(self, action):
        code = action_code(action)
        exps = [_exponent(v) for row in self.state_matrix for v in row] if self._small else [None]
        if any(e is None for e in exps):
            # tiles outside 2^e: the value-domain kernels, composed like GameClient.py:45-51
            self.state_matrix, reward, changed = self.update_matrix(self.state_matrix, code)
            if changed:
                self.state_matrix = Game.random_fill_grid(self.state_matrix)
            return self.state_matrix, reward, Game.has_game_over(self.state_matrix)
        b, hn = self._b, self._hn
        b[:] = exps
        st = torch.cuda.current_stream(self._dev)
        check(self._lib.r48_game_step1(b.ctypes.data, code, self._out, st.cuda_stream))
        st.synchronize()
        c = 0                                                      # unchanged: no spawn (GameClient.py:49)
        if hn[512]:
            r = random.randint(0, int(hn[513]) - 1)                # GameClient.py:121
            c = 2 * r + (0 if random.uniform(0, 1) > 0.1 else 1)  # GameClient.py:125
        over = (int(hn[516]) | int(hn[517]) << 8 | int(hn[518]) << 16 | int(hn[519]) << 24) >> c & 1
        cand = hn[16 * c:16 * c + 16]
        for k in range(16):  # write back into the SAME lists (aliasing, GameClient.py:45)
            e = int(cand[k])
            self.state_matrix[k // 4][k % 4] = (1 << e) if e else 0
        return self.state_matrix, 0, bool(over)

    # ---------------------------------------------------------------- static helpers (:55-269)
    @staticmethod
    def create_matrix(table_size=4):
        return [[0 for _ in range(table_size)] for _ in range(table_size)]

    @staticmethod
    def _check_kernel(game_matrix):
        rows, cols = len(game_matrix), len(game_matrix[0])
        if rows > 4 or cols > 4:
            return _grid_check(game_matrix)
        board, _, _ = _pad(game_matrix, 0)
        dev = _device()
        b = torch.tensor(board, dtype=torch.int32, device=dev)
        out = torch.empty(2, dtype=torch.uint8, device=dev)
        check(_lib.load().r48_values_check(ptr(b), 1, rows, cols, ptr(out[0:1]), ptr(out[1:2]),
                                           torch.cuda.current_stream(dev).cuda_stream))
        filled, over = out.cpu().tolist()
        return bool(filled), bool(over)

    @staticmethod
    def _check(game_matrix):
        """(has_table_filled, has_game_over). On a non-square matrix the reference's game-over loop
        (GameClient.py:74-91) runs i and j over range(len(matrix)) = the row count: with fewer rows
        than columns it only sees the leading rows x rows block; with more rows its first row's last
        column compares against m[0][cols] (IndexError) unless an equal pair met earlier in that
        row's scan -- (0, j)-(0, j + 1) or (0, j)-(1, j) -- returned first; both reproduced here.
        has_table_filled (:96-100) scans every item."""
        rows, cols = len(game_matrix), len(game_matrix[0])
        filled, over = Game._check_kernel(game_matrix)
        if rows == cols or not filled:
            return filled, over
        if rows > cols:
            r0, r1 = game_matrix[0], game_matrix[1]
            if any(r0[j] == r0[j + 1] for j in range(cols - 1)) or any(r0[j] == r1[j] for j in range(cols)):
                return filled, False
            raise IndexError("list index out of range")
        return filled, Game._check_kernel([row[:rows] for row in game_matrix])[1]

    @staticmethod
    def has_game_over(game_matrix):
        return Game._check(game_matrix)[1]

    @staticmethod
    def has_table_filled(game_matrix):
        return Game._check(game_matrix)[0]

    @staticmethod
    def random_fill_grid(game_matrix):
        """Host RNG glue (GameClient.py:102-127): enumerate the blanks row-major, draw with the
        global `random` like the reference, write the tile in place."""
        blank = [(i, j) for i in range(len(game_matrix)) for j in range(len(game_matrix))
                 if game_matrix[i][j] == 0]
        if not blank:
            return game_matrix
        i, j = blank[random.randint(0, len(blank) - 1)]
        game_matrix[i][j] = 2 if (random.uniform(0, 1) > 0.1) else 4
        return game_matrix

    @staticmethod
    def update_matrix(matrix, action):
        """GameClient.py:129-254 on the GPU (value-domain kernel): mutates `matrix` in place,
        returns (matrix, 0, changed)."""
        code = action_code(action)
        origin = copy.deepcopy(matrix)
        if len(matrix) > 4 or len(matrix[0]) > 4:
            _grid_move(matrix, code)
            return matrix, 0, (origin != matrix)
        board, r0, c0 = _pad(matrix, code)
        dev = _device()
        b = torch.tensor(board, dtype=torch.int32, device=dev)
        a = torch.tensor([code], dtype=torch.int8, device=dev)
        check(_lib.load().r48_values_move(ptr(b), ptr(a), 1, None, None,
                                          torch.cuda.current_stream(dev).cuda_stream))
        out = b.cpu().tolist()
        for i in range(len(matrix)):
            for j in range(len(matrix[0])):
                matrix[i][j] = out[4 * (r0 + i) + c0 + j]
        return matrix, 0, (origin != matrix)

    @staticmethod
    def print_terminal(matrix):
        width, height = len(matrix[0]), len(matrix)
        rule = "-" * (1 + 7 * width)
        lines = [rule]
        for i in range(height):
            cells = [(str(matrix[i][j]).center(6) if matrix[i][j] != 0 else " " * 6) for j in range(width)]
            lines.append("|" + "|".join(cells) + "|")
            lines.append(rule)
        print("\n".join(lines))
