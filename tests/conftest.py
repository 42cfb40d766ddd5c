import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via `pytest -m gpu`)")


@pytest.fixture(scope="session")
def golden():
    import json
    return {
        "kats": json.load(open(os.path.join(GOLDEN, "kats.json"))),
        "traj": dict(np.load(os.path.join(GOLDEN, "trajectories.npz"))),
        "table": json.load(open(os.path.join(GOLDEN, "line_table.json"))),
        "fingerprint": json.load(open(os.path.join(GOLDEN, "fingerprint.json"))),
    }


def to_exp_scaled(matrix):
    """KAT matrices hold values like 1, 2, 4 (GameClientTest.py); doubling every value keeps
    the move identical (it only compares and adds equal values) and makes them 2^e, e>=1."""
    out = []
    for row in matrix:
        for v in row:
            out.append(0 if v == 0 else (2 * v).bit_length() - 1)
    return out
