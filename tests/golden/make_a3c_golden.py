"""Generate golden fixtures for the A3C pieces of the reference that run without TensorFlow.

Runs only in the survey/build container, where the read-only reference lives at
/root/reference. algorithm/a3c/a3c.py cannot be imported (a3c.py:8 imports the missing
game.game_cli, and TensorFlow 1.x is absent), but two of its steps need nothing but numpy:

  returns   LocalAgent._get_target_value_list (a3c.py:246-256), a pure-numpy staticmethod.
            Its function definition is taken from the reference file with `ast` and executed
            with numpy only (no stand-ins for missing modules), on seeded reward lists.
  choice    LocalAgent.choose_action's sampling call (a3c.py:89-93):
            np.random.choice(range(4), p=prob_weights.ravel()) under np.random.seed(s), recorded
            together with the first np.random.random_sample() of the same seed (the uniform the
            legacy sampler consumes), so the oracle's "first k with cdf > u" rule is pinned to
            numpy's own implementation.

Writes a3c_golden.json next to this script (data only: inputs and the outputs the
reference code / numpy produced). Usage: python tests/golden/make_a3c_golden.py
"""
import ast
import json
import os
import sys

import numpy as np

REF = "/root/reference/algorithm/a3c/a3c.py"
HERE = os.path.dirname(os.path.abspath(__file__))


def reference_target_value_fn():
    tree = ast.parse(open(REF).read(), REF)
    for node in ast.walk(tree):
        if isinstance(node, ast.FunctionDef) and node.name == "_get_target_value_list":
            node.decorator_list = []                       # the staticmethod wrapper
            mod = ast.Module(body=[node], type_ignores=[])
            ns = {"np": np}
            exec(compile(mod, REF, "exec"), ns)
            return ns["_get_target_value_list"], node.lineno
    raise SystemExit("_get_target_value_list not found in " + REF)


def main():
    sys.dont_write_bytecode = True
    fn, line = reference_target_value_fn()
    rng = np.random.default_rng(0x2048A3C)
    returns = []
    for case in range(48):
        T = [1, 2, 3, 100][case % 4] if case < 8 else int(rng.integers(1, 101))
        kind = case % 3
        if kind == 0:       # the reference's env: reward is always 0 (GameClient.py:138)
            rewards = [0] * T
        elif kind == 1:     # merge-sum style integer rewards
            rewards = [int(x) for x in rng.integers(0, 64, T)]
        else:
            rewards = [float(x) for x in rng.normal(size=T)]
        last = 0.0 if case % 5 == 0 else float(rng.normal(scale=10.0))   # done -> 0 bootstrap (a3c.py:218-223)
        out = fn(rewards, last)
        returns.append({"rewards": rewards, "last_target_value": last,
                        "targets": [float(v) for v in np.asarray(out).reshape(-1)]})
    choice = []
    for s in range(400):
        p = rng.dirichlet(np.full(4, 0.7 if s % 2 else 3.0))
        if s % 7 == 0:
            p = np.eye(4)[s % 4] * 0.97 + 0.0075
        p = (p / p.sum()).astype(np.float32).astype(np.float64)   # prob_weights come out of TF as float32
        p = p / p.sum()
        np.random.seed(s)
        u = float(np.random.random_sample())
        np.random.seed(s)
        a = int(np.random.choice(range(len(p)), p=p.ravel()))
        choice.append({"seed": s, "p": [float(x) for x in p], "u": u, "action": a})
    out = {"source": "algorithm/a3c/a3c.py:%d (_get_target_value_list, executed), a3c.py:89-93 "
                     "(np.random.choice call form, numpy %s)" % (line, np.__version__),
           "returns": returns, "choice": choice}
    with open(os.path.join(HERE, "a3c_golden.json"), "w") as f:
        json.dump(out, f)
    print("wrote", len(returns), "return cases and", len(choice), "choice cases")


if __name__ == "__main__":
    main()
