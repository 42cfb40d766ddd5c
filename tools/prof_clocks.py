"""The config-3 (A3C, CNN bf16, both loss modes; reference MLP) and config-5 (DQN, ResNet-10) GPU
work of bench.py's extras, small counts, for one rocprofv3 --pmc GRBM_GUI_ACTIVE pass: every CNN /
MLP / ResNet kernel's average clock per dispatch = GRBM_GUI_ACTIVE / 8 XCDs / dispatch time
(tools/kernel_clocks.py). A profiled run clocks a few % below an unprofiled one
(/opt/skills/guides/MI355X_MICROARCH.md, DVFS give-back item 2): compare kernels within one pass.
    python tools/prof_clocks.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda:0")
n = 1 << 20
for mode, feats in (("textbook", "exponents"), ("reference", "values")):
    r = bench.a3c_config3(dev, 1, n, updates=2, mode=mode, features=feats, warmup=1)
    print("a3c cnn %s rollout %.2f update %.2f ms" % (mode, r["rollout_ms"], r["update_ms"]), flush=True)
r = bench.a3c_config3(dev, 1, n, updates=2, mode="reference", features="values", warmup=1, net="mlp", bf16=False)
print("a3c mlp reference rollout %.2f update %.2f ms" % (r["rollout_ms"], r["update_ms"]), flush=True)
r = bench.dqn_config5(dev, 1, 1 << 21, steps=2, warmup=2)
print("dqn act %.2f update %.2f ms" % (r["act_ms"], r["update_ms"]), flush=True)
