"""Probe: config-5 DQN step timing (bench.py's dqn_config5 extra) on its own."""
import json
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 21
    print(json.dumps(bench.dqn_config5(torch.device("cuda", 0), 0x20485EED, n)), flush=True)
