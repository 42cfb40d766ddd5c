"""The bench's config-5 step loop (bench.dqn_config5 at 2^21 boards) for a per-kernel clock pass:
    rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d <dir> -o clk -- python3 tools/prof_dqn_step.py
    python tools/kernel_clocks.py <dir>"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

r = bench.dqn_config5(torch.device("cuda", 0), 0x20485EED, 1 << 21)
print("act %.3f ms update %.3f ms" % (r["act_ms"], r["update_ms"]), flush=True)
