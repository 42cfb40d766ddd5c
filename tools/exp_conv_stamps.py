"""Reads the k_conv_wgrad<64> phase stamps of a tools/stamp_conv.py build (GPU): mean cycles per
step and wave in (vmcnt wait, barrier, k-steps + DMA issue) at `boards` boards.
    python tools/exp_conv_stamps.py build/lib_conv_stamp.so [boards]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd import _lib  # noqa: E402

_lib.LIB_PATH, _lib._lib = sys.argv[1], None
from rein48_amd.dqn import conv as C  # noqa: E402

B = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 16
dev = torch.device("cuda:0")
x = torch.randn(B, 16, 64, device=dev).to(torch.bfloat16)
dy = torch.randn(B, 16, 64, device=dev).to(torch.bfloat16)
for _ in range(3):
    C.conv3x3_wgrad(dy, x)
torch.cuda.synchronize()
ws = C._WS[(64, str(dev))]
grid = torch.cuda.get_device_properties(0).multi_processor_count
rec = 9 * 64 * 64
W = 8                                                                            # waves per workgroup
st = torch.stack([ws[g * rec:g * rec + 16 * W].view(torch.int64) for g in range(grid)]).cpu()   # [grid, 8 W]
steps = (B * 16 + 127) // 128 / grid
names = ["vmcnt wait", "barrier", "-", "-", "k-steps + DMAs"]
tot = st.double().mean(0).view(W, 8).mean(0)[:5]
print("boards %d, %.1f steps per workgroup; cycles per step per wave:" % (B, steps))
for k, n in enumerate(names):
    print("  %-12s %8.1f" % (n, float(tot[k]) / steps))
print("  total        %8.1f" % (float(tot.sum()) / steps))
