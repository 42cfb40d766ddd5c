"""GPU experiment: A3C rollout time (config 3: 2^20 boards x 100 steps, CNN bf16) for library
builds given on the command line (default: the product library), megakernel and per-step paths."""
import sys

import torch

sys.path.insert(0, ".")
from rein48_amd import _lib  # noqa: E402

libs = sys.argv[1:] or [_lib.LIB_PATH]
for path in libs:
    _lib.LIB_PATH, _lib._lib = path, None
    from rein48_amd.a3c import A3CConfig, A3CTrainer
    for mega in ((True,) if len(sys.argv) > 1 else (True, False)):
        cfg = A3CConfig(n_boards=1 << 20, max_steps=100, mode="textbook", net="cnn", bf16=True,
                        features="exponents", seed=3, fused_rollout=mega)
        tr = A3CTrainer(cfg, device="cuda:0")
        tr.rollout()
        torch.cuda.synchronize()
        # variants must reproduce the first rollout bit for bit (boards, actions, done)
        digest = int((tr.boards.view(torch.int32).long() * 2654435761).sum() + (tr.actions.long() * 40503).sum()
                     + tr.done.long().sum()) & 0xFFFFFFFF
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(3):
            tr.rollout()
        b.record()
        torch.cuda.synchronize()
        print("%-40s megakernel=%d  rollout %.2f ms  digest %08x" % (path.split("/")[-1], mega, a.elapsed_time(b) / 3,
                                                                     digest), flush=True)
        del tr
        torch.cuda.empty_cache()
