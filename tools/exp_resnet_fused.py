"""Probe: fused ResNet-10 inference (r48_resnet_q_forward) throughput at 2^21 boards.

Useful FLOPs count only in-grid taps (100 of 144 (cell, tap) pairs); issued MFMA FLOPs count
every MFMA the kernel runs (in-grid taps, 18 planes padded to 32, the skip connections as identity
MFMAs, the head's 4 rows padded to 16)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from rein48_amd.dqn.fused import pack_resnet, resnet_q_forward  # noqa: E402
from rein48_amd.dqn.nets import ResNet10Q  # noqa: E402

C = 64
USEFUL = 2 * 100 * (18 * C + 8 * C * C) + 2 * 16 * C * 4
ISSUED = 2 * 100 * (32 * C + 8 * C * C) + 2 * 16 * 4 * C * 32 + 2 * 16 * C * 16   # per board


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 21
    if len(sys.argv) > 2:                                 # a variant library (tools/build_variant.sh)
        from rein48_amd import _lib
        _lib.LIB_PATH, _lib._lib = sys.argv[2], None
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = ResNet10Q().to(dev).eval()
    packed = pack_resnet(net)
    boards = torch.randint(0, 12, (n, 16), dtype=torch.int8, device=dev)
    out = {}
    for name, kw in (("q", dict(q=True)), ("act", dict(q=False, actions=True, eps=0.1))):
        resnet_q_forward(boards, packed, **kw)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        reps = 5
        ev[0].record()
        for _ in range(reps):
            resnet_q_forward(boards, packed, **kw)
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / reps
        out[name] = {"ms": ms, "boards_per_s": n / ms * 1e3, "useful_TFLOPs": n * USEFUL / ms / 1e9,
                     "issued_mfma_TFLOPs": n * ISSUED / ms / 1e9, "frac_issued_of_2.5PF": n * ISSUED / ms / 1e9 / 2500}
    q, _ = resnet_q_forward(boards, packed)
    out["q_checksum"] = float(q.double().sum())              # tiling variants must agree bit for bit
    out["q_bits_hash"] = int(q.view(torch.int32).long().mul(2654435761).sum()) & 0xFFFFFFFF
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
