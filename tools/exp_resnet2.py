"""Probe: the two fused ResNet-10 inference kernels side by side at 2^21 boards.

dpp  = r48_resnet_q_forward  (32x32x16, columns = 2 boards x 16 cells, all 144 (cell, tap) pairs)
cell = r48_resnet2_q_forward (16x16x32, columns = 16 boards of one cell, 100 in-grid pairs)
Useful FLOPs count in-grid taps only; issued FLOPs what each kernel's MFMAs compute. Also the
max relative difference between the two kernels' Q (both bf16) and against the fp32 net."""
import json
import sys

import torch

sys.path.insert(0, ".")
from rein48_amd.dqn.fused import pack_resnet, pack_resnet2_gpu, resnet2_q_forward, resnet_q_forward  # noqa: E402
from rein48_amd.dqn.kernels import board_onehot  # noqa: E402
from rein48_amd.dqn.nets import ResNet10Q  # noqa: E402

C = 64
USEFUL = 2 * 100 * (18 * C + 8 * C * C) + 2 * 16 * C * 4
ISSUED = {"dpp": 2 * 16 * 9 * (32 * C + 8 * C * C), "cell": 2 * 100 * (32 * C + 8 * C * C) + 2 * 16 * C * 16}


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 21
    only = sys.argv[2] if len(sys.argv) > 2 else None
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = ResNet10Q().to(dev).eval()
    with torch.no_grad():
        for m in net.bns:
            m.running_mean.uniform_(-0.3, 0.3)
            m.running_var.uniform_(0.5, 2.0)
        net.head.weight.normal_(std=0.05)
    boards = torch.randint(0, 12, (n, 16), dtype=torch.int8, device=dev)
    kern = {"dpp": (resnet_q_forward, pack_resnet(net)), "cell": (resnet2_q_forward, pack_resnet2_gpu(net))}
    out, qs = {}, {}
    for name, (fwd, packed) in kern.items():
        if only and name != only:
            continue
        ms = timed(lambda: fwd(boards, packed, q=False, actions=True, eps=0.1))
        out[name] = {"ms": ms, "boards_per_s": n / ms * 1e3, "useful_TFLOPs": n * USEFUL / ms / 1e9,
                     "issued_TFLOPs": n * ISSUED[name] / ms / 1e9,
                     "useful_frac_of_2.5PF": n * USEFUL / ms / 1e9 / 2500}
        qs[name] = fwd(boards, packed)[0]
        print(name, json.dumps(out[name]), flush=True)
    m = min(n, 1 << 16)
    with torch.no_grad():
        ref = net(board_onehot(boards[:m], dtype=torch.float32))
    for name, q in qs.items():
        out[name]["max_rel_err_vs_fp32"] = float(((q[:m] - ref).abs() / (ref.abs() + ref.abs().mean())).max())
    if len(qs) == 2:
        d, c = qs["dpp"], qs["cell"]
        out["max_rel_diff_dpp_cell"] = float(((d - c).abs() / (d.abs() + d.abs().mean())).max())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
