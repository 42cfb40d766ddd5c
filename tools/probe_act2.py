"""GPU probe: config-5 acting time in the bench's step pattern (act -> env step + store -> update,
synchronized every step, as bench.dqn_config5) against back-to-back acting and against the same
pattern with no host synchronization between steps; per-phase HIP-event times (ms).

    python tools/probe_act2.py [steps]"""
import sys

import torch

sys.path.insert(0, ".")
from rein48_amd.dqn import DQNConfig, DQNTrainer  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
cfg = DQNConfig(n_boards=1 << 21, replay_capacity=1 << 25, batch=1 << 16, learn_start=1, seed=1)
tr = DQNTrainer(cfg, device="cuda:0")
tr.train_step()
s = torch.cuda.current_stream()


def step(ev):
    ev[0].record(s)
    st = tr.env.boards.clone()
    a = tr.act()
    ev[1].record(s)
    _, reward, done = tr.env.step(a, auto_reset=True, merge_reward=True)
    tr.replay.store(st, a, reward.float(), tr.env.boards, done)
    tr.steps += 1
    ev[2].record(s)
    tr.update()
    ev[3].record(s)


def report(name, evs):
    torch.cuda.synchronize()
    ph = [[e[i].elapsed_time(e[i + 1]) for e in evs] for i in range(3)]
    print("%-34s act %s | env %.3f | update %s" % (name, " ".join("%.2f" % x for x in ph[0]),
          sum(ph[1]) / len(ph[1]), " ".join("%.2f" % x for x in ph[2])), flush=True)


for rep in range(2):
    evs = []
    for _ in range(K):
        torch.cuda.synchronize()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        step(e)
        evs.append(e)
    report("bench pattern (sync per step)", evs)
    evs = []
    torch.cuda.synchronize()
    for _ in range(K):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        step(e)
        evs.append(e)
    report("no sync between steps", evs)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(K):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(s)
        tr.act()
        b.record(s)
        ts.append((a, b))
    torch.cuda.synchronize()
    print("%-34s act %s" % ("act only, back to back", " ".join("%.2f" % x.elapsed_time(y) for x, y in ts)), flush=True)
