"""GPU experiment: do the textbook trainers learn? Whole-episode evaluation (evaluate.play_episodes:
main.py's play() loop, score = tile sum at game over) of the reference random policy and of the A3C
(textbook loss, merge reward, CNN bf16) and DQN (ResNet-10 bf16) policies after a bounded amount
of training, against the reference random-policy fingerprint (tests/golden/fingerprint.json:
20,000 reference episodes, mean score 265.1).

    python tools/exp_learning.py [out.json] [--a3c-updates N] [--dqn-steps N]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rein48_amd.evaluate import play_episodes, random_policy  # noqa: E402

DEV = "cuda:0"


def log(*a):
    print(*a, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out", nargs="?", default="gpurun_out/learning.json")
    ap.add_argument("--a3c-updates", type=int, default=2000)
    ap.add_argument("--a3c-boards", type=int, default=1 << 16)
    ap.add_argument("--dqn-steps", type=int, default=3000)
    ap.add_argument("--dqn-boards", type=int, default=4096)
    ap.add_argument("--eval-boards", type=int, default=1 << 14)
    ap.add_argument("--evals", type=int, default=4)
    args = ap.parse_args()
    fp = json.load(open(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "fingerprint.json")))
    res = {"reference_random_fingerprint": {k: fp[k] for k in fp if not isinstance(fp[k], (list, dict))}}
    t0 = time.time()
    res["random_policy"] = play_episodes(random_policy(1), args.eval_boards, DEV, seed=11)
    log("random", res["random_policy"]["mean_score"], "%.1fs" % (time.time() - t0))

    from rein48_amd.a3c import A3CConfig, A3CTrainer
    cfg = A3CConfig(n_boards=args.a3c_boards, max_steps=100, mode="textbook", net="cnn", bf16=True,
                    features="exponents", seed=3)
    tr = A3CTrainer(cfg, device=DEV)
    curve = [dict(updates=0, **play_episodes(tr.policy(), args.eval_boards, DEV, seed=12))]
    every = max(1, args.a3c_updates // args.evals)
    t1 = time.time()
    for u in range(1, args.a3c_updates + 1):
        out = tr.train_step()
        if u % every == 0 or u == args.a3c_updates:
            ev = play_episodes(tr.policy(), args.eval_boards, DEV, seed=12)
            curve.append(dict(updates=u, train_s=time.time() - t1, losses=out, **ev))
            log("a3c", u, "score %.1f len %.1f" % (ev["mean_score"], ev["mean_length"]), "%.1fs" % (time.time() - t1))
    res["a3c_textbook_cnn"] = {"config": {k: getattr(cfg, k) for k in ("n_boards", "max_steps", "mode", "net", "features",
                                                                       "lr", "gamma", "beta")},
                               "curve": curve}
    del tr
    torch.cuda.empty_cache()

    from rein48_amd.dqn import DQNConfig, DQNTrainer
    dcfg = DQNConfig(n_boards=args.dqn_boards, replay_capacity=1 << 21, batch=4096, learn_start=16384, seed=5,
                     eps_decay_steps=max(1, args.dqn_steps // 2))
    dq = DQNTrainer(dcfg, device=DEV)
    curve = []
    every = max(1, args.dqn_steps // args.evals)
    t1 = time.time()
    for s in range(1, args.dqn_steps + 1):
        out = dq.train_step()
        if s % every == 0 or s == args.dqn_steps:
            ev = play_episodes(dq.policy(), args.eval_boards, DEV, seed=13)
            curve.append(dict(env_steps=s, train_s=time.time() - t1, loss=out.get("loss"), epsilon=out.get("epsilon"),
                              **ev))
            log("dqn", s, "score %.1f len %.1f" % (ev["mean_score"], ev["mean_length"]), "%.1fs" % (time.time() - t1))
    res["dqn_resnet10"] = {"config": {k: getattr(dcfg, k) for k in ("n_boards", "batch", "lr", "gamma", "target_sync",
                                                                     "eps_decay_steps", "reward_transform")},
                           "curve": curve}
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)
    log("wrote", args.out)


if __name__ == "__main__":
    main()
