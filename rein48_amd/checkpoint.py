"""Checkpoint / resume of the trainers (SURVEY.md section 5 lists it as optional: the reference keeps no
`tf.train.Saver` in algorithm/a3c/a3c.py, so there is no reference format to match).

A checkpoint is everything that decides the trainer's next step, so that training resumed from it
is bit-identical to training that never stopped (tests/test_checkpoint_gpu.py):
  A3CTrainer  the net (flat parameters), the TF1 RMSProp slots (ms, momentum), the env's boards and
              its Philox step / reset counters, the policy's sampling counter, the update count
  DQNTrainer  online and target nets (parameters, BN running statistics, num_batches_tracked),
              Adam's m, v and step, the env's boards and counters, the env-step count, the update
              count, and the HBM replay ring (its counters and, unless replay=False, its contents in
              slot order: 38 B per stored transition)
Draws are keyed by counters, not by RNG state in memory, so restoring the
counters restores every later draw.

One file per rank: each rank owns its boards and its replay shard, so pass a
per-rank path (e.g. "ckpt.rank%d.pt" % rank). Files are written with torch.save and read back with
torch.load(weights_only=True): plain tensors, numbers and strings, nothing executable.

load() also reads format-1 files (round 4: no draw contract or shard recorded; contract 3 is
assumed, with a warning). It refuses (ValueError) a file whose resume could not be bit-identical: another kind or format,
another draw contract (R48_DRAW_CONTRACT: the same counters would give other draws), another rank's
shard (its first global board id, which keys every Philox draw), or a configuration that differs in a
field that fixes buffer shapes, the draws (seed), the network's inputs (features) or numerics (bf16),
or the loss (mode). Hyper-parameters such as lr, gamma or epsilon may differ (a deliberate change).
"""
import dataclasses
import warnings

import torch

from ._lib import DRAW_CONTRACT

FORMAT = 2

# configuration fields a checkpoint must agree on: buffer shapes, draws, inputs, numerics, loss
_MATCH_FIELDS = {
    "a3c": ("n_boards", "max_steps", "net", "seed", "mode", "features", "bf16"),
    "dqn": ("n_boards", "replay_capacity", "channels", "blocks", "bn", "bf16", "seed", "reward_transform"),
}


def _gid0(trainer, kind):
    """Global id of the trainer's first board (rank * n_boards): keys the Philox draws of its shard."""
    return int(trainer.gid0) if kind == "a3c" else int(trainer.rank) * int(trainer.cfg.n_boards)


def _kind(trainer):
    from .a3c.trainer import A3CTrainer
    from .dqn.trainer import DQNLearner
    if isinstance(trainer, A3CTrainer):
        return "a3c"
    if isinstance(trainer, DQNLearner):
        return "dqn"
    raise TypeError("checkpoint: expected an A3CTrainer or a DQNLearner / DQNTrainer, got %r" % type(trainer))


def _cpu(t):
    return t.detach().to("cpu", copy=True)


def _cpu_state(module):
    return {k: _cpu(v) for k, v in module.state_dict().items()}


def _env_state(env):
    step, reset = env.counters
    return {"boards": _cpu(env.boards), "step_ctr": int(step), "reset_ctr": int(reset)}


def _load_env(env, st):
    if tuple(st["boards"].shape) != tuple(env.boards.shape):
        raise ValueError("checkpoint: env has %s boards, the file %s" % (tuple(env.boards.shape), tuple(st["boards"].shape)))
    env.boards.copy_(st["boards"].to(env.boards.device))
    env.counters = (st["step_ctr"], st["reset_ctr"])


def _replay_state(rep, contents):
    size, head, ctr = rep.counters
    st = {"size": int(size), "head": int(head), "sample_ctr": int(ctr), "mode": rep.mode, "capacity": rep.capacity}
    if contents and size:
        rows = rep.gather(torch.arange(size, dtype=torch.int64, device=rep.device))
        st["rows"] = {k: _cpu(rows[k]) for k in ("state", "action", "reward", "next_state", "done")}
    return st


def _load_replay(rep, st):
    if st["mode"] != rep.mode or st["capacity"] != rep.capacity:
        raise ValueError("checkpoint: replay is %s/%d, the file %s/%d" % (rep.mode, rep.capacity, st["mode"],
                                                                          st["capacity"]))
    rep.clear()
    rows = st.get("rows")
    if rows is not None:   # slot k <- row k (a cleared ring stores from slot 0), then the counters
        d = rep.device
        rep.store(rows["state"].to(d), rows["action"].to(d), rows["reward"].to(d), rows["next_state"].to(d),
                  rows["done"].to(d))
        rep.set_counters(st["size"], st["head"], st["sample_ctr"])
    else:                  # contents not saved: an empty ring that refills (no stale rows sampled)
        rep.set_counters(0, 0, st["sample_ctr"])


def save(trainer, path, replay=True):
    """Write `trainer`'s state to `path` (replay=False leaves the DQN ring's contents out: the
    resumed ring starts empty and refills from the env before it is sampled again, so that resume
    is not bit-identical to uninterrupted training)."""
    kind = _kind(trainer)
    if trainer.device.type == "cuda":
        torch.cuda.synchronize(trainer.device)
    st = {"format": FORMAT, "kind": kind, "cfg": dataclasses.asdict(trainer.cfg), "updates": int(trainer.updates),
          "draw_contract": DRAW_CONTRACT, "gid0": _gid0(trainer, kind)}
    if kind == "a3c":
        st.update(net=_cpu_state(trainer.net), ms=_cpu(trainer.opt.ms), mom=_cpu(trainer.opt.mom),
                  env=_env_state(trainer.env), sample_ctr=int(trainer.sample_ctr))
    else:
        st.update(net=_cpu_state(trainer.net), target=_cpu_state(trainer.target), adam_m=_cpu(trainer.opt.m),
                  adam_v=_cpu(trainer.opt.v), adam_t=int(trainer.opt.t))
        if hasattr(trainer, "env"):
            st.update(env=_env_state(trainer.env), steps=int(trainer.steps),
                      replay=_replay_state(trainer.replay, replay))
    torch.save(st, path)


def load(trainer, path):
    """Restore a checkpoint written by save() into a trainer built with a matching configuration."""
    kind = _kind(trainer)
    st = torch.load(path, map_location="cpu", weights_only=True)
    if st.get("format") not in (1, FORMAT) or st.get("kind") != kind:
        raise ValueError("checkpoint: %s is a %s checkpoint of format %s, not a %s one of format %d"
                         % (path, st.get("kind"), st.get("format"), kind, FORMAT))
    if st["format"] == 1:
        # format 1 (round 4) predates the recorded draw contract and shard: contract 3 (Philox4x32-7
        # step draws, commit 66448e8) is assumed -- a file written by a library from before that
        # commit resumes under other env draws -- and the shard cannot be checked
        warnings.warn("checkpoint: %s is format 1: draw contract 3 assumed (files from before it resume "
                      "under other draws), its rank shard is not recorded (pass this rank's own file)" % path,
                      stacklevel=2)
        st = dict(st, draw_contract=3, gid0=_gid0(trainer, kind))
    if st["draw_contract"] != DRAW_CONTRACT:
        raise ValueError("checkpoint: %s was written under draw contract %d, this library draws under %d"
                         % (path, st["draw_contract"], DRAW_CONTRACT))
    if st["gid0"] != _gid0(trainer, kind):
        raise ValueError("checkpoint: %s holds the shard starting at board %d, this trainer's starts at %d "
                         "(another rank's file?)" % (path, st["gid0"], _gid0(trainer, kind)))
    cfg = dataclasses.asdict(trainer.cfg)
    for f in _MATCH_FIELDS[kind]:
        if cfg[f] != st["cfg"][f]:
            raise ValueError("checkpoint: %s = %r in the trainer, %r in %s" % (f, cfg[f], st["cfg"][f], path))
    dev = trainer.device
    with torch.no_grad():
        trainer.net.load_state_dict(st["net"])   # copies into the flat buffers' views
        if kind == "a3c":
            trainer.opt.ms.copy_(st["ms"].to(dev))
            trainer.opt.mom.copy_(st["mom"].to(dev))
            _load_env(trainer.env, st["env"])
            trainer.sample_ctr = st["sample_ctr"]
            trainer._rollout_v = None            # the rollout's values belong to the old weights
            trainer._wepoch += 1                 # repack the kernels' weight images
            trainer._mask = None
        else:
            trainer.target.load_state_dict(st["target"])
            trainer.opt.m.copy_(st["adam_m"].to(dev))
            trainer.opt.v.copy_(st["adam_v"].to(dev))
            trainer.opt.t = st["adam_t"]
            trainer._version += 1                # repack the fused-kernel weights of both nets
            if hasattr(trainer, "env"):
                if "env" not in st:
                    raise ValueError("checkpoint: %s holds a learner without env / replay" % path)
                _load_env(trainer.env, st["env"])
                trainer.steps = st["steps"]
                _load_replay(trainer.replay, st["replay"])
    trainer.updates = st["updates"]
    return st["cfg"]
