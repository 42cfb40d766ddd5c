"""Batched, synchronous A3C on the gfx950 env (the rows around the env step in SURVEY.md §8 a11-a16).

The reference (algorithm/a3c/a3c.py) runs N_WORKERS Python threads, each with one Game and a
local TF1 net: per episode segment it resets its game (:194), plays until done or MAX_STEP_NUM
= 100 steps choosing actions by np.random.choice over the softmax (:201-212), bootstraps
V(s_T) unless done (:218-223), builds discounted targets with gamma 0.9 dropping the last
reward (:225, :246-256), and pushes its gradients into the global net with RMSProp (:233).

Here one rollout advances every board of a VecGame in lockstep (millions of "workers" per GPU):
    per step:  board_features kernel -> net forward (PyTorch-ROCm) -> r48_sample_actions
               (fused softmax + Philox draw) -> r48_env_step (the env kernel)
    update:    pass 1 (no grad) values, bootstrap and r48_discounted_returns, per-segment
               constants; pass 2 chunked forward/backward of the loss (losses.py); one
               all-reduce of the flat gradient (RCCL across GPUs); fused TF1 RMSProp kernel.
mode "reference" keeps the reference's quirks: training pairs the POST-step state with the
action chosen from the pre-step state (:203-209), reward is 0 (GameClient.py:138), the last
reward is dropped, and the actor loss is the literal broadcast form. mode "textbook" uses
pre-step states, the merge reward, full n-step returns and -(beta*H + td*log p[a]).
"""
from dataclasses import dataclass

import torch
import torch.distributed as dist

from .. import _lib

from ..env import VecGame
from . import kernels as K
from .fused import cnn_forward, pack_cnn
from .losses import chunk_loss, segment_stats
from .nets import make_net
from .optim import FlatParams, RMSPropTF1


def _lib_workspace_floats():
    return _lib.load().r48_cnn_train_workspace_floats()


@dataclass
class A3CConfig:
    n_boards: int = 4096          # boards (segments) per GPU
    max_steps: int = 100          # MAX_STEP_NUM, a3c.py:20
    gamma: float = 0.9            # a3c.py:247
    beta: float = 0.001           # ENTROPY_BETA, a3c.py:21
    lr: float = 1e-3              # LR_A = LR_C, a3c.py:22-23
    net: str = "mlp"              # "mlp" (a3c.py:136-169) or "cnn" (ddpg/actor.py:51-85 trunk)
    mode: str = "reference"       # "reference" | "textbook"
    features: str = "values"      # "values" (raw tiles, a3c.py:139) | "exponents"
    seed: int = 0
    update_chunk: int = 25        # time steps per forward/backward chunk of the update
    bf16: bool = False            # run the net's GEMMs in bf16 (MFMA, fp32 accumulate)
    fused_policy: bool = True     # cnn + bf16: rollout inference in one fused MFMA kernel (r48_policy.hip)
    fused_update: bool = True     # cnn + bf16: the whole update's gradient in one fused pass (r48_a3c_train.hip)
    fused_rollout: bool = True    # cnn + bf16: all max_steps policy + env steps in one launch (r48_cnn_rollout)
    rollout_values: bool = True   # fused rollout, reference loss: V(s_t) written by the rollout (no value pass)


class A3CTrainer:
    def __init__(self, cfg, device="cuda", group=None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_available() and dist.is_initialized() else 0
        n, T = cfg.n_boards, cfg.max_steps
        self.gid0 = self.rank * n
        self.env = VecGame(n, device=self.device, seed=cfg.seed, board_offset=self.gid0)
        torch.manual_seed(cfg.seed)
        self.net = make_net(cfg.net, bf16=cfg.bf16).to(self.device)
        self.flat = FlatParams(self.net)
        self.flat.broadcast_(0, group)
        self.opt = RMSPropTF1(self.flat, lr=cfg.lr)
        self.boards = torch.zeros((T + 1, n, 16), dtype=torch.int8, device=self.device)
        self.actions = torch.zeros((T, n), dtype=torch.int8, device=self.device)
        self.done = torch.zeros((T, n), dtype=torch.uint8, device=self.device)
        self.rewards = torch.zeros((T, n), dtype=torch.float32, device=self.device)
        self.sample_ctr = 0
        self.updates = 0
        # weight epoch: rollout() starts one (the weights may have been set from outside since the
        # last step), the optimizer step of update() ends it; the kernels' packed weight images are
        # made once per epoch (_packed)
        self._wepoch = 0
        self._packs = {}
        self._rollout_v = None       # ([T + 1, n] V(boards[t]) slab of the last megakernel rollout, updates)
        self._mask = None            # [T, n] valid-step mask of the last rollout, formed on first use
        # before the first rollout every step is valid (a full-length segment for every board)
        self.lengths = torch.full((n,), T, dtype=torch.int32, device=self.device)

    # ------------------------------------------------------------------ helpers
    def _features(self, boards):
        x = K.board_features(boards.reshape(-1, 16), exponents=self.cfg.features == "exponents")
        return x

    def _net(self, x):
        return self.net(x)  # bf16 (MFMA) or fp32 compute per cfg.bf16; outputs fp32

    # ------------------------------------------------------------------ rollout (a3c.py:194-212)
    def _packed(self, kind):
        """The packed weight image `kind` ("cnn": pack_cnn, "cnn_train": pack_cnn_train, "mlp":
        pack_mlp) of the current weights, made once per weight epoch."""
        c = self._packs.get(kind)
        if c is None or c[0] != self._wepoch:
            if kind == "cnn":
                v = pack_cnn(self.net)
            elif kind == "cnn_train":
                from .fused import pack_cnn_train
                v = pack_cnn_train(self.net)
            else:
                from .fused import pack_mlp
                v = pack_mlp(self.net, out=c[1] if c is not None else None)
            c = self._packs[kind] = (self._wepoch, v)
        return c[1]

    @torch.no_grad()
    def rollout(self):
        cfg, env = self.cfg, self.env
        self._wepoch += 1
        env.reset()
        self._rollout_v = None
        merge = cfg.mode == "textbook"
        if not merge:
            self.rewards.zero_()  # GameClient.py:138: reward is always 0
        fused = cfg.net == "cnn" and cfg.bf16 and cfg.fused_policy
        if fused:
            wfrag, bias = self._packed("cnn")   # weights are fixed for the whole rollout
        mlp_mega = self._mlp_fused() and cfg.fused_rollout
        mega = (fused and cfg.fused_rollout) or mlp_mega
        if merge and not mega and getattr(self, "_rewards_i32", None) is None:
            self._rewards_i32 = torch.zeros((cfg.max_steps, cfg.n_boards), dtype=torch.int32, device=self.device)
        if mlp_mega:   # the reference MLP: every step of every board in one launch (r48_mlp_rollout)
            self._rollout_megakernel(None, None, merge, mlp=True)
        elif mega:   # every step of every board in one persistent kernel (writes fp32 rewards itself)
            self._rollout_megakernel(wfrag, bias, merge)
        elif fused:   # per step: board -> CNN -> softmax -> Philox draw in one kernel, then the env kernel
            self._rollout_fused(wfrag, bias, merge)
        else:
            for t in range(cfg.max_steps):
                self.boards[t].copy_(env.boards)
                logits, _ = self._net(self._features(env.boards))
                act, _, _ = K.sample_actions(logits.contiguous(), cfg.seed, self.sample_ctr, gid0=self.gid0)
                self.actions[t].copy_(act)
                self.sample_ctr += 1
                # done (and the merge reward) land in the trajectory rows directly
                env.step(act, merge_reward=merge, done_out=self.done[t],
                         reward_out=self._rewards_i32[t] if merge else None)
        if merge and not mega:
            self.rewards.copy_(self._rewards_i32)     # one int32 -> fp32 pass for the whole rollout
        # segment length: through the first done step, else max_steps (a3c.py:201)
        if mega:                                       # the megakernel wrote boards[T] and the lengths
            self.lengths = self._lengths
            last = (self.lengths.long() - 1).view(1, -1)
            self.finished = self.done.gather(0, last)[0].bool()
        else:
            self.boards[cfg.max_steps].copy_(env.boards)
            notdone = (self.done.cumsum(0) == 0)
            self.lengths = (notdone.sum(0) + 1).clamp(max=cfg.max_steps).to(torch.int32)
            self.finished = self.done.bool().any(0)
        self._mask = None              # [T, n] valid-step mask, formed on first use (the fused update
        return self.lengths            # reads the lengths instead)

    @property
    def mask(self):
        if self._mask is None:
            t = torch.arange(self.cfg.max_steps, device=self.device).unsqueeze(1)
            self._mask = t < self.lengths.unsqueeze(0)
        return self._mask

    def _rollout_fused(self, wfrag, bias, merge):
        """The fused rollout's T steps as two raw C-ABI calls each: r48_cnn_policy_forward (CNN,
        softmax, Philox draw; writes the board snapshot boards[t] and the action actions[t]) and
        r48_env_step (reads actions[t]; writes done[t] and the merge reward). The buffers are the
        trainer's own contiguous trajectory tensors, so the per-call tensor checks of
        cnn_forward / VecGame.step are skipped: the host issues a step in a few microseconds and
        never gates the GPU (through the checked wrappers the rollout was host-bound)."""
        cfg, env = self.cfg, self.env
        lib = _lib.load()
        n = cfg.n_boards
        stream = torch.cuda.current_stream(self.device).cuda_stream
        mode = _lib.FEAT_EXPONENTS if cfg.features == "exponents" else _lib.FEAT_VALUES
        flags = _lib.MERGE_REWARD if merge else 0
        seed = int(cfg.seed) & (2 ** 64 - 1)
        bp, wp, biasp = env.boards.data_ptr(), wfrag.data_ptr(), bias.data_ptr()
        a0, b0, d0 = self.actions.data_ptr(), self.boards.data_ptr(), self.done.data_ptr()
        r0 = self._rewards_i32.data_ptr() if merge else None
        for t in range(cfg.max_steps):
            at = a0 + t * n
            _lib.check(lib.r48_cnn_policy_forward(bp, n, wp, biasp, mode, None, None, at, b0 + 16 * t * n, seed,
                                                  self.gid0, self.sample_ctr & 0xFFFFFFFF, stream))
            self.sample_ctr += 1
            _lib.check(lib.r48_env_step(env._env, at, flags, d0 + t * n, None,
                                        None if r0 is None else r0 + 4 * t * n, None, stream))

    def _mlp_fused(self):
        """The reference MLP in fp32 on the GPU runs its policy through r48_mlp.hip."""
        cfg = self.cfg
        return cfg.net == "mlp" and not cfg.bf16 and cfg.fused_policy and self.device.type == "cuda"

    def _mlp_weights(self):
        return self._packed("mlp")

    def _rollout_megakernel(self, wfrag, bias, merge, mlp=False):
        """r48_cnn_rollout (or, mlp=True, r48_mlp_rollout with the reference network): the T policy
        + env steps of every board in one launch (boards stay in registers; only the trajectory
        rows are written), bit-identical to the per-step kernels. The env's step counter then
        advances by T like T r48_env_step calls."""
        cfg, env = self.cfg, self.env
        T, n = cfg.max_steps, cfg.n_boards
        step0, resets = env.counters
        self._lengths = torch.empty(n, dtype=torch.int32, device=self.device)
        # the reference loss needs V of every training state (a3c.py:218-223): the rollout's policy
        # pass computes the value head anyway, so it writes V(boards[t]) (same arithmetic as the
        # r48_cnn_policy_forward value pass it replaces, bit for bit)
        values = None
        if cfg.mode == "reference" and cfg.rollout_values:
            if getattr(self, "_v_buf", None) is None:   # row T: V(boards[T]), filled by the update
                self._v_buf = torch.empty((T + 1, n), dtype=torch.float32, device=self.device)
            values = self._v_buf
        lib = _lib.load()
        mode = _lib.FEAT_EXPONENTS if cfg.features == "exponents" else _lib.FEAT_VALUES
        if mlp:
            call = lambda *rest: lib.r48_mlp_rollout(env.boards.data_ptr(), n, T, self._mlp_weights().data_ptr(),  # noqa: E731
                                                     mode, *rest)
        else:
            call = lambda *rest: lib.r48_cnn_rollout(env.boards.data_ptr(), n, T, wfrag.data_ptr(),  # noqa: E731
                                                     bias.data_ptr(), mode, *rest)
        _lib.check(call(
            self.boards.data_ptr(), self.actions.data_ptr(), self.done.data_ptr(),
            self.rewards.data_ptr() if merge else None, self._lengths.data_ptr(),
            None if values is None else values.data_ptr(), int(cfg.seed) & (2 ** 64 - 1), self.gid0,
            self.sample_ctr & 0xFFFFFFFF, int(env.seed) & (2 ** 64 - 1), step0,
            _lib.MERGE_REWARD if merge else 0, torch.cuda.current_stream(self.device).cuda_stream))
        self.sample_ctr += T
        env.counters = (step0 + T, resets)
        if values is not None:
            self._rollout_v = (values, self.updates)   # valid while the weights are those of this rollout

    # ------------------------------------------------------------------ update (a3c.py:218-234)
    def _states(self):
        T = self.cfg.max_steps
        return self.boards[1:T + 1] if self.cfg.mode == "reference" else self.boards[0:T]

    def update(self):
        cfg = self.cfg
        T, n = cfg.max_steps, cfg.n_boards
        states = self._states()
        # pass 1: values of the training states and the bootstrap V(s_last) (a3c.py:218-223)
        fused = cfg.net == "cnn" and cfg.bf16 and cfg.fused_policy
        with torch.no_grad():
            if fused:   # values of all T*n training states in one fused MFMA launch
                wfrag, bias = self._packed("cnn")
                value = lambda b: cnn_forward(b.reshape(-1, 16), wfrag, bias, exponents=cfg.features == "exponents",
                                              logits=False, value=True)[1]
            elif self._mlp_fused():   # the reference MLP: one fp32 VALU launch (r48_mlp_policy_forward)
                from .fused import mlp_forward
                w = self._mlp_weights()
                value = lambda b: mlp_forward(b.reshape(-1, 16).contiguous(), w,  # noqa: E731
                                              exponents=cfg.features == "exponents", logits=False, value=True)[1]
            else:
                value = lambda b: self._net(self._features(b))[1]
            # the fused textbook update computes td = target - V(s) in-kernel and needs no
            # per-segment td_sum, so only the reference loss (or the unfused path) pays this pass
            fused_upd = cfg.fused_update and (fused or self._mlp_fused())
            need_values = not (fused_upd and cfg.mode == "textbook")
            v_all = None
            rv = self._rollout_v
            v_T = None   # V(boards[T])
            if need_values and rv is not None and rv[1] == self.updates and cfg.mode == "reference":
                # V(boards[t]) from the rollout (rows 0..T-1 of a [T + 1, n] slab); the reference
                # states are boards[1..T], so V(boards[T]) -- never a rollout input -- takes one
                # forward into row T and the values are the view of rows 1..T (no copy)
                rv[0][T] = value(self.boards[T]).view(n)
                v_all = rv[0][1:T + 1]
                v_T = rv[0][T]
            elif need_values:
                v_all = torch.empty((T, n), dtype=torch.float32, device=self.device)
                ch = T if (fused or self._mlp_fused()) else cfg.update_chunk   # no activations kept
                for t0 in range(0, T, ch):
                    t1 = min(T, t0 + ch)
                    v_all[t0:t1] = value(states[t0:t1].contiguous()).view(t1 - t0, n)
            # the bootstrap V(s_last) (a3c.py:218-223) counts only for segments that did not finish,
            # and such a segment ran all T steps: its last post-step state is boards[T] (= boards[len]
            # for every board that needs it; no gather, and in reference mode the row-T value above)
            if v_T is None:
                v_T = value(self.boards[T]).view(n)
            boot = torch.where(self.finished, torch.zeros_like(v_T), v_T).float().contiguous()
            if fused_upd:
                # returns, per-board loss weights and (reference loss) action counts in ONE launch
                # (r48_a3c_segments): the fused kernels expand the weights per row themselves
                ref = cfg.mode == "reference"
                targets, seg, counts = K.segments(self.rewards, self.lengths, boot, cfg.gamma, drop_last=ref,
                                                  values=v_all if ref else None,
                                                  actions=self.actions if ref else None)
                stats = {"seg": seg, "counts": counts}
            else:
                targets = K.discounted_returns(self.rewards, self.lengths, boot, cfg.gamma,
                                               drop_last=cfg.mode == "reference")
                if self.actions.is_cuda:    # one launch (r48_a3c_segment_stats) for the masked sums + counts
                    stats = K.segment_stats(self.actions, self.lengths, v_all, None if v_all is None else targets)
                elif v_all is not None:
                    stats = segment_stats(v_all, targets, self.actions, self.mask)
                else:
                    stats = {"B": self.mask.float().sum(0).clamp(min=1.0)}
        if fused_upd:
            # pass 2 as ONE fused kernel over all T x n states (no activation hits HBM): MFMA for the
            # CNN (r48_a3c_train.hip), fp32 MFMA + VALU for the reference MLP (r48_mlp_train.hip)
            actor, critic = self._fused_gradient(states, targets, stats)
            # the reported scalars ride the gradient's all-reduce (one collective): every rank
            # reports the whole job's means, which equal a one-rank trainer's over the union of shards
            rep = self.flat.allreduce_grad(self.group, torch.stack([
                actor.float(), critic.float(), self.lengths.float().mean(), self.finished.float().mean()]))
            self.opt.step()
            self.updates += 1
            self._wepoch += 1
            a, c, ml, fin = rep.tolist()   # ONE device-to-host transfer (one synchronisation)
            return {"actor_loss": a, "critic_loss": c, "mean_length": ml, "finished": fin}
        # pass 2: chunked forward/backward, gradients accumulate in the flat buffer
        self.flat.zero_grad()
        actor_total = critic_total = torch.zeros((), dtype=torch.float32, device=self.device)
        for t0 in range(0, T, cfg.update_chunk):
            t1 = min(T, t0 + cfg.update_chunk)
            logits, v = self._net(self._features(states[t0:t1]))
            actor, critic = chunk_loss(logits.view(t1 - t0, n, 4), v.view(t1 - t0, n), self.actions[t0:t1],
                                       targets[t0:t1], self.mask[t0:t1], stats, mode=cfg.mode, beta=cfg.beta)
            (actor + critic).backward()
            actor_total = actor_total + actor.detach().float()
            critic_total = critic_total + critic.detach().float()
        # RCCL across GPUs (a3c.py:79-80's push, synchronous); the reported scalars ride along
        rep = self.flat.allreduce_grad(self.group, torch.stack([
            actor_total, critic_total, self.lengths.float().mean(), self.finished.float().mean()]))
        self.opt.step()                        # fused TF1 RMSProp (a3c.py:264-265)
        self.updates += 1
        self._wepoch += 1
        a, c, ml, fin = rep.tolist()
        return {"actor_loss": a, "critic_loss": c, "mean_length": ml, "finished": fin}

    def _fused_gradient(self, states, targets, stats):
        """Per-row weights of losses.chunk_loss for r48_cnn_train_grad: wn = mask / (B n) and, in
        reference mode, cm = (td_sum / (4 B^2)) mask / n with the per-segment action counts;
        the kernel's gradient lands in the flat gradient buffer (parameters() order)."""
        from .fused import cnn_train_grad
        cfg = self.cfg
        n = cfg.n_boards
        ref = cfg.mode == "reference"
        if "seg" in stats:   # per-board weights (r48_a3c_segments): no [T][n] weight rows
            wn = cm = None
            seg, counts = stats["seg"], stats["counts"]
        else:
            # wn = mask / (B n), cm = (td_sum / (4 B^2)) mask / n as one launch (r48_a3c_row_weights)
            wn, cm = K.row_weights(self.lengths, stats["B"].contiguous(), cfg.max_steps,
                                   stats["td_sum"].contiguous() if ref else None)
            seg, counts = None, stats["counts"].float().contiguous() if ref else None
        if self._mlp_fused():
            from .fused import mlp_train_grad
            rows = states.numel() // 16
            if getattr(self, "_mlp_ws", None) is None or self._mlp_ws[0] != rows:   # its size grows with rows
                self._mlp_ws = (rows, torch.empty(int(_lib.load().r48_mlp_train_workspace_floats(rows)),
                                                  dtype=torch.float32, device=self.device))
            g, actor, critic = mlp_train_grad(
                self.net, states.reshape(-1, 16), self.actions.reshape(-1), targets.reshape(-1).contiguous(),
                None if wn is None else wn.view(-1), None if cm is None else cm.view(-1), counts, beta=cfg.beta,
                exponents=cfg.features == "exponents", n_boards=n, w=self._mlp_weights(), workspace=self._mlp_ws[1],
                seg=seg)
            self.flat.grad.copy_(g)
            return actor, critic
        if getattr(self, "_train_ws", None) is None:
            self._train_ws = torch.empty(_lib_workspace_floats(), dtype=torch.float32, device=self.device)
        grads, actor, critic = cnn_train_grad(
            self.net, states.reshape(-1, 16), self.actions.reshape(-1), targets.reshape(-1).contiguous(),
            None if wn is None else wn.view(-1), None if cm is None else cm.view(-1), counts, beta=cfg.beta,
            exponents=cfg.features == "exponents", n_boards=n, packed=self._packed("cnn_train"),
            workspace=self._train_ws, seg=seg)
        with torch.no_grad():
            for p, g in zip(self.net.parameters(), grads):
                p.grad.copy_(g.view_as(p))
        return actor, critic

    def train_step(self):
        self.rollout()
        return self.update()

    def policy(self, seed=0x5A3C):
        """The current policy as `policy(boards int8 [n, 16], t) -> actions int8 [n]` (choose_action,
        a3c.py:89-93: a draw from the softmax; Philox keyed by (seed, board, t)) for
        evaluate.play_episodes. Weights are packed once, at the call."""
        cfg = self.cfg
        exps = cfg.features == "exponents"
        if cfg.net == "cnn" and cfg.bf16 and cfg.fused_policy:
            wfrag, bias = pack_cnn(self.net)
            return lambda boards, t: cnn_forward(boards, wfrag, bias, exponents=exps, logits=False, value=False,
                                                 actions=True, seed=seed, ctr=t)[2]
        if self._mlp_fused():
            from .fused import mlp_forward, pack_mlp
            w = pack_mlp(self.net)
            return lambda boards, t: mlp_forward(boards, w, exponents=exps, logits=False, value=False, actions=True,
                                                 seed=seed, ctr=t)[2]

        def act(boards, t):
            with torch.no_grad():
                logits, _ = self._net(self._features(boards))
            return K.sample_actions(logits.float().contiguous(), seed, t)[0]
        return act

    def scores(self):
        """a3c.py:214 SCORE: tile sum of each segment's final state."""
        return self.env.score()
