"""DQN around the vectorized env with an HBM-resident replay ring (BASELINE config 5).

No reference trainer exists (the reference's value-based code is the unfinished DDPG under
algorithm/ddpg/; its replay buffer, replay.py, is what ReplayStore's fill_drain mode restates).
One train_step per env step, per GPU:
  act      Q = ResNet10Q(boards) in eval mode + epsilon-greedy (Philox keyed by global board
           id) in ONE fused bf16 MFMA kernel (r48_resnet_q_forward; weights repacked with BN
           folded after every update), or the PyTorch structured-GEMM net + r48_egreedy_actions
  step     r48_env_step with the opt-in merge reward (the reference reward is always 0,
           GameClient.py:138, which gives a value learner nothing to learn) and auto-reset
  store    (s, a, r, s', done) of every board into the ring (r48_replay_store; 38 B each).
           For a done board s' is the auto-reset board: the target masks it, (1 - done)
  update   `updates_per_step` minibatches sampled uniformly from the ring, TD target from the
           target net (double DQN by default; r48_td_target), Huber loss, ONE all-reduce of
           the flat fp32 gradient across GPUs (RCCL), Adam, ONE all-reduce-mean of the BN
           running statistics (so the eval-mode nets, whose BN is folded into the acting
           kernel's weights, stay identical on every rank); target net synced every
           `target_sync` updates
Rewards enter the loss as log2(1 + merged value) (reward_transform="log2") or raw.
Each rank owns boards [rank*N, (rank+1)*N) and its own ring shard; no replay traffic crosses
GPUs.
"""
import copy
import ctypes as C
import math
from dataclasses import dataclass

import torch
import torch.distributed as dist
import torch.nn.functional as F

from ..a3c.optim import FlatBuffers, FlatParams
from ..env import VecGame
from ..replay import ReplayStore
from .kernels import board_onehot, egreedy_actions, td_target
from .nets import ResNet10Q


@dataclass
class DQNConfig:
    n_boards: int = 4096             # boards per GPU
    replay_capacity: int = 1 << 20   # transitions per GPU (38 B each)
    batch: int = 4096                # minibatch per GPU per update
    updates_per_step: int = 1
    learn_start: int = 16384         # transitions held before the first update
    gamma: float = 0.99
    lr: float = 1e-4
    eps_start: float = 1.0
    eps_end: float = 0.05
    eps_decay_steps: int = 1000
    target_sync: int = 250
    double: bool = True
    reward_transform: str = "log2"
    channels: int = 64
    blocks: int = 4
    bn: bool = True
    bf16: bool = True
    act_chunk: int = 1 << 18         # boards per Q forward while acting (PyTorch path)
    fused: bool = True               # eval-mode Q through r48_resnet_q_forward (bf16, C=64, 4 blocks)
    fused_step: bool = True          # training step through train_step.ResNetTrainStep (bf16 GPU, C=64)
    seed: int = 0


class Adam:
    """torch.optim.Adam semantics over one flat fp32 buffer (bias-corrected, eps outside sqrt)."""

    def __init__(self, flat, lr, betas=(0.9, 0.999), eps=1e-8):
        self.flat, self.lr, self.b1, self.b2, self.eps = flat, lr, betas[0], betas[1], eps
        self.m = torch.zeros_like(flat.data)
        self.v = torch.zeros_like(flat.data)
        self.t = 0

    @torch.no_grad()
    def step(self):
        self.t += 1
        g = self.flat.grad
        p = self.flat.data
        if p.is_cuda and p.dtype == torch.float32 and p.numel() % 4 == 0 and g.is_contiguous():
            # one fused launch (r48_adam) instead of the ~8 elementwise launches below
            from .. import _lib
            from .._lib import check, ptr
            check(_lib.load().r48_adam(ptr(p), ptr(g), ptr(self.m), ptr(self.v), p.numel(), float(self.lr),
                                       float(self.b1), float(self.b2), float(self.eps), self.t,
                                       C.c_void_p(torch.cuda.current_stream(p.device).cuda_stream)))
            return
        self.m.mul_(self.b1).add_(g, alpha=1 - self.b1)
        self.v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
        c1, c2 = 1 - self.b1 ** self.t, 1 - self.b2 ** self.t
        denom = (self.v / c2).sqrt_().add_(self.eps)
        self.flat.data.addcdiv_(self.m, denom, value=-self.lr / c1)


class DQNLearner:
    """The data-parallel learning half of DQN: online and target ResNet-10, flat parameters and
    gradient (one all-reduce), Adam, the BN running statistics as one flat buffer (one
    all-reduce-mean per update). Device-agnostic -- tests/test_dqn.py runs two gloo ranks of it on
    the CPU; DQNTrainer adds the GPU env, the replay ring and the fused kernels."""

    def __init__(self, cfg: DQNConfig, device="cuda:0"):
        self.cfg = cfg
        self.device = torch.device(device)
        self.rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        torch.manual_seed(cfg.seed)                       # identical init on every replica
        dt = torch.bfloat16 if cfg.bf16 else torch.float32
        self.net = ResNet10Q(cfg.channels, cfg.blocks, cfg.bn, dtype=dt).to(self.device)
        self.flat = FlatParams(self.net)
        self.bn_buffers = FlatBuffers(self.net)
        self.flat.broadcast_()                            # rank 0's replica everywhere
        self.bn_buffers.broadcast_()
        self.target = copy.deepcopy(self.net).eval()
        for p in self.target.parameters():
            p.requires_grad_(False)
        self.opt = Adam(self.flat, cfg.lr)
        self._train_step = None                           # train_step.ResNetTrainStep, built on first use
        self._grad_overwritten = False                    # the last step was the fused one (learn)
        self.updates = 0
        self._version = 0                                 # bumped by every optimizer step / sync

    def learn(self, x, action, y, sync=True):
        """One synchronous step: Huber loss of Q(x)[action] against the TD target y, gradient
        averaged over the group, Adam, BN running statistics averaged over the group; the target
        net follows every `target_sync` updates. Returns {"loss", "q_mean"} as floats, or as 0-d GPU
        tensors with sync=False (the host then never waits for the GPU inside an update)."""
        self.net.train()
        fused = self._fused_step_ok(x)
        if not (fused and self._grad_overwritten):
            # the fused step WRITES every parameter gradient but the conv biases' (exactly zero, never
            # written): after one zeroing, later fused steps need none (autograd accumulates: it does)
            self.flat.zero_grad()
        self._grad_overwritten = fused
        if fused:
            if self._train_step is None:
                from .train_step import ResNetTrainStep
                self._train_step = ResNetTrainStep(self.net)
            loss, q_mean = self._train_step(x, action, y)
        else:
            q = self.net(x)
            q_sa = q.gather(1, action.long().view(-1, 1)).squeeze(1)
            loss = F.smooth_l1_loss(q_sa, y)
            loss.backward()
            q_mean = q_sa.detach().mean()
        self.flat.allreduce_grad()
        self.opt.step()
        self.bn_buffers.allreduce_mean_()
        self._version += 1
        self.updates += 1
        if self.updates % self.cfg.target_sync == 0:
            self.sync_target()
        if not sync:
            return {"loss": loss.detach(), "q_mean": q_mean.detach()}
        lq = torch.stack([loss.detach().float(), q_mean.detach().float()]).tolist()   # one device-to-host copy
        return {"loss": lq[0], "q_mean": lq[1]}

    def _fused_step_ok(self, x):
        """The explicit fused step (train_step.py) takes the bf16 GPU net with the custom convs and
        the padded 32-plane input; everything else goes through autograd."""
        if not (self.cfg.fused_step and x.is_cuda and x.dim() == 2 and x.shape[1] == 16 * 32
                and getattr(self.net, "custom_conv", False)):
            return False
        from .train_step import supported
        return supported(self.net)

    def sync_target(self):
        self.target.load_state_dict(self.net.state_dict())
        self._version += 1


class DQNTrainer(DQNLearner):
    def __init__(self, cfg: DQNConfig, device="cuda:0"):
        super().__init__(cfg, device)
        n = cfg.n_boards
        self.env = VecGame(n, device=self.device, seed=cfg.seed, board_offset=self.rank * n)
        self.env.reset()
        self.replay = ReplayStore(cfg.replay_capacity, self.device, mode="ring",
                                  seed=(cfg.seed * 0x9E3779B97F4A7C15 + self.rank + 1) & (2 ** 64 - 1))
        self.steps = 0
        self.q = torch.empty((n, 4), dtype=torch.float32, device=self.device)
        self.actions = torch.empty(n, dtype=torch.int8, device=self.device)
        self.use_fused = cfg.fused and cfg.bf16 and cfg.channels == 64 and cfg.blocks == 4
        self._packed = {}                                   # id(net) -> (version, packed weights)

    def epsilon(self):
        c = self.cfg
        f = min(1.0, self.steps / max(1, c.eps_decay_steps))
        return c.eps_start + f * (c.eps_end - c.eps_start)

    @torch.no_grad()
    def q_values(self, net, boards, out=None):
        """Q [n, 4] of int8 boards [n, 16] in eval mode, in act_chunk slices."""
        n = boards.shape[0]
        out = torch.empty((n, 4), dtype=torch.float32, device=boards.device) if out is None else out
        was = net.training
        net.eval()
        dt = torch.bfloat16 if self.cfg.bf16 else torch.float32
        for s in range(0, n, self.cfg.act_chunk):
            e = min(n, s + self.cfg.act_chunk)
            out[s:e] = net(board_onehot(boards[s:e], dtype=dt))
        net.train(was)
        return out

    def packed(self, net):
        """Fused-kernel weights of `net` (eval-mode BN folded), repacked when the weights changed."""
        from .fused import pack_resnet_gpu
        ver, p = self._packed.get(id(net), (-1, None))
        if ver != self._version:
            p = pack_resnet_gpu(net, out=p)    # one HIP launch, into the previous buffers
            self._packed[id(net)] = (self._version, p)
        return p

    @torch.no_grad()
    def q_eval(self, net, boards):
        """Eval-mode Q [n, 4] of int8 boards [n, 16]."""
        if self.use_fused:
            from .fused import resnet_q_forward
            return resnet_q_forward(boards.contiguous(), self.packed(net))[0]
        return self.q_values(net, boards)

    @torch.no_grad()
    def act(self):
        eps, gid0 = self.epsilon(), self.rank * self.cfg.n_boards
        if self.use_fused:
            from .fused import resnet_q_forward
            _, a = resnet_q_forward(self.env.boards, self.packed(self.net), q=False, actions=True, eps=eps,
                                    seed=self.cfg.seed, ctr=self.steps, gid0=gid0)
            self.actions.copy_(a)
            return self.actions
        self.q_values(self.net, self.env.boards, out=self.q)
        return egreedy_actions(self.q, eps, self.cfg.seed, self.steps, gid0=gid0, out=self.actions)

    def policy(self, eps=0.01, seed=0x5D09):
        """The online net's epsilon-greedy policy as `policy(boards, t) -> actions` (Philox keyed by
        (seed, board, t); a small eps keeps a greedy policy from repeating a move that changes
        nothing) for evaluate.play_episodes."""
        def act(boards, t):
            with torch.no_grad():
                if self.use_fused:
                    from .fused import resnet_q_forward
                    return resnet_q_forward(boards.contiguous(), self.packed(self.net), q=False, actions=True,
                                            eps=eps, seed=seed, ctr=t)[1]
                q = self.q_values(self.net, boards)
                return egreedy_actions(q, eps, seed, t)
        return act

    @torch.no_grad()
    def env_step(self):
        """act + step + store: one transition per board into the ring."""
        s = self.env.boards.clone()
        a = self.act()
        _, reward, done = self.env.step(a, auto_reset=True, merge_reward=True)
        self.replay.store(s, a, reward.float(), self.env.boards, done)
        self.steps += 1
        return reward, done

    def _reward(self, r):
        return torch.log2(1.0 + r) if self.cfg.reward_transform == "log2" else r

    def update(self, batch=None, sync=True):
        """One update from a sampled minibatch; sync=False leaves the loss and mean Q as 0-d GPU
        tensors (learn), so that nothing waits for the GPU."""
        c = self.cfg
        dt = torch.bfloat16 if c.bf16 else torch.float32
        b = self.replay.sample(batch or c.batch)
        if self.net.wants_onehot32(b["state"].device, dt):
            from .conv import board_onehot32
            x = board_onehot32(b["state"]).view(-1, 16 * 32)     # the training stem's padded planes
        else:
            x = board_onehot(b["state"], dtype=dt)
        with torch.no_grad():
            self.target.eval()
            qt = self.q_eval(self.target, b["next_state"]).contiguous()
            qo = self.q_eval(self.net, b["next_state"]).contiguous() if c.double else None
            rw = b["reward"].contiguous()
            y = td_target(rw, b["done"], qt, qo, c.gamma, log2_reward=True) if c.reward_transform == "log2" \
                else td_target(self._reward(rw), b["done"], qt, qo, c.gamma)
        out = self.learn(x, b["action"], y, sync=sync)
        out["batch"] = b
        return out

    def train_step(self, sync=True):
        reward, done = self.env_step()
        out = {"loss": math.nan}
        if len(self.replay) >= self.cfg.learn_start:
            for _ in range(self.cfg.updates_per_step):
                out = self.update(sync=sync)
        out["epsilon"] = self.epsilon()
        return out
