#!/usr/bin/env python3
"""bench.py -- env steps/sec on 4x4 boards (BASELINE.json metric), MI355X.

Workload (BASELINE.json configs[1], "1M parallel 4x4 int8 boards, random policy, env-only
throughput on 1 MI355X"): 2^20 boards per GPU, in-kernel uniform random policy (control/rand.py),
move + spawn + game-over + auto-reset every step (game/GameClient.py:40-51). Boards start from
SURVEY.md 8(d)'s synthetic fill (each cell empty w.p. 1/2, else exponent ~U{1..7}; the reference
reset start is an extra) and are resident in HBM before the timed region. The K timed steps are
r48_env_step_n calls (one k_step_n launch per call, every board in VGPRs for all the call's steps;
a call covers the whole K unless --chunk splits it), bit-identical to K single-step launches.

Multi-GPU: one process per GPU (torchrun; `--gpus N` without WORLD_SIZE launches torchrun itself
as a child process before touching the GPU), rank r owns boards [r*N, (r+1)*N) (Philox keyed by
global board id); no data-path collective. Timing: synchronize + barrier + synchronize before
exactly K steps and synchronize after them on every rank; the job's window runs from the earliest
rank's start to the latest rank's end on the node's shared monotonic clock (both all-reduced), so
barrier skew cannot shorten it; value = all boards x K / that window.

Extra objects on the JSON line:
  roofline      k_step_n is VALU-issue bound (boards in VGPRs, no memory traffic inside its step
                loop): achieved = MODELLED VALU issue cycles per board-step (the shipped loop's
                static instruction mix x measured per-instruction issue costs, plus the measured
                operand costs -- literal, inline constant -- and the SIMD's SGPR-read limit,
                tools/isa_hist.py model(); committed in profiles/<round>/pmc_k_step_n.json together
                with the hash of the kernel sources it was made from) x board-steps / the SAME wall
                time as `value` -> frac; frac_device uses the HIP-event dispatch time of the same
                region instead; frac_counter beside them is the counter-only fraction (SQ_INSTS_VALU
                per board-step at the device rate / one wave64 VALU per 2 cycles per SIMD, no cost
                model); peak = one issue cycle per SIMD per clock (1024 SIMDs x 2.4 GHz). `hbm_def` expresses the same rate in GB/s
                at SURVEY.md 8(d)'s 34 B per board-step -- not a roofline fraction: k_step_n makes
                no per-step HBM round trip; the HBM roofline point is hbm.k_step_2p26 below. If the
                committed profile's source hash
                differs from the tree's, the profile-derived fields are null and `profile_stale`
                says so. `valu_instr_rate` gives the plain instruction-rate fraction.
                `hbm` holds the single-step kernel k_step (boards through HBM every step, 34
                algorithmic bytes per board-step) at 2^20 boards (Infinity-Cache resident) and at
                2^26 (past the 256 MiB cache: the HBM point) against the 8 TB/s spec, with PMC
                traffic from the committed profiles.
  repeat_5      5 repeats of the timed region (rank 0, N=1).
  cpu_baseline  oracle/game_port.py (faithful pure-Python restatement of the reference Game + Rand,
                calibrated against the reference in BASELINE.md) on one process per available host
                CPU (at most 16, the box's share) for a bounded sample, plus the 1-process figure;
                rank 0, N=1 only (oracle/port_bench.py).
  extras        N=1: the fused random-policy rollout kernel, the reference reset start, config 3
                (A3C + CNN), config 5 per GPU (DQN + ResNet-10 + HBM replay) and the C oracle as a
                strong CPU line. N>1: config 4 (A3C, 2^20 boards per GPU) and config 5 (DQN, 2^21
                boards per GPU) on all ranks with the gradient all-reduce (--no-extras skips them).
"""
import argparse
import datetime
import json
import os
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env steps/sec (whole node), 4×4 boards, at 1/2/4/8 MI355X"
ALGO_BYTES = 34            # per board-step of k_step: 16 B board in + 16 B out + 1 B action + 1 B done
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
HBM_MEASURED_GBS = 6290.0  # float4 copy measured on MI355X (same guide)
SIMDS, CLOCK_GHZ = 1024, 2.4            # 256 CUs x 4 SIMDs; max clock (same guide)
VALU_PEAK_G = SIMDS * CLOCK_GHZ / 2.0   # G wave-instructions/s: one full-rate wave64 VALU instr per 2 cycles
VALU_ISSUE_PEAK_G = SIMDS * CLOCK_GHZ   # G VALU issue-cycles/s
PROFILE_ROUND = "r06"
PROFILE_DIR = os.path.join(ROOT, "profiles", PROFILE_ROUND)
ENV_SOURCES = ("rein48_amd/csrc/r48_env.hip", "rein48_amd/csrc/r48_board.h")


def env_source_sha16():
    """Hash of the env kernel's sources: a committed profile describes the build it was made from."""
    import hashlib
    h = hashlib.sha256()
    for p in ENV_SOURCES:
        with open(os.path.join(ROOT, p), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def shard(rank, boards_per_gpu):
    """Rank r owns global boards [r*N, (r+1)*N): weak scaling, Philox keyed by global id, so
    the union of the shards is bit-identical to one N*world env (tests/test_distributed.py)."""
    return rank * boards_per_gpu, boards_per_gpu


def max_over_ranks(x, device, world):
    """Timing aggregation: the slowest rank's elapsed time defines the job's time."""
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def chunks(total, size):
    out = [size] * (total // size)
    if total % size:
        out.append(total % size)
    return out


def cpu_baseline(seconds):
    """oracle/port_bench.py: oracle/game_port.py on P processes (one per available CPU, at most
    the box's 16-CPU share) for ~`seconds`, plus a 1-process run -- a bounded sample. Runs as a
    child process before this process initialises the GPU."""
    out = subprocess.run([sys.executable, "-m", "oracle.port_bench", "--seconds", str(seconds),
                          "--single-seconds", str(max(1.0, seconds / 2))],
                         cwd=ROOT, capture_output=True, text=True, timeout=seconds * 3 + 120)
    if out.returncode != 0:
        return {"error": out.stderr[-500:]}
    return json.loads(out.stdout.strip().splitlines()[-1])


def strong_cpu_line(seconds=2.0):
    from oracle import native as O
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        O.bench_pyrand(n + 1, 1_000_000)
        n += 1_000_000
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "env steps/s", "cores": 1, "kind": "oracle C restatement",
            "sample": "%d steps, one board, CPython-compatible MT19937 draws" % n}


def _load_profile(name):
    p = os.path.join(PROFILE_DIR, name)
    return json.load(open(p)) if os.path.exists(p) else None


SETTLE_S = 0.3   # minimum untimed stepping before a timed region: GPU clocks ramp over ~20 ms+
SYNC_POLL = False  # --sync: poll the region's last HIP event before the closing synchronize
SETTLE_SPIN = False  # --settle-spin: the settle loop polls its last event instead of sleeping in the wait
DRY_PASSES = 3  # --dry-passes: untimed passes through the region's exact host path before t0
CLOSE_DEVICE = False  # --close device: t1 after torch.cuda.synchronize() instead of the last event's wait


def _now():
    """Node-wide monotonic clock (CLOCK_MONOTONIC is shared by every process of one host)."""
    return time.clock_gettime_ns(time.CLOCK_MONOTONIC) * 1e-9


def timed_steps(env, plan, W, chunk, world, dev):
    """W untimed warm-up steps through the same path (in calls of the timed chunk size) --
    continued, still untimed, until at least SETTLE_S of stepping has run -- then exactly sum(plan)
    steps. Opening: synchronize, barrier, synchronize, t0 (per rank); closing: synchronize, t1.
    -> (window seconds = max over ranks of t1 - min over ranks of t0 on the node's monotonic clock;
    device ms of the timed calls from HIP events on the launch stream, one entry per call;
    start skew = max - min over ranks of t0)."""
    t_w = time.perf_counter()
    for c in chunks(W, chunk) if W else []:
        env.step_n(c, auto_reset=True)
    torch.cuda.synchronize(dev)
    s = torch.cuda.current_stream(dev)
    done_ev = torch.cuda.Event()
    while time.perf_counter() - t_w < SETTLE_S:
        env.step_n(chunk, auto_reset=True)
        if SETTLE_SPIN:
            done_ev.record(s)
            while not done_ev.query():
                pass
        torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in plan]
    # untimed passes through the region's exact host path (event records, the calls, the closing
    # event wait): torch creates the HIP events at their first record, which does not belong in the
    # region, and the first pass of that host path in a process runs slower than later ones (launch
    # path 7.4 vs ~5 us, tools/exp_first_region.py; profiles/r04/env/first_region_probe.txt)
    for _ in range(max(1, DRY_PASSES)):
        for (a, b), c in zip(ev, plan):
            a.record(s)
            env.step_n(c, auto_reset=True)
            b.record(s)
        ev[-1][1].synchronize()
        torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
        torch.cuda.synchronize(dev)          # the barrier's own device work done before t0
    # the first opening event is recorded before t0: on an idle stream it completes at once, so the
    # device time it brackets is the launch's own plus the launch latency (conservative), and its
    # host-side cost does not delay the launch (tools/exp_sync.py: ~1-3 us of a ~95 us region)
    ev[0][0].record(s)
    if len(plan) == 1:   # the driver's region: one call
        last = ev[0][1]
        t0 = _now()
        env.step_n(plan[0], auto_reset=True)
        last.record(s)
    else:
        t0 = _now()
        for k, ((a, b), c) in enumerate(zip(ev, plan)):
            if k:
                a.record(s)
            env.step_n(c, auto_reset=True)
            b.record(s)
    if SYNC_POLL:
        # spin on the last event instead of sleeping in the driver's blocking wait: a ~80 us
        # region otherwise measures the wake-up jitter of the waiting thread
        last = ev[-1][1]
        while not last.query():
            pass
    if CLOSE_DEVICE:
        torch.cuda.synchronize(dev)      # the device is idle: every step of every call is done
    else:
        ev[-1][1].synchronize()          # the region's last event: every step of every call is done
    t1 = _now()
    torch.cuda.synchronize(dev)
    skew = 0.0
    if world > 1:
        # one window for the node: from the earliest rank's start to the latest rank's end
        t = torch.tensor([-t0, t1, t0, -t0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t0, t1, skew = -float(t[0]), float(t[1]), float(t[2]) + float(t[3])
    return t1 - t0, [a.elapsed_time(b) for a, b in ev], skew


def single_step_hbm(dev, seed, n, launches):
    """k_step (one launch per step, boards read and written through HBM every step): per-launch
    device time from HIP events over back-to-back launches, after a settle period."""
    from rein48_amd import VecGame
    env = VecGame(n, device=dev, seed=seed)
    env.fill_random(7)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < SETTLE_S:
        env.step(None, auto_reset=True)
        torch.cuda.synchronize(dev)
    s = torch.cuda.current_stream(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(launches):
        env.step(None, auto_reset=True)
    b.record(s)
    torch.cuda.synchronize(dev)
    ms = a.elapsed_time(b) / launches
    del env
    torch.cuda.empty_cache()
    gbs = n * ALGO_BYTES / (ms * 1e-3) / 1e9
    name = "pmc_k_step_2p%d.json" % (n.bit_length() - 1)
    prof = _load_profile(name)
    if prof is not None and prof.get("source_sha16") != env_source_sha16():
        prof = None   # made from other kernel sources than the tree's
    out = {"kernel": "k_step<RANDOM=1,AUTO_RESET=1,REWARD=0>", "boards": n, "launch_ms": ms,
           "env_steps_per_s": n / (ms * 1e-3), "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": gbs / HBM_PEAK_GBS, "frac_of_measured_copy_ceiling": gbs / HBM_MEASURED_GBS,
           "algorithmic_bytes_per_launch": n * ALGO_BYTES,
           "traffic": prof.get("hbm_bytes_per_launch") if prof else None,
           "traffic_source": ("profiles/%s/%s (committed rocprofv3 FETCH_SIZE + WRITE_SIZE passes, not "
                              "measured in this run)" % (PROFILE_ROUND, name)) if prof else None}
    if n * ALGO_BYTES < 256 * 2 ** 20:
        out["bound"] = "mall"
        out["note"] = ("%d MB per step stays in the 256 MiB Infinity Cache: a cache-resident rate, not HBM; the "
                       "2^26-board entry is the HBM point" % (n * ALGO_BYTES // 10 ** 6))
    else:
        out["bound"] = "hbm"
    return out


def roofline_step_n(n, wall_s, dev_ms, steps):
    """VALU roofline of k_step_n (boards stay in VGPRs for all steps of a call: no memory traffic
    inside the step loop). Work = MODELLED VALU issue cycles: the shipped loop's static instruction
    mix x each instruction's measured issue cost (modelled_cycles_per_board_step, profiles/<round>/
    pmc_k_step_n.json, made by tools/make_profiles.py from build/r48_env.s and the instruction-rate
    table); peak = one issue cycle per SIMD per clock (1024 SIMDs x 2.4 GHz). frac uses the same
    wall time as `value`, frac_device the HIP-event dispatch time of the region, frac_trace the
    committed kernel trace of the driver's command. hbm_def: the same board-step rate expressed as
    GB/s at 34 B per board-step -- an equivalent rate, not a roofline fraction (the
    HBM roofline point is the single-step kernel at 2^26 boards, roofline.hbm.k_step_2p26).
    Profile-derived fields are null when the profile was made from other kernel sources than the
    tree's (profile_stale)."""
    prof = _load_profile("pmc_k_step_n.json")
    trace = _load_profile("roofline_from_trace.json")
    sha = env_source_sha16()
    stale = prof is None or prof.get("source_sha16") != sha
    bsteps = n * steps
    rate_wall = bsteps / wall_s
    rate_dev = bsteps / (dev_ms * 1e-3)
    hbm = {"bytes_per_board_step": ALGO_BYTES, "equivalent_gbs": rate_wall * ALGO_BYTES / 1e9,
           "note": "SURVEY.md 8(d)'s 34 B per board-step priced at the wall rate of `value`: NOT a fraction of the HBM "
                   "roofline -- k_step_n reads and writes each board once per call (no per-step HBM round trip), so "
                   "the kernel is VALU-bound, not HBM-bound. The HBM roofline point is roofline.hbm.k_step_2p26 "
                   "(one step per launch through HBM, 2^26 boards past the Infinity Cache)"}
    out = {"bound": "valu", "unit": "G VALU issue-cycles/s", "peak": VALU_ISSUE_PEAK_G,
           "achieved": None, "frac": None, "frac_device": None, "achieved_is": "modelled",
           "hbm_def": hbm, "board_steps_timed": bsteps, "wall_ms_timed": wall_s * 1e3, "device_ms_timed": dev_ms,
           "kernel": "k_step_n<RANDOM=1,AUTO_RESET=1,REWARD=0> (board pair per lane in VGPRs for all steps of the "
                     "call, line-form orientation tracking)",
           "source_sha16": sha, "profile": "profiles/%s/pmc_k_step_n.json" % PROFILE_ROUND,
           "profile_stale": stale, "traffic": None}
    if stale:
        return out
    cyc, per = prof["modelled_cycles_per_board_step"], prof["valu_wave_instr_per_board_step"]
    out.update({
        "achieved": cyc * rate_wall / 1e9, "frac": cyc * rate_wall / 1e9 / VALU_ISSUE_PEAK_G,
        "frac_device": cyc * rate_dev / 1e9 / VALU_ISSUE_PEAK_G,
        # beside the modelled fraction: the counter-only one (SQ_INSTS_VALU per board-step at this run's
        # device rate / one wave64 VALU per 2 cycles per SIMD), no cost model in it
        "frac_counter": per * rate_dev / 1e9 / VALU_PEAK_G,
        "traffic": prof["hbm_bytes_per_dispatch"] * n / prof["boards"],
        "traffic_unit": "bytes per launch (HBM/fabric; the boards are read and written once per call)",
        "traffic_source": "profiles/%s/pmc_k_step_n.json: rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE passes of a 2^20-board "
                          "K=%d dispatch (committed profile; scaled to this run's boards)"
                          % (PROFILE_ROUND, prof.get("steps_per_dispatch", 20)),
        "issue_cycles_per_board_step": cyc,
        "issue_cycles_source": "build/r48_env.s hot loop (tools/isa_hist.py model(): opcode costs of "
                               "profiles/r02/instr_rate.txt + literal / inline-constant costs and the SGPR-read "
                               "bound of profiles/r05/env/instr_rate_r05.txt)",
        "opcode_only_cycles_per_board_step": prof.get("opcode_only_cycles_per_board_step"),
        "valu_wave_instr_per_board_step": per,
        "valu_instr_rate": {"achieved": per * rate_dev / 1e9, "peak": VALU_PEAK_G, "unit": "G VALU wave-instr/s",
                            "frac": per * rate_dev / 1e9 / VALU_PEAK_G,
                            "note": "SQ_INSTS_VALU per board-step (PMC) at the device rate; peak = one wave64 "
                                    "instruction per 2 cycles per SIMD (half-rate instructions take ~4.3)"}})
    if trace is not None and trace.get("source_sha16") == sha:
        out["frac_trace"] = trace["frac"]
        out["frac_trace_source"] = "profiles/%s/roofline_from_trace.json (median k_step_n dispatch of the traced " \
                                   "driver command)" % PROFILE_ROUND
    return out


def extras(dev, seed, n_small):
    from rein48_amd import VecGame
    out = {}
    # fused rollout: K steps per launch with the per-step trajectory (action, done) written
    env = VecGame(n_small, device=dev, seed=seed)
    env.reset()
    K = 64
    acts = torch.empty((K, n_small), dtype=torch.int8, device=dev)
    dn = torch.empty((K, n_small), dtype=torch.uint8, device=dev)
    env.rollout(K, actions=acts, done=dn)
    s = torch.cuda.current_stream(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    a.record(s)
    for _ in range(reps):
        env.rollout(K, actions=acts, done=dn)
    b.record(s)
    torch.cuda.synchronize(dev)
    ms = a.elapsed_time(b) / reps
    out["rollout_fused"] = {"boards": n_small, "steps_per_launch": K, "kernel_ms": ms,
                            "env_steps_per_s": n_small * K / (ms * 1e-3),
                            "note": "r48_env_rollout (k_step_n with trajectory rows): boards stay in VGPRs for K "
                                    "steps; writes action+done per step (2 B) and the board once per launch"}
    return out


def _sync_max(ms_list, dev, world):
    """Per-phase mean device time (ms), max over ranks (the slowest replica sets the pace)."""
    return max_over_ranks(sum(ms_list) / len(ms_list), dev, world)


def _allreduce_label(world):
    if world <= 1:
        return None
    b = dist.get_backend()
    return "%s all_reduce(SUM)/world" % ("RCCL (torch backend 'nccl')" if b == "nccl" else "torch backend '%s'" % b)


def a3c_config3(dev, seed, n_boards, updates=3, world=1, mode="textbook", features="exponents", warmup=2,
                net="cnn", bf16=True):
    """BASELINE configs[2] (world 1: 2^20 boards + 2-layer CNN policy on 1 MI355X) and configs[3]
    (world > 1: 2^20 boards per GPU, 8M boards on 8 GPUs, one all-reduce of the flat fp32
    gradient per update): A3C rollout (MAX_STEP_NUM = 100 steps: fused CNN inference + softmax +
    Philox sampling -> env kernel) and the synchronous update (fused MFMA gradient pass,
    all-reduce, TF1 RMSProp kernel). mode "reference" + features "values" is what a user of the
    reference gets (raw tile values in, a3c.py:37-39,139; post-step states, reward 0, dropped last
    reward and the literal [B,B,4]-broadcast actor loss, a3c.py:99-123,187-256); "textbook" +
    "exponents" is the build's learning-oriented variant. net "mlp" + bf16 False is the reference's
    own network (a3c.py:136-169, fp32) at the same size."""
    from rein48_amd.a3c import A3CConfig, A3CTrainer
    cfg = A3CConfig(n_boards=n_boards, max_steps=100, mode=mode, net=net, bf16=bf16,
                    features=features, seed=seed, update_chunk=10)
    tr = A3CTrainer(cfg, device=dev)
    for _ in range(warmup):                           # warm-up (allocator, kernels, first collective, clocks)
        tr.train_step()
    s = torch.cuda.current_stream(dev)
    roll_ms, upd_ms, steps = [], [], 0
    for _ in range(updates):
        a, b, c = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        a.record(s)
        tr.rollout()
        b.record(s)
        out = tr.update()                             # includes the gradient all-reduce when world > 1
        c.record(s)
        torch.cuda.synchronize(dev)
        roll_ms.append(a.elapsed_time(b))
        upd_ms.append(b.elapsed_time(c))
        steps += int(tr.lengths.sum())
    r, u = _sync_max(roll_ms, dev, world), _sync_max(upd_ms, dev, world)
    board_steps = world * n_boards * cfg.max_steps  # every board is stepped every rollout step
    lab = _allreduce_label(world)
    return {"boards": world * n_boards, "boards_per_gpu": n_boards, "n_gpus": world,
            "net": ("cnn (conv2x2x32, conv2x2x64, heads 256->4/1)" if net == "cnn" else
                    "mlp (a3c.py:136-169: 16->64 ReLU6->4 ReLU softmax, 16->64 ReLU6->1)")
                   + (", bf16" if bf16 else ", fp32"), "mode": mode, "features": features,
            "gradient_allreduce": ("%s of %d fp32 per update" % (lab, tr.flat.grad.numel())) if lab else None,
            "rollout_ms": r, "update_ms": u,
            "rollout_env_steps_per_s": board_steps / (r * 1e-3),
            "train_env_steps_per_s": board_steps / ((r + u) * 1e-3),
            "valid_segment_steps_per_update": steps / updates, "warmup_updates": warmup, "timed_updates": updates,
            "last_losses": {k: out[k] for k in ("actor_loss", "critic_loss")}}


def dqn_config5(dev, seed, n_boards, steps=5, world=1, warmup=3):
    """BASELINE configs[4] (16M boards over 8 GPUs = 2^21 per GPU): ResNet-10 Q-network in bf16
    (fused MFMA inference kernel for acting, hand-written training step: dqn/train_step.py), epsilon-greedy acting
    on every board, env step with merge reward + auto-reset, (s, a, r, s', done) of every board
    into the HBM replay ring, one 64K-transition double-DQN update per env step (gradient and BN
    running statistics all-reduced when world > 1; each rank samples its own ring shard)."""
    from rein48_amd.dqn import DQNConfig, DQNTrainer
    cfg = DQNConfig(n_boards=n_boards, replay_capacity=1 << 25, batch=1 << 16, learn_start=1, seed=seed,
                    act_chunk=1 << 18)
    tr = DQNTrainer(cfg, device=dev)
    # warm-up: allocator, packing caches, clocks; the first acts after start-up run 10-25 % slow
    # (tools/probe_act2.py: 11.0, 9.8, 9.2, then 8.9-9.2 ms per 2^21-board act)
    for _ in range(warmup):
        tr.train_step()
    s = torch.cuda.current_stream(dev)
    act, env, upd = [], [], []
    for _ in range(steps):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        e[0].record(s)
        st = tr.env.boards.clone()
        a = tr.act()
        e[1].record(s)
        _, reward, done = tr.env.step(a, auto_reset=True, merge_reward=True)
        tr.replay.store(st, a, reward.float(), tr.env.boards, done)
        tr.steps += 1
        e[2].record(s)
        out = tr.update(sync=False)                   # the loss stays on the GPU: no host wait inside
        e[3].record(s)
        torch.cuda.synchronize(dev)
        act.append(e[0].elapsed_time(e[1]))
        env.append(e[1].elapsed_time(e[2]))
        upd.append(e[2].elapsed_time(e[3]))
    a_ms, e_ms, u_ms = (_sync_max(x, dev, world) for x in (act, env, upd))
    C = cfg.channels
    useful = 2 * 100 * (18 * C + 2 * cfg.blocks * C * C) + 2 * 16 * C * 4     # valid taps only
    lab = _allreduce_label(world)
    return {"boards": world * n_boards, "boards_per_gpu": n_boards, "n_gpus": world,
            "net": "ResNet-10 (stem + 4 basic blocks, C=%d, BN) bf16" % C,
            "replay_capacity_per_gpu": cfg.replay_capacity, "batch_per_gpu": cfg.batch,
            "gradient_allreduce": ("%s of %d fp32 per update (+ %d BN running-statistics floats)"
                                   % (lab, tr.flat.grad.numel(), tr.bn_buffers.data.numel())) if lab else None,
            "act_ms": a_ms, "env_step_store_ms": e_ms, "update_ms": u_ms,
            "warmup_steps": warmup, "timed_steps": steps,
            "env_steps_per_s": world * n_boards / ((a_ms + e_ms + u_ms) * 1e-3),
            "act_useful_TFLOPs": n_boards * useful / (a_ms * 1e-3) / 1e12,
            "act_frac_of_bf16_dense_peak": n_boards * useful / (a_ms * 1e-3) / 2.5e15,
            "loss": float(out["loss"])}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """`--gpus N` without torchrun: run torchrun (one rank per GPU) as a CHILD process -- this
    process never touches the GPU -- and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % n,
           "--master-addr=127.0.0.1", "--master-port=%d" % _free_port(), os.path.abspath(__file__)] + sys.argv[1:]
    print("bench.py: --gpus %d without WORLD_SIZE -> %s" % (n, " ".join(cmd)), file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def run_extras_all_ranks(world, rank, items):
    """Trainer extras on every rank (each issues collectives). After each one every rank posts
    its status to the rendezvous store and reads everyone's; on any failure the remaining extras
    are skipped on all ranks, so no rank enters a collective its peers will never join. (A rank
    that fails INSIDE a collective leaves its peers blocked until the process group's timeout.)"""
    store = dist.distributed_c10d._get_default_store()
    ex = {}
    for i, (key, fn) in enumerate(items):
        try:
            ex[key] = fn()
            ok = b"1"
        except Exception as e:      # recorded in the line; the check below keeps the ranks in step
            ex[key] = {"error": repr(e)}
            ok = b"0"
        store.set("r48/%s/%d" % (key, rank), ok)
        keys = ["r48/%s/%d" % (key, r) for r in range(world)]
        store.wait(keys, datetime.timedelta(seconds=900))
        if any(store.get(k) != b"1" for k in keys):
            if ok == b"1":
                ex[key]["error"] = "failed on another rank"
            for k2, _ in items[i + 1:]:
                ex[k2] = {"skipped": "an earlier extra failed on some rank"}
            break
    return ex


def hip_schedule_spin(local):
    """hipSetDeviceFlags(hipDeviceScheduleSpin) on torch's own HIP runtime, before torch creates the
    device context: synchronisations spin on the completion signal instead of sleeping until an
    interrupt wakes the thread."""
    import ctypes
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    if hip.hipSetDevice(local) != 0 or hip.hipSetDeviceFlags(1) != 0:
        print("bench.py: hipSetDeviceFlags(hipDeviceScheduleSpin) failed", file=sys.stderr)


def main():
    global SYNC_POLL, SETTLE_S, CLOSE_DEVICE, DRY_PASSES, SETTLE_SPIN
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=6000)
    ap.add_argument("--warmup", type=int, default=10000,
                    help="untimed steps; stepping continues untimed until %.0f ms have run (GPU clock ramp)"
                    % (SETTLE_S * 1e3))
    ap.add_argument("--boards", type=int, default=1 << 20, help="boards per GPU")
    ap.add_argument("--chunk", type=int, default=0, help="steps per r48_env_step_n call (0 = all K in one call)")
    ap.add_argument("--seed", type=int, default=0x20485EED)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--settle", type=float, default=SETTLE_S,
                    help="seconds of untimed stepping before each timed region (after the warm-up steps)")
    ap.add_argument("--sync", choices=("poll", "block", "spin"), default="block",
                    help="end of the timed region: spin on its last event, then synchronize (poll), only "
                         "synchronize (block), or synchronize with the HIP runtime set to spin-wait "
                         "(hipDeviceScheduleSpin) instead of sleeping (spin)")
    ap.add_argument("--close", choices=("event", "device"), default="event",
                    help="end of the timed region: wait on the region's last HIP event (event) or on the "
                         "device (torch.cuda.synchronize) before t1")
    ap.add_argument("--settle-spin", action="store_true",
                    help="the settle loop spins on its last event instead of sleeping in the blocking wait")
    ap.add_argument("--dry-passes", type=int, default=DRY_PASSES,
                    help="untimed passes through the timed region's exact host path before t0")
    args = ap.parse_args()
    SYNC_POLL = args.sync == "poll"
    DRY_PASSES = args.dry_passes
    SETTLE_SPIN = args.settle_spin
    CLOSE_DEVICE = args.close == "device"
    SETTLE_S = args.settle

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world), file=sys.stderr)
        sys.exit(2)
    cpu_line = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_line = cpu_baseline(args.cpu_seconds)          # before this process touches the GPU
    # R48_DIST_BACKEND=gloo only rehearses several ranks sharing one GPU (RCCL refuses two ranks
    # on one device); the product path is RCCL ("nccl" on ROCm), one rank per GPU
    backend = os.environ.get("R48_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend != "nccl":
        local %= max(1, ndev)
    if args.sync == "spin":
        hip_schedule_spin(local)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None,
                                timeout=datetime.timedelta(seconds=900))

    from rein48_amd import VecGame

    n, K, W = args.boards, args.steps, args.warmup
    offset, n = shard(rank, n)
    env = VecGame(n, device=dev, seed=args.seed, board_offset=offset)
    env.fill_random(7)                                    # SURVEY.md 8(d) synthetic start boards
    chunk = K if args.chunk <= 0 else max(1, min(args.chunk, K))
    plan = chunks(K, chunk)
    elapsed, dev_ms, skew = timed_steps(env, plan, W, chunk, world, dev)
    value = world * n * K / elapsed
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "env steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": elapsed * 1e3 / K,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int8",
        "data": "synthetic: start boards with each cell empty w.p. 1/2 else exponent ~U{1..7} (Philox, "
                "r48_env_fill_random), in-kernel uniform random policy and spawns from Philox4x32-7 (draw contract 3), "
                "auto-reset on game over",
        "config": {"workload": "BASELINE configs[1]: 2^20 4x4 int8 boards per GPU, random policy, env-only",
                   "boards_per_gpu": n, "global_boards": n * world,
                   "parallelism": "env shards x%d, no collective" % world,
                   "steps_per_launch": chunk, "launches": len(plan),
                   "world_size": dist.get_world_size() if world > 1 else 1,
                   "dist_backend": dist.get_backend() if world > 1 else None,
                   "start_skew_us": skew * 1e6,
                   "visible_devices": ndev},
        "roofline": roofline_step_n(n, elapsed, sum(dev_ms), K),
    }
    if cpu_line is not None:
        line["cpu_baseline"] = cpu_line
    if rank == 0 and world == 1:
        # 5 repeats of the same K-step region, each re-warmed
        reps = [timed_steps(env, plan, chunk, chunk, world, dev)[0] for _ in range(5)]
        vals = [n * K / r for r in reps]
        line["repeat_5"] = {"values": vals, "median": sorted(vals)[2],
                            "spread": (max(vals) - min(vals)) / sorted(vals)[2], "sync": args.sync}
    if rank == 0 and world == 1 and not args.no_extras:
        # the single-step HBM kernel: at 2^20 (cache-resident) and 2^26 boards (1 GiB, past the
        # 256 MiB Infinity Cache: the HBM-honest point)
        line["roofline"]["hbm"] = {"k_step_2p20": single_step_hbm(dev, args.seed, 1 << 20, 400),
                                   "k_step_2p26": single_step_hbm(dev, args.seed, 1 << 26, 30)}
        ex = extras(dev, args.seed, n)
        # the reference reset-distribution start (one tile per board) instead of the synthetic fill
        env2 = VecGame(n, device=dev, seed=args.seed, board_offset=offset)
        env2.reset()
        el2, _, _ = timed_steps(env2, plan, W, chunk, world, dev)
        ex["reset_start"] = {"value": n * K / el2, "note": "boards start from Game.reset (one 2/4 tile)"}
        del env2
        for key, fn in (("a3c_config3", lambda: a3c_config3(dev, args.seed, n)),
                        ("a3c_config3_reference",
                         lambda: a3c_config3(dev, args.seed, n, mode="reference", features="values")),
                        ("a3c_config3_reference_mlp",
                         lambda: a3c_config3(dev, args.seed, n, mode="reference", features="values", net="mlp",
                                             bf16=False)),
                        ("dqn_config5", lambda: dqn_config5(dev, args.seed, 1 << 21))):
            try:
                ex[key] = fn()
            except Exception as e:  # one rank: the env bench line must print even if a trainer fails
                ex[key] = {"error": repr(e)}
        if not args.no_cpu_baseline:
            ex["cpu_strong_line"] = strong_cpu_line()
        line["extras"] = ex
    if world > 1 and not args.no_extras:
        # BASELINE configs[3] (A3C, 2^20 boards per GPU: 8M on 8 GPUs) and configs[4] (DQN,
        # 2^21 boards per GPU: 16M on 8 GPUs), every rank stepping its own shard, gradients
        # all-reduced over the process group's backend
        line["extras"] = run_extras_all_ranks(world, rank, [
            ("a3c_config4", lambda: a3c_config3(dev, args.seed, n, world=world)),
            ("dqn_config5", lambda: dqn_config5(dev, args.seed, 1 << 21, world=world))])
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
