"""N>1 path on CPU (gloo, world_size 2): the env shards with no data-path collective.

Each rank steps its shard [rank*N, (rank+1)*N) with the kernel's Philox contract (restated by
the oracle, which the GPU tests pin the kernel to bit-for-bit); gathered, the shards equal one
unsharded env. The bench's timing aggregation (max over ranks) is exercised over gloo too.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from oracle import native as O
        off, cnt = bench.shard(rank, n)
        rng = np.random.default_rng(123)
        b_all = rng.integers(0, 6, size=(n * world, 16)).astype(np.int8)
        b = b_all[off:off + cnt]
        b = O.reset_philox(b, seed=5, reset_ctr=0, board_offset=off)
        for t in range(6):
            b = O.step_philox(b, seed=5, step=t, flags=O.RANDOM_POLICY | O.AUTO_RESET, board_offset=off)["boards"]
        parts = [None] * world
        dist.all_gather_object(parts, b)
        elapsed = bench.max_over_ranks(0.5 + rank, torch.device("cpu"), world)
        if rank == 0:
            out_q.put((np.concatenate(parts), elapsed, b_all))
    finally:
        dist.destroy_process_group()


def test_two_rank_shards_equal_unsharded_env():
    from oracle import native as O
    world, n = 2, 4096
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    sharded, elapsed, b_all = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    whole = O.reset_philox(b_all, seed=5, reset_ctr=0)
    for t in range(6):
        whole = O.step_philox(whole, seed=5, step=t, flags=O.RANDOM_POLICY | O.AUTO_RESET)["boards"]
    assert np.array_equal(sharded, whole)
    assert elapsed == pytest.approx(1.5)


def _extras_worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        calls = []

        def first():
            calls.append("first")
            if rank == 1:
                raise RuntimeError("simulated OOM on rank 1")
            return {"ok": True}

        def second():
            calls.append("second")
            dist.all_reduce(torch.ones(1))          # a collective every rank would need to join
            return {"ok": True}

        ex = bench.run_extras_all_ranks(world, rank, [("a", first), ("b", second)])
        out_q.put((rank, ex, calls))
    finally:
        dist.destroy_process_group()


def test_bench_extras_failure_on_one_rank_skips_the_rest_everywhere():
    """an extra that raises on ONE rank must not leave the other ranks inside a
    collective the failed rank never joins. bench.run_extras_all_ranks exchanges a status per
    extra through the rendezvous store and skips the remaining extras on every rank."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_extras_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=90) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ex, calls in res:
        assert calls == ["first"]                            # "second" ran nowhere
        assert "error" in ex["a"] and "skipped" in ex["b"]
    assert "simulated OOM" in res[1][1]["a"]["error"]
    assert res[0][1]["a"]["error"] == "failed on another rank"


def test_bench_world_size_mismatch_exits_before_the_gpu():
    """--gpus N that disagrees with torchrun's WORLD_SIZE is an error (exit 2), not a warning."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "1"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_bench_gpus_without_torchrun_launches_ranks(monkeypatch):
    """--gpus N with no WORLD_SIZE: bench.py starts torchrun (N ranks, 127.0.0.1) as a child
    process and exits with its status -- it never benchmarks one GPU under an N-GPU label."""
    import subprocess
    import sys
    import bench
    seen = {}
    monkeypatch.setattr(subprocess, "call", lambda cmd: seen.setdefault("cmd", cmd) and 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "20"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.launch_ranks(8) == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=8" in cmd
    assert "--master-addr=127.0.0.1" in cmd and cmd[-4:] == ["--gpus", "8", "--steps", "20"]
