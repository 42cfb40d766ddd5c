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
