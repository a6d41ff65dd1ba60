"""world_size-2 gloo tests of the sharding / gather path (CPU; the GPU env itself is covered by
test_gpu_parity.py::test_determinism_and_sharding, which checks that a shard's results equal the
same envs of an unsharded batch)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from heligym_amd.distributed import all_gather_rows, gather_rows, shard_bounds


def test_shard_bounds_cover_exactly():
    for total in (1, 7, 8, 65536, 1048576, 1000003):
        for world in (1, 2, 3, 4, 8):
            if total < world:
                continue
            spans = [shard_bounds(total, r, world) for r in range(world)]
            assert spans[0][0] == 0
            for (o0, c0), (o1, _) in zip(spans, spans[1:]):
                assert o0 + c0 == o1
            assert sum(c for _, c in spans) == total
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
    with pytest.raises(ValueError):
        shard_bounds(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        off, cnt = shard_bounds(total, rank, world)
        # stand-in observation rows: value = global env id * 17 + column
        local = (torch.arange(off, off + cnt, dtype=torch.float32)[:, None] * 17
                 + torch.arange(17, dtype=torch.float32)[None, :])
        full = all_gather_rows(local, total)
        g = gather_rows(local, total, dst=0)
        ref = torch.arange(total, dtype=torch.float32)[:, None] * 17 + torch.arange(17, dtype=torch.float32)
        ok = bool(torch.equal(full, ref)) and (g is None if rank else bool(torch.equal(g, ref)))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("total", [64, 1001])
def test_gather_world_size_2_gloo(total):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


class _FakeVecEnv:
    """CPU stand-in for HeliVecEnv inside ShardedHeliVecEnv (no HIP device here): observation rows
    that name their global env id, so a gather shows where every row came from."""

    def __init__(self, num_envs, env_offset=0, **kw):
        self.num_envs, self.env_offset = num_envs, env_offset
        self.obs = (torch.arange(env_offset, env_offset + num_envs, dtype=torch.float32)[:, None] * 17
                    + torch.arange(17, dtype=torch.float32)[None, :])

    def close(self):
        pass


def _sharded_worker(rank, world, port, total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from heligym_amd import vector
        from heligym_amd.distributed import ShardedHeliVecEnv
        vector.HeliVecEnv = _FakeVecEnv   # (this spawned process only)
        env = ShardedHeliVecEnv(total, task="hover")
        off, cnt = shard_bounds(total, rank, world)
        ok = env.offset == off and env.count == cnt and env.env.num_envs == cnt and env.env.env_offset == off
        ref = torch.arange(total, dtype=torch.float32)[:, None] * 17 + torch.arange(17, dtype=torch.float32)
        g = env.gather_obs(dst=0)
        ok = ok and (g is None if rank else bool(torch.equal(g, ref)))
        g7 = env.gather_obs(dst=world - 1)   # another destination rank
        ok = ok and (g7 is None if rank != world - 1 else bool(torch.equal(g7, ref)))
        ok = ok and bool(torch.equal(env.all_gather_obs(), ref))
        env.close()
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_sharded_env_gather_obs_world_size_8_ragged():
    """BASELINE config 5's exchange at the driver's world size: ShardedHeliVecEnv over 8 gloo ranks
    with a ragged batch (2 049 envs: rank 0 holds 257 rows, the others 256), gathered to rank 0, to
    the last rank and to every rank, each row landing at its global env id."""
    world, total = 8, 2049
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}
