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
