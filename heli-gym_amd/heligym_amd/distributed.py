"""Multi-GPU sharding of the vectorised env: one process per GPU (torchrun), contiguous env ranges.

Envs never interact, so the data path needs no collective: rank r owns global envs
[offset_r, offset_r + count_r) and passes offset_r as `env_offset`, which keys the in-kernel Philox
noise by GLOBAL env id -- results are identical for any number of ranks.  The only optional
exchange is for a single-host policy: gather every rank's observations (and rewards / flags) to one
rank, or all-gather them, over RCCL ("nccl" backend = RCCL on ROCm, xGMI between GPUs).
"""
import torch
import torch.distributed as dist


def shard_bounds(total, rank, world):
    """(offset, count) of rank's contiguous share of `total` envs; the first total % world ranks
    get one extra env."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, extra = divmod(int(total), int(world))
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


def _staged(t, group):
    """gloo collectives take host tensors: GPU rows go through the host there (the rehearsal of the
    RCCL path on one GPU; RCCL itself moves device memory over xGMI)."""
    return t.cpu() if t.is_cuda and dist.get_backend(group) == "gloo" else t


def _pad_to(t, rows):
    if t.shape[0] == rows:
        return t
    pad = torch.zeros((rows - t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    return torch.cat([t, pad], 0)


def all_gather_rows(local, total, group=None):
    """All-gather per-rank row blocks (uneven shards allowed) into one [total, ...] tensor on every
    rank, in global env order."""
    world = dist.get_world_size(group)
    counts = [shard_bounds(total, r, world)[1] for r in range(world)]
    m = max(counts)
    x = _staged(_pad_to(local.contiguous(), m), group)
    buf = torch.empty((world * m,) + tuple(local.shape[1:]), dtype=local.dtype, device=x.device)
    dist.all_gather_into_tensor(buf, x, group=group)
    parts = [buf[r * m: r * m + counts[r]] for r in range(world)]
    return torch.cat(parts, 0).to(local.device)


def gather_rows(local, total, dst=0, group=None):
    """Gather per-rank row blocks to rank `dst` only ([total, ...] there, None elsewhere)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    counts = [shard_bounds(total, r, world)[1] for r in range(world)]
    m = max(counts)
    x = _staged(_pad_to(local.contiguous(), m), group)
    if rank == dst:
        bufs = [torch.empty_like(x) for _ in range(world)]
        dist.gather(x, gather_list=bufs, dst=dst, group=group)
        return torch.cat([bufs[r][:counts[r]] for r in range(world)], 0).to(local.device)
    dist.gather(x, dst=dst, group=group)
    return None


class ShardedHeliVecEnv:
    """This rank's shard of a `total_envs` batch (one GPU per process).  step()/reset() act on the
    local shard only; gather_obs()/all_gather_obs() assemble the global observation batch."""

    def __init__(self, total_envs, rank=None, world=None, group=None, **env_kwargs):
        from .vector import HeliVecEnv
        self.group = group
        self.rank = dist.get_rank(group) if rank is None else rank
        self.world = dist.get_world_size(group) if world is None else world
        self.total_envs = int(total_envs)
        self.offset, self.count = shard_bounds(total_envs, self.rank, self.world)
        self.env = HeliVecEnv(self.count, env_offset=self.offset, **env_kwargs)

    def reset(self, **kw):
        return self.env.reset(**kw)

    def step(self, actions, **kw):
        return self.env.step(actions, **kw)

    def step_async(self, actions, **kw):
        return self.env.step_async(actions, **kw)

    def gather_obs(self, dst=0):
        return gather_rows(self.env.obs, self.total_envs, dst=dst, group=self.group)

    def all_gather_obs(self):
        return all_gather_rows(self.env.obs, self.total_envs, group=self.group)

    def close(self):
        self.env.close()
