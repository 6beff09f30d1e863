"""Multi-GPU plumbing: one process per GPU, games sharded by global env id.

Games never interact, so the step loop has no collective.  Rank r of a
world of W owns global env ids [r*B, (r+1)*B) (B lanes per rank); because
every lane's random stream is keyed by its global id,
the union of the ranks' trajectories equals a single-process run over W*B
lanes.  `collate` gathers per-lane results over RCCL (xGMI) -- or gloo on
CPU tensors in tests -- outside the step loop.
"""
import os

import torch
import torch.distributed as dist


def world_info():
    """(rank, world_size, local_rank) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def env_id_base(rank, lanes_per_rank):
    """First global env id of a rank's shard."""
    return rank * lanes_per_rank


def init(backend="nccl", gpu=None, force=False):
    """Initialise the process group for a torchrun launch (no-op for one
    process unless `force`).  Returns the torch device of this rank:
    cuda:LOCAL_RANK for nccl (RCCL); for gloo the CPU, or with gpu=True a GPU
    shared round-robin by the ranks (a rehearsal of the multi-GPU path on a
    box with fewer GPUs than ranks; RCCL refuses two ranks on one GPU).
    force: create the group even for one process (a one-rank RCCL
    communicator), so that collate / max_over_ranks(force=True) run the
    collectives the multi-GPU job runs; the rendezvous still comes from
    MASTER_ADDR / MASTER_PORT."""
    rank, world, local = world_info()
    if backend == "nccl":
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
    elif gpu:
        dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    if (world > 1 or force) and not dist.is_initialized():
        kw = {"device_id": dev} if backend == "nccl" else {}
        dist.init_process_group(backend, **kw)
    return dev


def collate(t, dim=0, force=False):
    """All-gather a per-lane tensor from every rank; lanes are along `dim`
    ([B, ...] by default, dim=1 for [T, B, ...] trajectories).  Returns the
    concatenation along `dim` in rank (= global env id) order.  One rank
    returns `t` itself unless `force` (and a group exists): then the
    collective runs anyway, over a one-rank communicator."""
    if not dist.is_initialized() or (dist.get_world_size() == 1 and not force):
        return t
    if dim == 0 and dist.get_backend() == "nccl":
        # RCCL writes the rank-ordered concatenation in place: no gather list, no cat
        out = torch.empty((dist.get_world_size() * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t.contiguous())
        return out
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t.contiguous())
    return torch.cat(parts, dim)


def max_over_ranks(x, device, force=False):
    """Max of a host float over ranks (the bench's timing rule)."""
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    if dist.is_initialized() and (dist.get_world_size() > 1 or force):
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
