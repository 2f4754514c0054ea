"""shard.py -- file-parallel sharding of the checksum path across GPUs (SURVEY.md §8 e).

Files are independent units (a file's Generator pass and Sender scan depend only on that file, its
basis table and the seed), so a multi-GPU job is N independent processes, one per GPU, each owning a
shard of the files: no collective on the data path.  The only collectives are the benchmark's barrier
and the max-over-ranks time reduction.
"""
import os


def shard_files(sizes, world):
    """Longest-processing-time-first bin packing of file sizes onto `world` ranks.

    Returns a list (one per rank) of file indices in ascending order.  Deterministic: ties go to the
    lowest rank, equal sizes keep their index order.
    """
    load = [0] * world
    out = [[] for _ in range(world)]
    for i in sorted(range(len(sizes)), key=lambda i: (-sizes[i], i)):
        r = min(range(world), key=lambda r: (load[r], r))
        out[r].append(i)
        load[r] += sizes[i]
    return [sorted(x) for x in out]


def env_rank():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("LOCAL_RANK", "0"))


def rank_device(local, world, ngpu):
    """(device, backend, shared) for a rank: its own GPU LOCAL_RANK and RCCL for the barrier and the time
    reduction when the node has a GPU per local rank; otherwise (a rehearsal of N ranks on a box with fewer GPUs)
    ranks share GPUs round-robin and the collectives run on gloo, since RCCL refuses two ranks on one device.
    The choice depends only on (LOCAL_WORLD_SIZE, ngpu), so every rank picks the same backend."""
    if ngpu < 1:
        raise RuntimeError("no GPU visible to this rank")
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if local_world <= ngpu:
        return local, "nccl", False
    return local % ngpu, "gloo", True


def init_distributed(backend, device=None):
    """torch.distributed over 127.0.0.1 (the container hostname may not resolve)."""
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    kw = {}
    if device is not None:
        kw["device_id"] = device
    dist.init_process_group(backend, **kw)
    return dist


def reduce_over_ranks(value, op, device="cpu"):
    """All-reduce one float (op: 'max' or 'sum'); identity when not distributed."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return float(t.item())


def gather_over_ranks(value, device="cpu"):
    """Every rank's value of one float, in rank order; [value] when not distributed."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [float(value)]
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(x.item()) for x in out]
