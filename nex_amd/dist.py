"""Multi-GPU plumbing: one process per GPU, index-range shards, no data-path
collective. The only collectives are the timing barrier and
a MAX over the per-rank elapsed time."""
import os


def env_rank_world():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def shard(total: int, rank: int, world: int):
    """Contiguous index range [begin, end) of `total` frames owned by `rank`."""
    begin = total * rank // world
    end = total * (rank + 1) // world
    return begin, end


def init(backend: str):
    import torch.distributed as dist
    rank, world, _ = env_rank_world()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world


def barrier(device=None):
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        if device is not None and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()


def max_over_ranks(value: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return value
    t = torch.tensor([value], dtype=torch.float64,
                     device=device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: int, device=None) -> int:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return value
    t = torch.tensor([value], dtype=torch.int64,
                     device=device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())
