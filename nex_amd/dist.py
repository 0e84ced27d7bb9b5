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


def pick_backend() -> str:
    """RCCL ("nccl" on ROCm) when this process has a GPU, gloo otherwise;
    NEXG_DIST_BACKEND overrides (gloo lets several ranks share one GPU for a
    rehearsal of the multi-rank path, which RCCL refuses). Only the timing
    barrier and two scalar reductions ever use it."""
    import torch
    import torch.distributed as dist
    forced = os.environ.get("NEXG_DIST_BACKEND")
    if forced:
        return forced
    if torch.cuda.is_available() and dist.is_nccl_available():
        return "nccl"
    return "gloo"


def device_index(local: int) -> int:
    """GPU of a rank: its LOCAL_RANK, folded onto the visible devices when
    there are fewer (the shared-GPU rehearsal; the 8-GPU run maps 1:1)."""
    import torch
    n = torch.cuda.device_count()
    return local % n if n else local


def init(backend: str = None, force: bool = False):
    """Create the process group for world > 1 (or at world 1 with `force`,
    so the RCCL branches below can be exercised on a one-GPU box)."""
    import torch.distributed as dist
    rank, world, _ = env_rank_world()
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        dist.init_process_group(backend=backend or pick_backend(), rank=rank, world_size=world)
    return rank, world


def timed_steps(step, steps: int, warmup: int, sync=None, device=None, before=None, after=None,
                warmup_seconds: float = 0.0, stats=None):
    """bench.py's timing discipline: `warmup` untimed steps (continued, in
    batches of 32, until at least `warmup_seconds` of wall time have passed),
    then exactly `steps` steps bracketed by sync + barrier + sync on both
    sides; returns (max-over-ranks elapsed seconds, this rank's elapsed
    seconds). `sync` waits for this rank's device work (torch.cuda.synchronize
    on a GPU); before/after run inside the timed bracket around the steps (HIP
    event records). A `stats` dict receives the warmup actually run
    (`warmup_steps`, `warmup_s`)."""
    import time
    sync = sync or (lambda: None)
    t_w = time.perf_counter()
    n_w = warmup
    for _ in range(warmup):
        step()
    sync()
    while time.perf_counter() - t_w < warmup_seconds:
        for _ in range(32):
            step()
        n_w += 32
        sync()
    if stats is not None:
        stats.update(warmup_steps=n_w, warmup_s=round(time.perf_counter() - t_w, 4))
    barrier(device)
    sync()
    t0 = time.perf_counter()
    if before:
        before()
    for _ in range(steps):
        step()
    if after:
        after()
    sync()
    t1 = time.perf_counter()
    barrier(device)
    return max_over_ranks(t1 - t0, device), t1 - t0


def throughput(frames_per_rank: int, bytes_per_rank: int, steps: int, elapsed_max: float, device=None):
    """Whole-job numbers of a weak-scaling run: every rank processed its own
    shard `steps` times; value = frames over all ranks / MAX elapsed."""
    total_frames = sum_over_ranks(frames_per_rank, device) * steps
    total_bytes = sum_over_ranks(bytes_per_rank, device) * steps
    return {"value": round(total_frames / elapsed_max / 1e6, 2), "unit": "Mpkt/s",
            "ms_per_step": round(elapsed_max / steps * 1e3, 4),
            "gib_s": round(total_bytes / elapsed_max / 2**30, 2),
            "total_frames": total_frames, "total_bytes": total_bytes}


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


def all_ranks(value: float, device=None) -> list:
    """Every rank's `value`, in rank order (per-rank kernel times in the
    multi-rank bench line: the balance across GPUs)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return [value]
    dev = device if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(x.item()) for x in out]
