"""CPU (gloo, world_size 2): the sharded path bench.py uses. Each rank owns a
contiguous index range, regenerates its shard from (seed, global index), parses
it with no data-path collective, and the concatenation over ranks equals the
single-process result; timing is reduced with MAX as bench.py does."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from nex_amd import abi, dist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as tdist
    from oracle import oracle
    dist.init("gloo")
    b, e = dist.shard(total, rank, world)
    recs = np.array([oracle.parse_frame(oracle.gen_frame(abi.WL_IMIX, i)) for i in range(b, e)],
                    dtype=abi.RECORD_DTYPE)
    dist.barrier()
    t = dist.max_over_ranks(float(rank + 1))
    n = dist.sum_over_ranks(e - b)
    q.put((rank, b, e, recs.tobytes(), t, n))
    tdist.destroy_process_group()


def test_two_rank_shards_equal_single(oracle):
    total, world = 301, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][2] == res[1][1] and res[0][1] == 0 and res[1][2] == total
    assert all(r[4] == 2.0 for r in res)          # MAX over ranks
    assert all(r[5] == total for r in res)        # frames summed over ranks
    joined = np.frombuffer(b"".join(r[3] for r in res), dtype=abi.RECORD_DTYPE)
    single = np.array([oracle.parse_frame(oracle.gen_frame(abi.WL_IMIX, i)) for i in range(total)],
                      dtype=abi.RECORD_DTYPE)
    assert joined.tobytes() == single.tobytes()


def test_shard_covers_range():
    for total in (0, 1, 7, 1000, 16 << 20):
        for world in (1, 2, 3, 8):
            spans = [dist.shard(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))


def _bench_worker(rank, world, port, q):
    """bench.py's multi-rank leg with a stub step: dist.timed_steps (barriers,
    MAX over ranks) + dist.throughput (SUM over ranks), the functions
    bench.py's timed() / main() call, on gloo."""
    import time
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as tdist
    assert dist.pick_backend() == "gloo"  # no GPU in this process
    dist.init()
    calls = []
    step = lambda: (calls.append(1), time.sleep(0.002 * (rank + 1)))
    elapsed_max, local = dist.timed_steps(step, steps=5, warmup=2)
    frames, nbytes = 1000 + rank, 64 * (1000 + rank)
    tp = dist.throughput(frames, nbytes, 5, elapsed_max)
    per_rank = dist.all_ranks(float(10 * rank + 1))  # bench.py's per-rank kernel_ms list
    q.put((rank, len(calls), elapsed_max, local, tp, per_rank))
    tdist.destroy_process_group()


def test_two_rank_bench_reduction():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] == 7 for r in res)  # warmup + exactly the timed steps
    emax = max(r[3] for r in res)
    assert all(r[2] == emax for r in res)  # every rank sees the MAX of the local times
    assert emax >= 5 * 0.004  # the slower rank bounds the job
    total = (1000 + 1001) * 5
    for r in res:
        tp = r[4]
        assert tp["total_frames"] == total and tp["total_bytes"] == 64 * total
        assert tp["value"] == round(total / emax / 1e6, 2)
        assert tp["ms_per_step"] == round(emax / 5 * 1e3, 4)
        assert r[5] == [1.0, 11.0]  # every rank's value, in rank order


def test_timed_steps_warmup_floor():
    """bench.py's warmup floor (dist.timed_steps warmup_seconds): W untimed
    steps, then whole batches of 32 until the floor has passed; the timed
    region is still exactly `steps` steps."""
    import time
    calls = []

    def step():
        calls.append(time.perf_counter())
        time.sleep(0.0005)
    elapsed, local = dist.timed_steps(step, steps=7, warmup=3, warmup_seconds=0.05)
    warm = len(calls) - 7
    assert warm >= 3 + 32 and (warm - 3) % 32 == 0
    assert calls[warm - 1] - calls[0] >= 0.04 and elapsed == local > 0
    calls.clear()
    dist.timed_steps(step, steps=7, warmup=3)
    assert len(calls) == 10
