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
