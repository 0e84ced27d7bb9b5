"""GPU: the RCCL branches of nex_amd/dist.py (device-tensor barrier, MAX / SUM
reductions and the per-rank gather bench.py runs) on a world-1 "nccl"
process group on cuda:0, around a real parse under timed_steps — so the
driver's 8-GPU run is not the first contact of this code with RCCL
(VERDICT r02 weak 6). Multi-rank semantics are covered on gloo in
tests/test_multirank.py."""
import socket

import pytest

from nex_amd import abi, dist

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_world1_branches(engine, oracle, monkeypatch):
    import torch
    import torch.distributed as tdist
    from tests import helpers
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("LOCAL_RANK", "0")
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(_free_port()))
    monkeypatch.delenv("NEXG_DIST_BACKEND", raising=False)
    assert dist.pick_backend() == "nccl"
    rank, world = dist.init(force=True)
    try:
        assert (rank, world) == (0, 1) and tdist.get_backend() == "nccl"
        dev = torch.device("cuda", dist.device_index(0))
        dist.barrier(dev)
        assert dist.max_over_ranks(1.25, dev) == 1.25
        assert dist.sum_over_ranks(7, dev) == 7
        assert dist.all_ranks(2.5, dev) == [2.5]
        n = 1 << 16
        b = engine.gen_batch(abi.WL_UDP64, n)
        out = torch.empty(engine.out_bytes(abi.OUT_DESC, n), dtype=torch.uint8, device=dev)
        calls = []
        step = lambda: (calls.append(1), engine.parse(b, out_kind=abi.OUT_DESC, out=out))
        elapsed, local = dist.timed_steps(step, 4, 2, sync=lambda: torch.cuda.synchronize(dev), device=dev)
        assert len(calls) == 6 and elapsed == local > 0
        tp = dist.throughput(n, 64 * n, 4, elapsed, dev)
        assert tp["total_frames"] == 4 * n and tp["total_bytes"] == 256 * n
        got = out.cpu().numpy().view(abi.DESC_DTYPE)
        raw = b.data.cpu().numpy().reshape(n, 64)[:2048]
        want = oracle.parse_frames([bytes(r) for r in raw])
        for k in abi.DESC_DTYPE.names:
            assert (got[k][:2048] == want[k]).all(), k
    finally:
        tdist.destroy_process_group()
