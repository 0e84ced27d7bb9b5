"""GPU: the bench's malformed mix (nex_amd/workloads.py)
parses to exactly the oracle's records in every output kind, and its tiled
full-size form repeats the per-copy results."""
import numpy as np
import pytest

from nex_amd import abi, workloads
from tests import helpers

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mix(engine):
    return workloads.malformed_mix(engine, 60000, seed=77)


def host_frames(batch):
    offs = batch.offsets.cpu().numpy().astype(np.int64)
    data = batch.data.cpu().numpy()
    return [bytes(data[a:b]) for a, b in zip(offs[:-1], offs[1:])]


def test_mix_shape(mix):
    batch, counts = mix
    assert sum(counts.values()) == batch.count == 60000
    assert 0.45 < counts["unmodified"] / batch.count < 0.55
    assert all(counts[m] > 2000 for m in workloads.MUTATIONS)


def test_malformed_mix_matches_oracle(engine, oracle, mix):
    batch, _ = mix
    frames = host_frames(batch)
    want = oracle.parse_frames(frames)
    got = engine.parse_to_numpy(batch, out_kind=abi.OUT_RECORD)
    helpers.records_equal(got, want, frames, "malformed mix record")
    d = np.zeros(len(frames), abi.DESC_DTYPE)
    for n in abi.DESC_DTYPE.names:
        d[n] = want[n]
    got = engine.parse_to_numpy(batch, out_kind=abi.OUT_SPARSE)
    helpers.records_equal(got, d, frames, "malformed mix sparse")
    got = engine.parse_to_numpy(batch, out_kind=abi.OUT_GROUPED)
    helpers.records_equal(got, d, frames, "malformed mix grouped")
    # the mutations leave the canonical shapes (exception slots) and reach
    # the error statuses (lenient parsing turns most into shorter layer stacks)
    codes = engine.parse(batch, out_kind=abi.OUT_SPARSE)[: batch.count].cpu().numpy()
    assert (codes == 0).mean() > 0.05
    assert ((want["flags"] >> abi.STATUS_SHIFT) != 0).sum() > 100


def test_tiled_repeats(engine, mix):
    import torch
    batch, _ = mix
    t = workloads.tiled(batch, 3)
    one = engine.parse(batch, out_kind=abi.OUT_DESC)[: batch.count * 8]
    three = engine.parse(t, out_kind=abi.OUT_DESC)[: t.count * 8]
    torch.cuda.synchronize()
    span = int(batch.offsets[batch.count].item())
    d1 = one.cpu().numpy().view(abi.DESC_DTYPE)
    d3 = three.cpu().numpy().view(abi.DESC_DTYPE)
    for k in range(3):
        assert (d3[k * batch.count:(k + 1) * batch.count] == d1).all()
    assert int(t.offsets[-1].item()) == 3 * span


def test_tcp_timestamps_match_oracle(engine, oracle):
    """The real-traffic TCP shape (NOP NOP Timestamps, data offset 8; the
    register fast path takes it behind IPv4 and IPv6, damaged layouts go to
    the generic core) at every byte alignment the packed IMIX layout
    produces, in record and sparse form."""
    batch, counts = workloads.malformed_mix(engine, 40000, seed=78, kinds=("tcp_ts",))
    assert counts["tcp_ts"] > 15000
    frames = host_frames(batch)
    want = oracle.parse_frames(frames)
    assert ((want["l4_nopt"] == 3) & (want["l4_length"] == 32)).sum() > 3000
    got = engine.parse_to_numpy(batch, out_kind=abi.OUT_RECORD)
    helpers.records_equal(got, want, frames, "tcp_ts record")
    d = np.zeros(len(frames), abi.DESC_DTYPE)
    for n in abi.DESC_DTYPE.names:
        d[n] = want[n]
    got = engine.parse_to_numpy(batch, out_kind=abi.OUT_SPARSE)
    helpers.records_equal(got, d, frames, "tcp_ts sparse")


def test_fastpath_edge_shapes_on_gpu(engine, oracle):
    """The register fast path's round-3 shapes (frames under 14 B, one IPv6
    extension header, TCP option walks failing at the first TLV) and their
    near misses on the GPU: span kernel (packed, frames at every byte
    alignment; capture gaps with the monotone hint) and lane kernel (explicit lengths), record
    and grouped output, lenient and strict, equal the oracle."""
    import torch
    from nex_amd.engine import FrameBatch
    from nex_amd.frame import ParseMode, ParseOption
    frames = helpers.fastpath_edge_frames(np.random.default_rng(31))
    for mode in (ParseMode.Lenient, ParseMode.Strict):
        opt = ParseOption()
        want = oracle.parse_frames(frames, opt.flags(mode))
        d = np.zeros(len(frames), abi.DESC_DTYPE)
        for n in abi.DESC_DTYPE.names:
            d[n] = want[n]
        batches = [FrameBatch.from_packed(frames, shift=s) for s in (0, 4)]  # packed: every byte alignment occurs
        batches.append(FrameBatch.from_frames(frames, pad_to=4))
        b = FrameBatch.from_frames(frames, pad_to=16)
        b.hints = abi.FRAMES_MONOTONE
        batches.append(b)
        for k, batch in enumerate(batches):
            helpers.records_equal(engine.parse_to_numpy(batch, opt, mode, abi.OUT_RECORD), want, frames,
                                  f"edge record layout {k} {mode}")
            helpers.records_equal(engine.parse_to_numpy(batch, opt, mode, abi.OUT_GROUPED), d, frames,
                                  f"edge grouped layout {k} {mode}")
    torch.cuda.synchronize()
