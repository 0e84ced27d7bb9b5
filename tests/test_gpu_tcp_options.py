"""GPU parity of the register fast path's one-TLV TCP option branch
(frame_core.hpp fast_canonical80: MSS alone, NOP NOP + any-kind TLV — SACK
1-4 blocks, timestamps, unknown kinds — exactly filling the data offset) as the
gfx950 kernels run it: the span kernel's LDS staging, `v_alignbyte`
realignment and sparse-code hand-over (packed offsets; offsets + lengths with
the monotone hint at every byte alignment), the TwoPass lane kernel (offsets +
lengths, no hint) and the fixed-stride tile kernel — against the oracle's
literal restatement of the reference's option walk and re-serialisation
(tcp.rs:731-836, :521-575), in record, sparse (host decode) and
sparse-expanded (device) form. VERDICT r02 weak 1 / next 1."""
import numpy as np
import pytest

from nex_amd import abi, workloads
from nex_amd.engine import FrameBatch
from tests import helpers

pytestmark = pytest.mark.gpu


def desc_of(recs):
    d = np.zeros(len(recs), abi.DESC_DTYPE)
    for n in abi.DESC_DTYPE.names:
        d[n] = recs[n]
    return d


@pytest.fixture(scope="module")
def sweep(oracle):
    rng = np.random.default_rng(731)
    bases = [oracle.gen_frame(abi.WL_IMIX, i) for i in range(600)]
    P = bytes(range(40))
    bases += [helpers._eth(helpers._ipv4(helpers._tcp(P[:k]), 6)) for k in (0, 1, 7, 26)]
    bases += [helpers._eth(helpers._ipv6(helpers._tcp(P[:k]), 6), 0x86DD) for k in (0, 3, 40)]
    frames = helpers.tcp_option_sweep(oracle, rng, bases)
    # canonical IMIX frames around them, so groups mix fast shapes, TLV shapes and declines
    frames += [oracle.gen_frame(abi.WL_IMIX, i) for i in range(600, 3600)]
    order = np.random.default_rng(1).permutation(len(frames))
    frames = [frames[i] for i in order]
    want = oracle.parse_frames(frames)
    tcp = (want["flags"] & abi.L_TCP) != 0
    # both verdicts on both option shapes, for both families
    for nopt in (1, 3):
        for fam in (abi.L_IPV4, abi.L_IPV6):
            sel = tcp & (want["l4_nopt"] == nopt) & ((want["flags"] & fam) != 0)
            assert ((want["flags"][sel] & abi.C_L4_OK) != 0).sum() > 50, (nopt, fam)
            assert ((want["flags"][sel] & abi.C_L4_OK) == 0).sum() > 50, (nopt, fam)
    return frames, want


def gapped(frames, rng, max_gap):
    """offsets + lengths, frames 0..max_gap bytes apart (every byte alignment)."""
    import torch
    gaps = rng.integers(0, max_gap + 1, len(frames))
    blob, offs = bytearray(), []
    for f, g in zip(frames, gaps):
        blob += bytes(int(g))
        offs.append(len(blob))
        blob += f
    data = torch.frombuffer(bytes(blob) + bytes(16), dtype=torch.uint8).cuda()
    return (data, torch.tensor(offs, dtype=torch.int64, device="cuda"),
            torch.tensor([len(f) for f in frames], dtype=torch.int32, device="cuda"))


def layouts(frames):
    rng = np.random.default_rng(836)
    out = [("packed", FrameBatch.from_packed(frames)),
           ("packed shift 4", FrameBatch.from_packed(frames, pad_to=1, shift=4))]
    data, ot, lt = gapped(frames, rng, 3)
    out.append(("gaps 0-3 + monotone", FrameBatch(data=data, count=len(frames), offsets=ot, lengths=lt,
                                                  hints=abi.FRAMES_MONOTONE)))
    out.append(("gaps 0-3 two-pass", FrameBatch(data=data, count=len(frames), offsets=ot, lengths=lt)))
    return out


@pytest.mark.parametrize("out_kind", [abi.OUT_RECORD, abi.OUT_SPARSE, abi.OUT_DESC])
def test_one_tlv_options_every_layout(engine, sweep, out_kind):
    import torch
    frames, want = sweep
    w = want if out_kind == abi.OUT_RECORD else desc_of(want)
    for name, batch in layouts(frames):
        got = engine.parse_to_numpy(batch, out_kind=out_kind)
        helpers.records_equal(got, w, frames, f"tcp options {name} out={out_kind}")
        if out_kind == abi.OUT_SPARSE:
            raw = engine.parse(batch, out_kind=abi.OUT_SPARSE)
            dev = engine.sparse_expand(batch, raw)
            torch.cuda.synchronize()
            dev = dev.cpu().numpy()[: len(frames) * 8].view(abi.DESC_DTYPE)
            helpers.records_equal(dev, w, frames, f"tcp options expand {name}")


def test_one_tlv_options_verdict_and_strict(engine, oracle, sweep):
    """The narrow outputs (TwoPass hands tail sums over through the ctx
    scratch) and strict mode (the fast path declines strict errors)."""
    from nex_amd.frame import ParseMode, ParseOption
    frames, want = sweep
    for name, batch in layouts(frames):
        got = engine.parse_to_numpy(batch, out_kind=abi.OUT_VERDICT)
        assert (abi.verdict_to_flags(got["verdict"]) == want["flags"].astype(np.uint32)).all(), name
    ws = oracle.parse_frames(frames, abi.PARSE_STRICT)
    for name, batch in layouts(frames)[::2]:
        got = engine.parse_to_numpy(batch, ParseOption(), ParseMode.Strict, abi.OUT_RECORD)
        helpers.records_equal(got, ws, frames, f"tcp options strict {name}")


@pytest.mark.parametrize("stride", [128, 144])
def test_one_tlv_options_fixed_stride(engine, oracle, sweep, stride):
    """Frames that fit a fixed stride (128: TileStride kernel, 144: span kernel
    over a stride), trailing bytes random (Ethernet padding)."""
    frames, _ = sweep
    sel = [f for f in frames if len(f) <= stride][:6000]
    rng = np.random.default_rng(stride)
    arr = rng.integers(0, 256, (len(sel), stride), dtype=np.uint8)
    for i, f in enumerate(sel):
        arr[i, :len(f)] = np.frombuffer(f, np.uint8)
    full = [bytes(arr[i]) for i in range(len(sel))]
    want = oracle.parse_frames(full)
    assert ((want["l4_nopt"] == 3) | (want["l4_nopt"] == 1)).sum() > 500
    got = engine.parse_to_numpy(FrameBatch.from_strided(arr))
    helpers.records_equal(got, want, full, f"tcp options stride={stride}")


def test_real_traffic_imix_full_size(engine, oracle):
    """16M frames of real-traffic TCP shapes: IMIX with timestamps, SACK
    blocks and MSS on TCP frames (the `tcp_ts` / `tcp_sack` / `tcp_mss`
    workload kinds, checksums stale so both verdicts occur), a 1M-frame mix
    tiled x16; records and sparse codes of a 65536-frame random sample equal
    the oracle's, and the sparse output expands to the 8-B output bit for
    bit at full size."""
    import torch
    base, counts = workloads.malformed_mix(engine, 1 << 20, seed=79, mutate_share=0.7,
                                           kinds=("tcp_ts", "tcp_sack", "tcp_mss"))
    assert min(counts[k] for k in ("tcp_ts", "tcp_sack", "tcp_mss")) > 150000
    b = workloads.tiled(base, 16)
    n = b.count
    assert n == 16 << 20
    rec = engine.parse(b, out_kind=abi.OUT_RECORD)
    sp = engine.parse(b, out_kind=abi.OUT_SPARSE)
    d8 = engine.parse(b, out_kind=abi.OUT_DESC)
    ex = engine.sparse_expand(b, sp)
    torch.cuda.synchronize()
    assert torch.equal(ex[: n * 8], d8[: n * 8])
    want = _sample_equal(oracle, b, rec, "real-traffic 16M sample")
    assert ((want["l4_nopt"] == 3) & ((want["flags"] & abi.C_L4_OK) == 0)).sum() > 1000
    assert ((want["l4_nopt"] == 1) & (want["l4_length"] == 24)).sum() > 100


def _sample_equal(oracle, b, rec, label, k=65536, seed=5):
    """Records of a random k-frame sample of a packed batch == the oracle's
    on the same bytes (gathered on the device); returns the oracle records."""
    import torch
    n = b.count
    idx = np.sort(np.random.default_rng(seed).choice(n, k, replace=False))
    offs = b.offsets.cpu().numpy().astype(np.int64)
    it = torch.from_numpy(idx).cuda()
    lo = torch.from_numpy(offs[idx]).cuda()
    ln = torch.from_numpy(offs[idx + 1] - offs[idx]).cuda()
    frames = []
    data = b.data
    for c in range(0, len(idx), 8192):  # gather the sampled frames' bytes on the device
        a, l = lo[c:c + 8192], ln[c:c + 8192]
        m = int(l.max().item())
        g = data[(a[:, None] + torch.arange(m, device="cuda")[None, :]).clamp(max=data.numel() - 1)]
        gc, lc = g.cpu().numpy(), l.cpu().numpy()
        frames += [bytes(gc[j, :lc[j]]) for j in range(len(lc))]
    want = oracle.parse_frames(frames)
    got = rec.view(torch.uint8).reshape(-1, 64)[it].cpu().numpy().reshape(-1).view(abi.RECORD_DTYPE)
    helpers.records_equal(got, want, frames, label)
    return want


def test_real_traffic_bench_batch(engine, oracle):
    """The batch bench.py's `real_traffic` object times (16M frames, TCP
    option lists on 70 % of the TCP segments, checksums fixed up on the device
    by nexg_recompute_checksums_batch): records of a 65536-frame sample equal
    the oracle's, the fixed-up checksums verify, and the grouped output (the
    bench's) expands to the 8-B descriptors bit for bit at full size."""
    import torch

    import bench
    b, desc = bench.real_traffic_batch(engine, 16 << 20, 0)
    n = b.count
    assert n == 16 << 20 and "checksums made valid" in desc
    rec = engine.parse(b, out_kind=abi.OUT_RECORD)
    gr = engine.parse(b, out_kind=abi.OUT_GROUPED)
    d8 = engine.parse(b, out_kind=abi.OUT_DESC)
    ex = engine.sparse_expand(b, gr, grouped=True)
    torch.cuda.synchronize()
    assert torch.equal(ex[: n * 8], d8[: n * 8])
    want = _sample_equal(oracle, b, rec, "real-traffic bench batch sample", seed=11)
    tcp = (want["flags"] & abi.L_TCP) != 0
    opt = tcp & (want["l4_nopt"] > 0)
    assert opt.sum() > 0.5 * tcp.sum()
    # every checksum the fix-up wrote verifies (IPv4 header and L4)
    l4c = (want["flags"] & abi.C_L4_CHECKED) != 0
    assert ((want["flags"][l4c] & abi.C_L4_OK) != 0).all()
