"""GPU: NEXG_OUT_SPARSE (1-B shape codes + per-64-frame exceptions) restores
the oracle's nexg_desc bit-exactly in every kernel layout and parse mode,
through both the device expander (nexg_sparse_expand) and the host decoder;
TwoPass (explicit lengths) takes the ctx tail scratch; full-size batches have
no exceptions and expand to exactly the 8-B descriptor output."""
import numpy as np
import pytest

from nex_amd import abi
from nex_amd.engine import FrameBatch
from nex_amd.frame import ParseMode, ParseOption
from tests import helpers

pytestmark = pytest.mark.gpu

MODES = [(ParseOption(), ParseMode.Lenient), (ParseOption(), ParseMode.Strict),
         (ParseOption(True, 14), ParseMode.Lenient), (ParseOption(unwrap_vlan=True), ParseMode.Lenient)]


def desc_of(recs):
    d = np.zeros(len(recs), abi.DESC_DTYPE)
    for n in abi.DESC_DTYPE.names:
        d[n] = recs[n]
    return d


@pytest.fixture(scope="module")
def corpus(oracle):
    base = ([bytes.fromhex(v["frame"]) for v in helpers.golden()["frames"]] + helpers.crafted_frames() +
            helpers.vlan_frames() + [oracle.gen_frame(abi.WL_IMIX, i) for i in range(200)] +
            [oracle.gen_frame(abi.WL_UDP64, i) for i in range(40)])
    return base + helpers.mutate_frames(np.random.default_rng(4242), base, 30000)


def layouts(frames):
    """packed (SpanTile), explicit lengths (TwoPass), explicit lengths with the
    monotone hint (SpanTile through gaps)."""
    b1 = FrameBatch.from_packed(frames, shift=4)
    b2 = FrameBatch.from_frames(frames, pad_to=4)
    b3 = FrameBatch.from_frames(frames, pad_to=16)
    b3.hints = abi.FRAMES_MONOTONE
    return [("packed", b1), ("lengths", b2), ("lengths+monotone", b3)]


@pytest.mark.parametrize("opt,mode", MODES, ids=lambda x: str(x))
def test_sparse_matches_oracle_every_layout(engine, oracle, corpus, opt, mode):
    import torch
    flags = opt.flags(mode)
    want = desc_of(oracle.parse_frames(corpus, flags, opt.offset))
    for name, batch in layouts(corpus):
        got = engine.parse_to_numpy(batch, opt, mode, abi.OUT_SPARSE)  # host decode
        helpers.records_equal(got, want, corpus, f"sparse {name} flags={flags}")
        raw = engine.parse(batch, opt, mode, abi.OUT_SPARSE)
        dev = engine.sparse_expand(batch, raw, opt, mode)  # device expand
        torch.cuda.synchronize()
        dev = dev.cpu().numpy()[: len(corpus) * 8].view(abi.DESC_DTYPE)
        helpers.records_equal(dev, want, corpus, f"sparse expand {name} flags={flags}")
        codes = raw.cpu().numpy()[: len(corpus)]
        assert (codes == 0).any() and (codes != 0).mean() > 0.5  # both paths exercised


@pytest.mark.parametrize("stride", [64, 128])
def test_sparse_fixed_strides(engine, oracle, corpus, stride):
    sel = [f for f in corpus if len(f) <= stride][:20000]
    arr = np.zeros((len(sel), stride), np.uint8)
    for i, f in enumerate(sel):
        arr[i, :len(f)] = np.frombuffer(f, np.uint8)
    full = [bytes(arr[i]) for i in range(len(sel))]
    want = desc_of(oracle.parse_frames(full))
    got = engine.parse_to_numpy(FrameBatch.from_strided(arr), out_kind=abi.OUT_SPARSE)
    helpers.records_equal(got, want, full, f"sparse stride={stride}")


@pytest.mark.parametrize("workload", [abi.WL_UDP64, abi.WL_IMIX])
def test_sparse_full_size_equals_desc(engine, workload):
    """configs[1] / configs[2] at full size: no exceptions, and the expanded
    codes equal the 8-B descriptor output of the same batch bit for bit."""
    import torch
    n = 16 << 20
    b = engine.gen_batch(workload, n)
    sp = engine.parse(b, out_kind=abi.OUT_SPARSE)
    d8 = engine.parse(b, out_kind=abi.OUT_DESC)
    ex = engine.sparse_expand(b, sp)
    torch.cuda.synchronize()
    assert (sp[:n] != 0).all().item()
    assert torch.equal(ex[: n * 8], d8[: n * 8])


def test_sparse_partial_groups_and_empty(engine, oracle):
    """Counts that are not multiples of 4 / 64 / 256 and the empty batch."""
    frames = [oracle.gen_frame(abi.WL_IMIX, i) for i in range(301)] + [b"", bytes(13)] * 3
    for n in (1, 3, 5, 63, 65, 257, len(frames)):
        fr = frames[:n]
        want = desc_of(oracle.parse_frames(fr))
        for name, batch in layouts(fr):
            got = engine.parse_to_numpy(batch, out_kind=abi.OUT_SPARSE)
            helpers.records_equal(got, want, fr, f"n={n} {name}")
    import torch
    e = engine.parse(FrameBatch(data=torch.zeros(16, dtype=torch.uint8, device="cuda"), count=0, stride=64),
                     out_kind=abi.OUT_SPARSE)
    assert e.numel() >= 16


def test_verdict_twopass_uses_scratch(engine, oracle, corpus):
    """NEXG_OUT_VERDICT on explicit lengths now runs the real TwoPass kernels
    (tail sums through the ctx scratch), not the lane-window fallback."""
    want = oracle.parse_frames(corpus)["flags"].astype(np.uint32)
    got = engine.parse_to_numpy(FrameBatch.from_frames(corpus, pad_to=4), out_kind=abi.OUT_VERDICT)
    assert (abi.verdict_to_flags(got["verdict"]) == want).all()


def test_monotone_hint_matches_twopass(engine, oracle):
    """The capture-file shape: 16-B record headers between frames in one
    buffer, offsets + lengths. With and without NEXG_FRAMES_MONOTONE (span vs
    two-pass kernels) every record equals the oracle's."""
    import torch
    frames = [oracle.gen_frame(abi.WL_IMIX, i) for i in range(20000)] + helpers.crafted_frames()
    blob, offs = bytearray(), []
    for f in frames:
        blob += bytes(16)  # record header
        offs.append(len(blob))
        blob += f
    data = torch.frombuffer(bytes(blob) + bytes(16), dtype=torch.uint8).cuda()
    ot = torch.tensor(offs, dtype=torch.int64, device="cuda")
    lt = torch.tensor([len(f) for f in frames], dtype=torch.int32, device="cuda")
    want = oracle.parse_frames(frames)
    for hints in (0, abi.FRAMES_MONOTONE):
        b = FrameBatch(data=data, count=len(frames), offsets=ot, lengths=lt, hints=hints)
        got = engine.parse_to_numpy(b, out_kind=abi.OUT_RECORD)
        helpers.records_equal(got, want, frames, f"pcap-shaped hints={hints}")
    # a wrong hint (scattered frames) costs speed, never correctness
    perm = np.random.default_rng(1).permutation(len(frames))
    b = FrameBatch(data=data, count=len(frames), offsets=ot[torch.from_numpy(perm).cuda()],
                   lengths=lt[torch.from_numpy(perm).cuda()], hints=abi.FRAMES_MONOTONE)
    got = engine.parse_to_numpy(b, out_kind=abi.OUT_RECORD)
    helpers.records_equal(got, want[perm], [frames[i] for i in perm], "scattered with hint")


@pytest.mark.parametrize("out_kind", [abi.OUT_RECORD, abi.OUT_SPARSE])
def test_unaligned_frames_take_fast_path_bit_exact(engine, oracle, out_kind):
    """Canonical IMIX frames at every byte alignment (0-3 byte gaps, offsets +
    lengths + monotone hint -> span kernel; without the hint -> two-pass), a
    share with a corrupted payload byte so both checksum verdicts occur, and
    windows straddling 16-KiB sub-tile edges: records equal the oracle's."""
    import torch
    rng = np.random.default_rng(99)
    frames = [bytearray(oracle.gen_frame(abi.WL_IMIX, i)) for i in range(30000)]
    for i in rng.choice(len(frames), 3000, replace=False):
        f = frames[i]
        f[int(rng.integers(40, len(f)))] ^= 0x5A
    frames = [bytes(f) for f in frames]
    gaps = rng.integers(0, 4, len(frames))
    blob, offs = bytearray(), []
    for f, g in zip(frames, gaps):
        blob += bytes(int(g))
        offs.append(len(blob))
        blob += f
    data = torch.frombuffer(bytes(blob) + bytes(16), dtype=torch.uint8).cuda()
    ot = torch.tensor(offs, dtype=torch.int64, device="cuda")
    lt = torch.tensor([len(f) for f in frames], dtype=torch.int32, device="cuda")
    want = oracle.parse_frames(frames)
    assert ((want["flags"] & abi.C_L4_OK) == 0).sum() > 1000
    if out_kind == abi.OUT_SPARSE:
        want = desc_of(want)
    for hints in (abi.FRAMES_MONOTONE, 0):
        b = FrameBatch(data=data, count=len(frames), offsets=ot, lengths=lt, hints=hints)
        got = engine.parse_to_numpy(b, out_kind=out_kind)
        helpers.records_equal(got, want, frames, f"unaligned hints={hints} out={out_kind}")


def test_record_gap_batches_match_oracle(engine, oracle):
    """gen_batch(record_gap=16): the capture-record layout bench.py's
    imix_pcap line times; every frame parses to the oracle's record of the
    generator's frame, through the span kernel (monotone hint)."""
    n = 20000
    b = engine.gen_batch(abi.WL_IMIX, n, record_gap=16)
    assert b.hints == abi.FRAMES_MONOTONE and b.lengths is not None
    frames = [oracle.gen_frame(abi.WL_IMIX, i) for i in range(n)]
    offs = b.offsets[:n].cpu().numpy()
    assert (np.diff(offs) == np.array([len(f) + 16 for f in frames[:-1]])).all() and offs[0] == 16
    want = oracle.parse_frames(frames)
    helpers.records_equal(engine.parse_to_numpy(b, out_kind=abi.OUT_RECORD), want, frames, "record gap")
    helpers.records_equal(engine.parse_to_numpy(b, out_kind=abi.OUT_SPARSE), desc_of(want), frames, "gap sparse")


def test_twopass_scratch_across_streams(engine, oracle, corpus):
    """narrow-output TwoPass parses hand their tail sums over
    through the one ctx scratch. Calls on one context from two streams are
    ordered by the context (an event per hand-over), so interleaved verdict /
    sparse parses of two different batches on two streams, with no sync in
    between, each equal the oracle."""
    import torch
    fa, fb = corpus[:20000], corpus[-20000:]
    ba, bb = FrameBatch.from_frames(fa, pad_to=4), FrameBatch.from_frames(fb, pad_to=4)
    wa, wb = oracle.parse_frames(fa), oracle.parse_frames(fb)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    outs = []
    for k in range(6):
        outs.append(("a", engine.parse(ba, out_kind=abi.OUT_VERDICT, stream=sa)))
        outs.append(("b", engine.parse(bb, out_kind=abi.OUT_VERDICT, stream=sb)))
        outs.append(("a", engine.parse(ba, out_kind=abi.OUT_SPARSE, stream=sa)))
        outs.append(("b", engine.parse(bb, out_kind=abi.OUT_SPARSE, stream=sb)))
    torch.cuda.synchronize()
    for k, (which, out) in enumerate(outs):
        frames, want, batch = (fa, wa, ba) if which == "a" else (fb, wb, bb)
        h = out.cpu().numpy()
        if k % 4 < 2:
            got = abi.verdict_to_flags(h[: 2 * len(frames)].view(abi.VERDICT_DTYPE)["verdict"])
            assert (got == want["flags"].astype(np.uint32)).all(), (k, which)
        else:
            d = abi.sparse_to_desc(h, batch.count, batch.frame_lengths())
            helpers.records_equal(d, desc_of(want), frames, f"stream {which} call {k}")
