"""GPU: NEXG_OUT_GROUPED (NEXG_OUT_SPARSE with each single-shape 64-frame
group stored as a head byte and two 64-bit verdict masks) restores the oracle's
nexg_desc bit-exactly in every kernel layout and parse mode, through the host
decoder and the device expander (nexg_grouped_expand): uniform groups with
both verdicts varying, groups one frame off uniform, mixed groups with
exceptions, partial last groups; full-size batches equal the 8-B descriptor
output and the 64-B workload is all uniform groups."""
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


def udp64_frames(oracle, n, seed):
    """64-B UDP frames, every 3rd with a corrupted payload byte (L4 verdict
    varies inside groups) and every 7th with a corrupted IPv4 header byte."""
    rng = np.random.default_rng(seed)
    fr = [bytearray(oracle.gen_frame(abi.WL_UDP64, i)) for i in range(n)]
    for f in fr[::3]:
        f[int(rng.integers(42, 64))] ^= 0x5A
    for f in fr[1::7]:
        f[24] ^= 0x01
    return [bytes(f) for f in fr]


@pytest.fixture(scope="module")
def corpus(oracle):
    base = ([bytes.fromhex(v["frame"]) for v in helpers.golden()["frames"]] + helpers.crafted_frames() +
            helpers.vlan_frames() + [oracle.gen_frame(abi.WL_IMIX, i) for i in range(200)])
    mixed = helpers.mutate_frames(np.random.default_rng(4243), base, 12000)
    uni = udp64_frames(oracle, 64 * 40, 1)
    uni[64 * 7 + 5] = mixed[0]  # a group one frame off uniform
    return uni + mixed + udp64_frames(oracle, 64 * 20 + 33, 2)


def layouts(frames):
    b1 = FrameBatch.from_packed(frames, shift=4)
    b2 = FrameBatch.from_frames(frames, pad_to=4)
    b3 = FrameBatch.from_frames(frames, pad_to=16)
    b3.hints = abi.FRAMES_MONOTONE
    return [("packed", b1), ("lengths", b2), ("lengths+monotone", b3)]


def marks(out, n):
    """per group: stored as a single-shape group (a head byte other than 0
    and NEXG_GROUPED_TILE_RUN, the two mixed forms)"""
    h = out.cpu().numpy()[: (n + 63) >> 6]
    return (h != 0) & (h != abi.GROUPED_TILE_RUN)


@pytest.mark.parametrize("opt,mode", MODES, ids=lambda x: str(x))
def test_grouped_matches_oracle_every_layout(engine, oracle, corpus, opt, mode):
    import torch
    flags = opt.flags(mode)
    want = desc_of(oracle.parse_frames(corpus, flags, opt.offset))
    for name, batch in layouts(corpus):
        got = engine.parse_to_numpy(batch, opt, mode, abi.OUT_GROUPED)  # host decode
        helpers.records_equal(got, want, corpus, f"grouped {name} flags={flags}")
        raw = engine.parse(batch, opt, mode, abi.OUT_GROUPED)
        dev = engine.sparse_expand(batch, raw, opt, mode, grouped=True)  # device expand
        torch.cuda.synchronize()
        dev = dev.cpu().numpy()[: len(corpus) * 8].view(abi.DESC_DTYPE)
        helpers.records_equal(dev, want, corpus, f"grouped expand {name} flags={flags}")
        h = marks(raw, len(corpus))
        assert (~h).sum() >= 100
        if name == "lengths":  # the lane kernel stores single-shape groups as such (the span kernel: all mixed)
            assert h.sum() >= 40
        else:  # the span kernel: every group mixed, exceptions in one run per 256-frame tile
            assert (raw.cpu().numpy()[: (len(corpus) + 63) >> 6] == abi.GROUPED_TILE_RUN).all()


@pytest.mark.parametrize("stride", [64, 128])
def test_grouped_fixed_strides(engine, oracle, corpus, stride):
    """The tile kernels (stride 64: the headline's register fast path)."""
    sel = [f for f in corpus if len(f) <= stride][:30000]
    arr = np.zeros((len(sel), stride), np.uint8)
    for i, f in enumerate(sel):
        arr[i, :len(f)] = np.frombuffer(f, np.uint8)
    full = [bytes(arr[i]) for i in range(len(sel))]
    want = desc_of(oracle.parse_frames(full))
    b = FrameBatch.from_strided(arr)
    got = engine.parse_to_numpy(b, out_kind=abi.OUT_GROUPED)
    helpers.records_equal(got, want, full, f"grouped stride={stride}")
    if stride == 64:
        assert marks(engine.parse(b, out_kind=abi.OUT_GROUPED), len(full)).sum() >= 40


@pytest.mark.parametrize("workload", [abi.WL_UDP64, abi.WL_IMIX])
def test_grouped_full_size_equals_desc(engine, workload):
    """configs[1] / configs[2] at full size: the expanded grouped output equals
    the 8-B descriptor output bit for bit; the 64-B batch is all single-shape
    groups (17 B per 64 frames written)."""
    import torch
    n = 16 << 20
    b = engine.gen_batch(workload, n)
    g = engine.parse(b, out_kind=abi.OUT_GROUPED)
    d8 = engine.parse(b, out_kind=abi.OUT_DESC)
    ex = engine.sparse_expand(b, g, grouped=True)
    torch.cuda.synchronize()
    assert torch.equal(ex[: n * 8], d8[: n * 8])
    if workload == abi.WL_UDP64:
        assert (g[: n >> 6] != 0).all().item()


def test_grouped_partial_groups_and_empty(engine, oracle):
    frames = udp64_frames(oracle, 130, 3) + [oracle.gen_frame(abi.WL_IMIX, i) for i in range(171)] + [b"", bytes(13)] * 3
    for n in (1, 3, 5, 63, 64, 65, 129, 257, len(frames)):
        fr = frames[:n]
        want = desc_of(oracle.parse_frames(fr))
        for name, batch in layouts(fr):
            got = engine.parse_to_numpy(batch, out_kind=abi.OUT_GROUPED)
            helpers.records_equal(got, want, fr, f"n={n} {name}")
        arr = np.zeros((n, 64), np.uint8)
        for i, f in enumerate(fr):
            arr[i, :min(len(f), 64)] = np.frombuffer(f[:64], np.uint8)
        full = [bytes(arr[i]) for i in range(n)]
        got = engine.parse_to_numpy(FrameBatch.from_strided(arr), out_kind=abi.OUT_GROUPED)
        helpers.records_equal(got, desc_of(oracle.parse_frames(full)), full, f"n={n} stride 64")
    import torch
    e = engine.parse(FrameBatch(data=torch.zeros(16, dtype=torch.uint8, device="cuda"), count=0, stride=64),
                     out_kind=abi.OUT_GROUPED)
    assert e.numel() >= 16
