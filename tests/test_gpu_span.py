"""GPU parity of the packed-span path (k_parse_span: offset table without a
lengths array, or a stride the tile kernels do not take) against the oracle's
batch parser on the very same layout (oracle/nex_oracle.c nexo_parse_batch).

The span kernel streams each 256-frame group's bytes through 16-KiB LDS
sub-tiles and derives L4 sums from chunk prefix sums, so the cases here aim at
its edges: frames crossing sub-tile edges, frames far longer than a sub-tile
(up to the 65535-B ceiling), odd frame starts (the batch base itself is 4-B
aligned, nexg.h), groups with a frame the layout rejects (BAD_EXTENT ->
per-frame fallback), partial last groups."""
import numpy as np
import pytest

from nex_amd import abi
from nex_amd.engine import FrameBatch
from tests import helpers

pytestmark = pytest.mark.gpu


def _big_frames(rng):
    """Checksum-valid long frames: IPv4/IPv6 x UDP/TCP, 1.5-64 KiB."""
    out = []
    for n in (1400, 4000, 9000, 16300, 16384, 20000, 40000, 65535 - 14 - 20 - 8):
        p = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        out.append(helpers._eth(helpers._ipv4(helpers._udp(p), 17)))
        q = p[: n - 12]
        out.append(helpers._eth(helpers._ipv4(helpers._tcp(q), 6)))
        if n + 40 + 8 <= 65535:
            out.append(helpers._eth(helpers._ipv6(helpers._udp(p[: n - 40]), 17), 0x86DD))
    return out


def _oracle_same_layout(oracle, batch, flags=0, ip_offset=0):
    data = batch.data.cpu().numpy()
    offs = batch.offsets.cpu().numpy().astype(np.uint64)
    return oracle.parse_packed(data, offs, None, flags=flags, ip_offset=ip_offset)


@pytest.fixture(scope="module")
def mixed(oracle):
    rng = np.random.default_rng(2024)
    g = helpers.golden()
    base = ([bytes.fromhex(v["frame"]) for v in g["frames"]] + helpers.crafted_frames() +
            [oracle.gen_frame(abi.WL_IMIX, i) for i in range(300)] + _big_frames(rng))
    frames = base + helpers.mutate_frames(rng, base, 6000)
    order = rng.permutation(len(frames))
    return [frames[i] for i in order]


@pytest.mark.parametrize("pad,shift", [(1, 0), (1, 4), (2, 8), (4, 0), (4, 12), (16, 4)])
def test_packed_offsets_only(engine, oracle, mixed, pad, shift):
    batch = FrameBatch.from_packed(mixed, pad_to=pad, shift=shift)
    want = _oracle_same_layout(oracle, batch)
    got = engine.parse_to_numpy(batch, out_kind=abi.OUT_RECORD)
    helpers.records_equal(got, want, None, f"packed pad={pad} shift={shift}")
    got_d = engine.parse_to_numpy(batch, out_kind=abi.OUT_DESC)
    for n in abi.DESC_DTYPE.names:
        assert (got_d[n] == want[n]).all(), n


@pytest.mark.parametrize("flags,ip_offset", [(abi.PARSE_STRICT, 0), (abi.PARSE_FROM_IP, 14),
                                             (abi.PARSE_FROM_IP | abi.PARSE_STRICT, 14)])
def test_packed_parse_options(engine, oracle, mixed, flags, ip_offset):
    from nex_amd.frame import ParseMode, ParseOption
    batch = FrameBatch.from_packed(mixed[:3000], pad_to=4)
    want = _oracle_same_layout(oracle, batch, flags, ip_offset)
    opt = ParseOption(bool(flags & abi.PARSE_FROM_IP), ip_offset)
    mode = ParseMode.Strict if flags & abi.PARSE_STRICT else ParseMode.Lenient
    got = engine.parse_to_numpy(batch, opt, mode, abi.OUT_RECORD)
    helpers.records_equal(got, want, None, f"packed flags={flags}")


def test_packed_bad_extent_group(engine, oracle, mixed):
    """A 70000-B gap in the offset table: that frame is BAD_EXTENT, its group
    falls back to per-frame parsing, every other group stays on spans."""
    import torch
    frames = mixed[:2000]
    batch = FrameBatch.from_packed(frames, pad_to=4)
    offs = batch.offsets.cpu().numpy().copy()
    data = batch.data.cpu().numpy()
    k = 700
    grown = np.concatenate([data[:offs[k + 1]], np.zeros(70000, np.uint8), data[offs[k + 1]:]])
    offs[k + 1:] += 70000
    b2 = FrameBatch(data=torch.from_numpy(grown).cuda(), count=len(frames),
                    offsets=torch.from_numpy(offs).cuda())
    want = oracle.parse_packed(grown, offs.astype(np.uint64), None)
    assert abi.status_of(np.array([want["flags"][k]]))[0] == abi.ERR_BAD_EXTENT
    got = engine.parse_to_numpy(b2, out_kind=abi.OUT_RECORD)
    helpers.records_equal(got, want, None, "bad extent group")
    # the fallback group's grouped / sparse stores (a tile run of exceptions in
    # the grouped form, the per-group run in the sparse one), host-decoded
    for kind in (abi.OUT_GROUPED, abi.OUT_SPARSE):
        got_d = engine.parse_to_numpy(b2, out_kind=kind)
        for n in abi.DESC_DTYPE.names:
            assert (got_d[n] == want[n]).all(), (kind, n)


@pytest.mark.parametrize("stride", [144, 200, 1518])
def test_wide_stride_spans(engine, oracle, mixed, stride):
    """Fixed strides the tile kernels do not take go through spans too."""
    sel = [f for f in mixed if len(f) <= stride][:4000]
    rng = np.random.default_rng(stride)
    arr = rng.integers(0, 256, (len(sel), stride), dtype=np.uint8)
    for i, f in enumerate(sel):
        arr[i, :len(f)] = np.frombuffer(f, np.uint8)
    full = [bytes(arr[i]) for i in range(len(sel))]
    want = oracle.parse_frames(full)
    got = engine.parse_to_numpy(FrameBatch.from_strided(arr))
    helpers.records_equal(got, want, full, f"stride={stride}")


@pytest.mark.parametrize("count", [1, 255, 257, 1000])
def test_partial_groups(engine, oracle, mixed, count):
    batch = FrameBatch.from_packed(mixed[:count], pad_to=2, shift=4)
    want = _oracle_same_layout(oracle, batch)
    got = engine.parse_to_numpy(batch, out_kind=abi.OUT_RECORD)
    helpers.records_equal(got, want, None, f"count={count}")


class _ShiftedOffsets:
    """An offset table copied to `shift` bytes past a 16-B aligned device
    buffer: FrameBatch.to_c reads only data_ptr()."""

    def __init__(self, offsets, shift):
        import torch
        n = offsets.numel() * 8
        self.buf = torch.zeros(n + 16, dtype=torch.uint8, device=offsets.device)
        self.buf[shift: shift + n].copy_(offsets.view(torch.uint8))
        self.shift = shift

    def data_ptr(self):
        return self.buf.data_ptr() + self.shift


@pytest.mark.parametrize("shift", [4, 1])
def test_packed_offsets_table_alignment(engine, mixed, shift):
    """An offset table at 4 mod 8 or at an odd address gives the aligned
    table's output (the span kernel reads it with per-lane loads; scalar loads
    of its span bounds would need dword alignment and measured 0.1-0.5 %
    slower, profiles/r05/scalar_bounds_ab.log)."""
    batch = FrameBatch.from_packed(mixed, pad_to=1, shift=0)
    moved = FrameBatch(data=batch.data, count=batch.count, offsets=_ShiftedOffsets(batch.offsets, shift))
    import torch
    for kind in (abi.OUT_RECORD, abi.OUT_GROUPED, abi.OUT_DESC):
        n = max(engine.out_bytes(kind, batch.count), 16)
        want, got = (torch.zeros(n, dtype=torch.uint8, device=batch.data.device) for _ in range(2))
        engine.parse(batch, out_kind=kind, out=want)
        engine.parse(moved, out_kind=kind, out=got)
        assert torch.equal(got, want), kind


@pytest.mark.parametrize("layout", ["packed", "udp64"])
def test_desc_output_at_8_mod_16(engine, mixed, layout):
    """NEXG_OUT_DESC into an output at 8 mod 16 (the API asks 8-B alignment):
    the span kernel's paired 16-B copy-out falls back to 8-B stores there;
    the descriptors equal the aligned output's, and nothing past the last
    one is written."""
    import torch
    batch = (FrameBatch.from_packed(mixed, pad_to=1, shift=0) if layout == "packed"
             else engine.gen_batch(abi.WL_UDP64, 70_001))
    n = engine.out_bytes(abi.OUT_DESC, batch.count)
    want = torch.zeros(n, dtype=torch.uint8, device=batch.data.device)
    buf = torch.full((n + 32,), 0xA5, dtype=torch.uint8, device=batch.data.device)
    assert buf.data_ptr() % 16 == 0
    engine.parse(batch, out_kind=abi.OUT_DESC, out=want)
    engine.parse(batch, out_kind=abi.OUT_DESC, out=buf[8: 8 + n])
    torch.cuda.synchronize()
    assert torch.equal(buf[8: 8 + n], want)
    assert bool((buf[:8] == 0xA5).all()) and bool((buf[8 + n:] == 0xA5).all())


def test_offsets32_small_layouts(engine, mixed):
    """NEXG_FRAMES_OFFSETS32 under 4 GiB (no group bases): packed, packed at
    an unaligned start, offsets + lengths with and without the monotone hint
    give the u64 table's outputs in every output kind, and the checksum batch
    and the fix-up read the same frames."""
    import torch
    for b64 in (FrameBatch.from_packed(mixed, pad_to=1, shift=0), FrameBatch.from_packed(mixed, pad_to=4, shift=12),
                FrameBatch.from_frames(mixed)):
        for hints in ((0, abi.FRAMES_MONOTONE) if b64.lengths is not None else (0,)):
            b64.hints = hints
            b32 = b64.with_offsets32()
            assert b32.hints & abi.FRAMES_OFFSETS32
            for kind in (abi.OUT_RECORD, abi.OUT_GROUPED, abi.OUT_DESC, abi.OUT_SPARSE, abi.OUT_FLAGS):
                n = max(engine.out_bytes(kind, b64.count), 16)
                want, got = (torch.zeros(n, dtype=torch.uint8, device="cuda") for _ in range(2))
                engine.parse(b64, out_kind=kind, out=want)
                engine.parse(b32, out_kind=kind, out=got)
                assert torch.equal(got, want), (kind, hints)
            assert torch.equal(engine.checksum(b32, 5), engine.checksum(b64, 5))


def test_offsets32_imix_over_4gib(engine):
    """The 16M IMIX batch (5.95 GB, past 4 GiB: the table's group bases carry
    the high bits) with a u32 table: the grouped output equals the u64
    table's byte for byte, and the descriptors too."""
    import torch
    b64 = engine.gen_batch(abi.WL_IMIX, 16 << 20)
    assert b64.data.numel() > 0xFFFFFFFF
    b32 = b64.with_offsets32()
    assert b32.offsets.numel() == abi.offsets32_layout(b64.count, True)[3]
    assert b32.total_bytes == b64.total_bytes
    for kind in (abi.OUT_GROUPED, abi.OUT_DESC):
        n = engine.out_bytes(kind, b64.count)
        # (zeroed: the grouped layout writes exception slots only where frames have one)
        want = torch.zeros(n, dtype=torch.uint8, device="cuda")
        got = torch.zeros(n, dtype=torch.uint8, device="cuda")
        engine.parse(b64, out_kind=kind, out=want)
        engine.parse(b32, out_kind=kind, out=got)
        torch.cuda.synchronize()
        assert torch.equal(got, want), kind
        del want, got
