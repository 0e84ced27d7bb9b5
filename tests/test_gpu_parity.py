"""GPU parity: the gfx950 kernels (through the C ABI) against the oracle.

Bit-exact on every record/descriptor field: this is integer/byte work, there
is no tolerance. Small cases compare every frame; full-size (16M-frame)
batches compare a random sample plus size-independent properties."""
import numpy as np
import pytest

from nex_amd import abi
from nex_amd.engine import FrameBatch
from nex_amd.frame import ParseMode, ParseOption
from tests import helpers

pytestmark = pytest.mark.gpu

FLAGS = [(ParseOption(), ParseMode.Lenient), (ParseOption(), ParseMode.Strict),
         (ParseOption(True, 14), ParseMode.Lenient), (ParseOption(True, 14), ParseMode.Strict)]


def desc_of(recs):
    d = np.zeros(len(recs), abi.DESC_DTYPE)
    for n in abi.DESC_DTYPE.names:
        d[n] = recs[n]
    return d


@pytest.fixture(scope="module")
def corpus(oracle):
    g = helpers.golden()
    base = ([bytes.fromhex(v["frame"]) for v in g["frames"]] + helpers.crafted_frames() +
            [oracle.gen_frame(abi.WL_IMIX, i) for i in range(60)] +
            [oracle.gen_frame(abi.WL_UDP64, i) for i in range(20)])
    rng = np.random.default_rng(99)
    return base + helpers.mutate_frames(rng, base, 30000)


def test_golden_frames_on_gpu(engine, oracle):
    g = helpers.golden()["frames"]
    for v in g:
        fr = bytes.fromhex(v["frame"])
        opt = ParseOption(bool(v["parse_flags"] & abi.PARSE_FROM_IP), v["ip_offset"])
        mode = ParseMode.Strict if v["parse_flags"] & abi.PARSE_STRICT else ParseMode.Lenient
        rec = engine.parse_to_numpy(FrameBatch.from_frames([fr]), opt, mode)[0]
        helpers.check_expect(rec, fr, v["expect"], v["name"],
                             reparse=lambda b: engine.parse_to_numpy(FrameBatch.from_frames([b]), opt, mode)[0])
        want = oracle.parse_frame(fr, v["parse_flags"], v["ip_offset"])
        assert rec.tobytes() == want.tobytes(), v["name"]


@pytest.mark.parametrize("pad", [1, 4, 16])
@pytest.mark.parametrize("opt,mode", FLAGS, ids=lambda x: str(x))
def test_packed_mix_matches_oracle(engine, oracle, corpus, pad, opt, mode):
    batch = FrameBatch.from_frames(corpus, pad_to=pad)
    flags = opt.flags(mode)
    want = oracle.parse_frames(corpus, flags, opt.offset)
    got = engine.parse_to_numpy(batch, opt, mode, abi.OUT_RECORD)
    helpers.records_equal(got, want, corpus, f"packed pad={pad} flags={flags}")
    got_d = engine.parse_to_numpy(batch, opt, mode, abi.OUT_DESC)
    helpers.records_equal(got_d, desc_of(want), corpus, "desc")


@pytest.mark.parametrize("stride", [64, 128, 96, 80, 200])
def test_fixed_stride_matches_oracle(engine, oracle, corpus, stride):
    rng = np.random.default_rng(stride)
    sel = [f for f in corpus if len(f) <= stride][:20000]
    arr = np.zeros((len(sel), stride), np.uint8)
    fill = rng.integers(0, 256, arr.shape, dtype=np.uint8)  # bytes past each frame: junk
    arr[:] = fill
    for i, f in enumerate(sel):
        arr[i, :len(f)] = np.frombuffer(f, np.uint8)
    lens = np.array([len(f) for f in sel], np.int32)
    want = oracle.parse_frames(sel)
    got = engine.parse_to_numpy(FrameBatch.from_strided(arr, lengths=lens))
    helpers.records_equal(got, want, sel, f"stride={stride} with lengths")
    full = [bytes(arr[i]) for i in range(len(sel))]
    want = oracle.parse_frames(full)
    got = engine.parse_to_numpy(FrameBatch.from_strided(arr))
    helpers.records_equal(got, want, full, f"stride={stride} full")
    # NEXG_OUT_DESC: staged through LDS, two descriptors per 16-B store; a
    # ragged last tile (odd frame count) ends in one 8-B store
    for m in (len(full), len(full) - 1 - (len(full) % 2 == 0)):
        got_d = engine.parse_to_numpy(FrameBatch.from_strided(arr[:m]), out_kind=abi.OUT_DESC)
        helpers.records_equal(got_d, desc_of(want[:m]), full[:m], f"stride={stride} desc count={m}")


def test_generators_match_oracle(engine, oracle):
    import torch
    n = 3000
    b = engine.gen_batch(abi.WL_UDP64, n, first_index=12345)
    torch.cuda.synchronize()
    data = b.data.cpu().numpy()
    for i in range(0, n, 7):
        assert bytes(data[i * 64:(i + 1) * 64]) == oracle.gen_frame(abi.WL_UDP64, 12345 + i), i
    b = engine.gen_batch(abi.WL_IMIX, n, first_index=777)
    offs = b.offsets.cpu().numpy()
    data = b.data.cpu().numpy()
    for i in range(0, n, 3):
        assert bytes(data[offs[i]:offs[i + 1]]) == oracle.gen_frame(abi.WL_IMIX, 777 + i), i
    p = [t.cpu().numpy() for t in engine.gen_udp4_params(100, first_index=5)]
    for i in range(100):
        want = oracle.gen_udp4_params(5 + i)
        got = (int(p[0][i]) & 0xFFFFFFFF, int(p[1][i]) & 0xFFFFFFFF, int(p[2][i]) & 0xFFFF,
               int(p[3][i]) & 0xFFFF, int(p[4][i]) & 0xFFFF)
        assert got == want


@pytest.mark.parametrize("workload,count", [(abi.WL_UDP64, 16 << 20), (abi.WL_IMIX, 16 << 20),
                                            (abi.WL_UDP64, 52 << 20)])
def test_full_size_sampled(engine, oracle, workload, count):
    """BASELINE.json full sizes: sample 65536 frames bit-exact + properties.
    52M x 64 B is 3.25 GiB."""
    import torch
    b = engine.gen_batch(workload, count)
    desc = engine.parse(b, out_kind=abi.OUT_DESC)
    torch.cuda.synchronize()
    d = desc.cpu().numpy().view(abi.DESC_DTYPE)
    f = d["flags"]
    assert (abi.status_of(f) == 0).all()
    assert (f & abi.C_L4_CHECKED).all()
    bad = ((f & abi.C_L4_OK) == 0) | (((f & abi.C_IP_CHECKED) != 0) & ((f & abi.C_IP_OK) == 0))
    assert abs(bad.mean() - 1 / 16) < 0.002
    rng = np.random.default_rng(workload)
    idx = np.sort(rng.choice(count, 65536, replace=False))
    if workload == abi.WL_UDP64:
        assert (d["payload_len"] == 22).all() and (d["payload_off"] == 42).all()
        raw = b.data.cpu().numpy().reshape(count, 64)[idx]
        frames = [bytes(r) for r in raw]
    else:
        offs = b.offsets.cpu().numpy()
        data = b.data.cpu().numpy()
        frames = [bytes(data[offs[i]:offs[i + 1]]) for i in idx]
    want = oracle.parse_frames(frames)
    helpers.records_equal(d[idx], desc_of(want), frames, "full-size sample")
    # generated frames are exactly the oracle generator's
    for k in range(0, 65536, 4096):
        assert frames[k] == oracle.gen_frame(workload, int(idx[k]))


def test_checksum_batch_kats(engine, oracle):
    util = helpers.golden()["util"]
    bufs = [bytes.fromhex(v["data"]) for v in util["checksum"]]
    got = engine.checksum(FrameBatch.from_frames(bufs), 2**32 - 1).cpu().numpy().astype(np.uint16)
    assert list(got) == [v["checksum"] for v in util["checksum"]]
    rng = np.random.default_rng(3)
    bufs = [bytes(rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8)) for _ in range(5000)]
    for skip in (0, 1, 5, 70, 2**32 - 1):
        got = engine.checksum(FrameBatch.from_frames(bufs, pad_to=1), skip).cpu().numpy().astype(np.uint16)
        want = [oracle.checksum(x, skip) for x in bufs]
        assert list(got) == want, skip
    # KAT: checksum(0..11, 1) == !sum_be_words == !7190 (util.rs:193)
    got = engine.checksum(FrameBatch.from_frames([bytes(range(11))]), 1).cpu().numpy().astype(np.uint16)
    assert int(got[0]) == (~7190) & 0xFFFF


@pytest.mark.parametrize("payload_len", [0, 5, 22])
def test_build_udp4_matches_oracle(engine, oracle, payload_len):
    import torch
    n = 20000
    p = engine.gen_udp4_params(n, first_index=42)
    payload = bytes(range(7, 7 + payload_len))
    pt = torch.tensor(list(payload), dtype=torch.uint8, device="cuda") if payload_len else None
    smac, dmac = bytes([2, 0, 0, 0, 0, 1]), bytes([2, 0, 0, 0, 0, 2])
    out = engine.build_udp4(p[0], p[1], p[2], p[3], p[4], src_mac=smac, dst_mac=dmac, ttl=64,
                            ip_flags=2, payload=pt)
    torch.cuda.synchronize()
    L = 42 + payload_len
    data = out.cpu().numpy()[: n * L].reshape(n, L)
    host = [t.cpu().numpy() for t in p]
    for i in range(0, n, 97):
        want = oracle.build_udp4(smac, dmac, int(host[0][i]) & 0xFFFFFFFF, int(host[1][i]) & 0xFFFFFFFF,
                                 int(host[2][i]) & 0xFFFF, int(host[3][i]) & 0xFFFF,
                                 int(host[4][i]) & 0xFFFF, 64, 2, 0, payload)
        assert bytes(data[i]) == want, i
    # every built frame verifies through the GPU parse path
    recs = engine.parse_to_numpy(FrameBatch(data=out, count=n, stride=L), out_kind=abi.OUT_DESC)
    assert ((recs["flags"] & (abi.C_IP_OK | abi.C_L4_OK)) == (abi.C_IP_OK | abi.C_L4_OK)).all()


@pytest.mark.parametrize("payload_len,stride", [(0, None), (0, 64), (0, 63), (5, None), (22, 130),
                                                (1, 65)])
def test_build_udp6_matches_oracle(engine, oracle, payload_len, stride):
    """udp_ping's IPv6 branch on the GPU == the oracle, byte for byte, in the
    LDS-staged (even / odd stride) and direct (stride > 128) kernels."""
    import torch
    n = 5000
    rng = np.random.default_rng(payload_len * 1000 + (stride or 0))
    src = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    dst = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    sp = rng.integers(0, 65536, n).astype(np.uint16)
    dp = rng.integers(0, 65536, n).astype(np.uint16)
    payload = bytes(rng.integers(0, 256, payload_len, dtype=np.uint8))
    pt = torch.tensor(list(payload), dtype=torch.uint8, device="cuda") if payload_len else None
    smac, dmac = bytes([2, 0, 0, 0, 0, 1]), bytes([2, 0, 0, 0, 0, 2])
    L = 62 + payload_len
    S = stride or L
    out = engine.build_udp6(torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda(),
                            torch.from_numpy(sp.view(np.int16)).cuda(),
                            torch.from_numpy(dp.view(np.int16)).cuda(), src_mac=smac, dst_mac=dmac,
                            hop_limit=61, traffic_class=0x3C, flow_label=0xABCDE, payload=pt,
                            out_stride=S)
    torch.cuda.synchronize()
    data = out.cpu().numpy()[: n * S].reshape(n, S)
    for i in range(0, n, 13):
        want = oracle.build_udp6(smac, dmac, bytes(src[i]), bytes(dst[i]), int(sp[i]), int(dp[i]),
                                 61, 0x3C, 0xABCDE, payload)
        assert bytes(data[i, :L]) == want, i
        if S > L and S <= 128:
            assert not data[i, L:].any(), i  # staged tiles zero the gap
    recs = engine.parse_to_numpy(FrameBatch.from_strided(np.ascontiguousarray(data[:, :L])),
                                 out_kind=abi.OUT_DESC)
    assert (recs["flags"] & abi.C_L4_OK).all()


@pytest.mark.parametrize("stride", [43, 64, 200])
def test_build_udp4_strides(engine, oracle, stride):
    import torch
    n = 3000
    p = engine.gen_udp4_params(n, first_index=7)
    smac, dmac = bytes([2, 0, 0, 0, 0, 1]), bytes([2, 0, 0, 0, 0, 2])
    out = engine.build_udp4(p[0], p[1], p[2], p[3], p[4], src_mac=smac, dst_mac=dmac, ttl=64,
                            ip_flags=2, out_stride=stride)
    torch.cuda.synchronize()
    data = out.cpu().numpy()[: n * stride].reshape(n, stride)
    host = [t.cpu().numpy() for t in p]
    for i in range(0, n, 11):
        want = oracle.build_udp4(smac, dmac, int(host[0][i]) & 0xFFFFFFFF, int(host[1][i]) & 0xFFFFFFFF,
                                 int(host[2][i]) & 0xFFFF, int(host[3][i]) & 0xFFFF,
                                 int(host[4][i]) & 0xFFFF, 64, 2, 0, b"")
        assert bytes(data[i, :42]) == want, i


def test_udp_ping_golden_on_gpu(engine):
    import torch
    from nex_amd.engine import u32_tensor
    b = helpers.golden()["build"][0]
    ip = lambda s: int.from_bytes(bytes(map(int, s.split("."))), "big")
    out = engine.build_udp4(u32_tensor([ip(b["src_ip"])]), u32_tensor([ip(b["dst_ip"])]),
                            def_src_port=b["sport"], def_dst_port=b["dport"], ip_flags=b["ip_flags"])
    torch.cuda.synchronize()
    f = bytes(out.cpu().numpy()[:42])
    assert f.hex() == "00000000000000000000000008004500001c00004000401176c3c0a8016401010101d0c3829b0008e870"


def test_bad_extent_and_empty(engine):
    import torch
    data = torch.zeros(100, dtype=torch.uint8, device="cuda")
    offs = torch.tensor([0, 90, 200], dtype=torch.int64, device="cuda")
    lens = torch.tensor([64, 20, 4], dtype=torch.int32, device="cuda")
    d = engine.parse_to_numpy(FrameBatch(data=data, count=3, offsets=offs, lengths=lens), out_kind=abi.OUT_DESC)
    assert list(abi.status_of(d["flags"])) == [0, abi.ERR_BAD_EXTENT, abi.ERR_BAD_EXTENT]
    d = engine.parse_to_numpy(FrameBatch(data=data, count=0, stride=64), out_kind=abi.OUT_DESC)
    assert len(d) == 0


def test_pcap_ingest_to_gpu_parse(engine, oracle, tmp_path):
    """Capture file -> native batch reader (pinned) -> H2D -> span parse ==
    the oracle on the same frames (SURVEY.md 8(f)2 ingest path)."""
    from nex_amd.ingest import PcapReader, device_batches
    from tests import pcapfile
    frames = [oracle.gen_frame(abi.WL_IMIX, i) for i in range(3000)] + helpers.crafted_frames()[1:]
    path = tmp_path / "x.pcapng"
    blob = pcapfile.ng_shb() + pcapfile.ng_idb(1)
    blob += b"".join(pcapfile.ng_epb(f, i) for i, f in enumerate(frames))
    path.write_bytes(blob)
    got = []
    with PcapReader(str(path)) as r:
        for b in device_batches(r, max_frames=1000, data_cap=1 << 20):
            got.append(engine.parse_to_numpy(b, out_kind=abi.OUT_RECORD))
    got = np.concatenate(got)
    helpers.records_equal(got, oracle.parse_frames(frames), frames, "pcap ingest")


@pytest.mark.parametrize("fmt", ["classic", "pcapng"])
def test_pcap_mapped_ingest_to_gpu_parse(engine, oracle, tmp_path, fmt):
    """Zero-copy capture ingest (nexg_pcap_map: the page-cache mapping
    registered for DMA, windows of records copied H2D in place, offsets +
    lengths + monotone hint) -> span parse == the oracle, with windows that
    cut records (several batches)."""
    from nex_amd.ingest import PcapReader, device_mapped_batches
    from tests import pcapfile
    frames = [oracle.gen_frame(abi.WL_IMIX, i) for i in range(3000)] + helpers.crafted_frames()[1:]
    path = tmp_path / ("x.pcap" if fmt == "classic" else "x.pcapng")
    if fmt == "classic":
        path.write_bytes(pcapfile.classic(frames))
    else:
        blob = pcapfile.ng_shb() + pcapfile.ng_idb(1)
        path.write_bytes(blob + b"".join(pcapfile.ng_epb(f, i) for i, f in enumerate(frames)))
    got, batches = [], 0
    with PcapReader(str(path)) as r:
        for b in device_mapped_batches(r, max_frames=700, window=1 << 18):
            got.append(engine.parse_to_numpy(b, out_kind=abi.OUT_RECORD))
            batches += 1
    got = np.concatenate(got)
    assert batches > 3
    helpers.records_equal(got, oracle.parse_frames(frames), frames, f"mapped ingest {fmt}")


@pytest.mark.parametrize("flags", [abi.PARSE_VLAN, abi.PARSE_VLAN | abi.PARSE_STRICT])
def test_vlan_extension_on_gpu(engine, oracle, corpus, flags):
    """NEXG_PARSE_VLAN in every kernel variant == the oracle's extension."""
    from nex_amd.frame import ParseMode, ParseOption
    frames = corpus[:8000] + helpers.vlan_frames() * 20
    opt = ParseOption(unwrap_vlan=True)
    mode = ParseMode.Strict if flags & abi.PARSE_STRICT else ParseMode.Lenient
    for batch in (FrameBatch.from_frames(frames, pad_to=4), FrameBatch.from_packed(frames, pad_to=2)):
        data = batch.data.cpu().numpy()
        offs = batch.offsets.cpu().numpy().astype(np.uint64)
        lens = None if batch.lengths is None else batch.lengths.cpu().numpy().astype(np.uint32)
        want = oracle.parse_packed(data, offs, lens, flags=flags)
        got = engine.parse_to_numpy(batch, opt, mode, abi.OUT_RECORD)
        helpers.records_equal(got, want, None, f"vlan lengths={lens is not None}")
    for stride in (64, 128):
        sel = [f for f in frames if len(f) <= stride][:6000]
        arr = np.zeros((len(sel), stride), np.uint8)
        for i, f in enumerate(sel):
            arr[i, :len(f)] = np.frombuffer(f, np.uint8)
        want = oracle.parse_packed(arr.reshape(-1), stride=stride, flags=flags)
        got = engine.parse_to_numpy(FrameBatch.from_strided(arr), opt, mode, abi.OUT_RECORD)
        helpers.records_equal(got, want, None, f"vlan stride={stride}")


def flags_of(recs):
    d = np.zeros(len(recs), abi.FLAGS_DTYPE)
    d["flags"] = recs["flags"]
    return d


def test_flags_output_matches_oracle(engine, oracle, corpus):
    """NEXG_OUT_FLAGS (4 B: nexg_desc.flags alone) in every kernel layout:
    packed (SpanTile), explicit lengths (TwoPass), fixed strides 64
    (TileStride64 fast path) and 128 (TileStride)."""
    import torch
    want = oracle.parse_frames(corpus)
    got = engine.parse_to_numpy(FrameBatch.from_packed(corpus, shift=4), out_kind=abi.OUT_FLAGS)
    assert got.dtype == abi.FLAGS_DTYPE and len(got) == len(corpus)
    helpers.records_equal(got, flags_of(want), corpus, "flags packed")
    got = engine.parse_to_numpy(FrameBatch.from_frames(corpus, pad_to=4), out_kind=abi.OUT_FLAGS)
    helpers.records_equal(got, flags_of(want), corpus, "flags explicit lengths")
    for stride in (64, 128):
        sel = [f for f in corpus if len(f) <= stride][:20000]
        arr = np.zeros((len(sel), stride), np.uint8)
        for i, f in enumerate(sel):
            arr[i, :len(f)] = np.frombuffer(f, np.uint8)
        full = [bytes(arr[i]) for i in range(len(sel))]
        got = engine.parse_to_numpy(FrameBatch.from_strided(arr), out_kind=abi.OUT_FLAGS)
        helpers.records_equal(got, flags_of(oracle.parse_frames(full)), full, f"flags stride={stride}")
    b = engine.gen_batch(abi.WL_UDP64, 1 << 20)
    f4 = engine.parse(b, out_kind=abi.OUT_FLAGS)
    d8 = engine.parse(b, out_kind=abi.OUT_DESC)
    torch.cuda.synchronize()
    assert (f4.cpu().numpy().view("<u4") == d8.cpu().numpy().view(abi.DESC_DTYPE)["flags"]).all()


def test_verdict_output_matches_oracle(engine, oracle, corpus):
    """NEXG_OUT_VERDICT (2 B) decodes to the oracle's flags word exactly, in
    every layout (packed, explicit lengths -> lane window, strides 64 / 128)
    and in strict / from-IP modes, where error statuses are common."""
    import torch
    for mode, opt in ((ParseMode.Lenient, ParseOption()), (ParseMode.Strict, ParseOption()),
                      (ParseMode.Lenient, ParseOption(True, 14))):
        want = oracle.parse_frames(corpus, opt.flags(mode), opt.offset)["flags"].astype(np.uint32)
        for batch in (FrameBatch.from_packed(corpus, shift=4), FrameBatch.from_frames(corpus, pad_to=4)):
            got = engine.parse_to_numpy(batch, opt, mode, out_kind=abi.OUT_VERDICT)
            assert got.dtype == abi.VERDICT_DTYPE and len(got) == len(corpus)
            bad = np.nonzero(abi.verdict_to_flags(got["verdict"]) != want)[0]
            assert len(bad) == 0, (mode, opt, batch.count, bad[:8])
        assert (want >> abi.STATUS_SHIFT).any()
    for stride in (64, 128):
        sel = [f for f in corpus if len(f) <= stride][:20000]
        arr = np.zeros((len(sel), stride), np.uint8)
        for i, f in enumerate(sel):
            arr[i, :len(f)] = np.frombuffer(f, np.uint8)
        full = [bytes(arr[i]) for i in range(len(sel))]
        got = engine.parse_to_numpy(FrameBatch.from_strided(arr), out_kind=abi.OUT_VERDICT)
        assert (abi.verdict_to_flags(got["verdict"]) == oracle.parse_frames(full)["flags"]).all(), stride
    b = engine.gen_batch(abi.WL_UDP64, 1 << 20)
    v2 = engine.parse(b, out_kind=abi.OUT_VERDICT)
    d8 = engine.parse(b, out_kind=abi.OUT_DESC)
    torch.cuda.synchronize()
    assert (abi.verdict_to_flags(v2.cpu().numpy().view("<u2")) ==
            d8.cpu().numpy().view(abi.DESC_DTYPE)["flags"]).all()


def test_build_udp4_default_fields(engine, oracle):
    """The general builder form (ports / id from the batch defaults) next to
    the all-arrays form the udp_ping bench takes: same bytes as the oracle."""
    import torch
    n = 5000
    p = engine.gen_udp4_params(n, first_index=9)
    smac, dmac = bytes([2, 0, 0, 0, 0, 1]), bytes([2, 0, 0, 0, 0, 2])
    host = [t.cpu().numpy() for t in p]
    for kw, pick in (({"src_port": p[2]}, lambda i: (int(host[2][i]) & 0xFFFF, 33435, 7)),
                     ({"dst_port": p[3], "ip_id": p[4]},
                      lambda i: (53443, int(host[3][i]) & 0xFFFF, int(host[4][i]) & 0xFFFF)),
                     ({}, lambda i: (53443, 33435, 7))):
        out = engine.build_udp4(p[0], p[1], def_src_port=53443, def_dst_port=33435, def_ip_id=7,
                                src_mac=smac, dst_mac=dmac, ttl=64, ip_flags=2, **kw)
        torch.cuda.synchronize()
        data = out.cpu().numpy()[: n * 42].reshape(n, 42)
        for i in range(0, n, 31):
            sp, dp, ident = pick(i)
            want = oracle.build_udp4(smac, dmac, int(host[0][i]) & 0xFFFFFFFF, int(host[1][i]) & 0xFFFFFFFF,
                                     sp, dp, ident, 64, 2, 0, b"")
            assert bytes(data[i]) == want, (sorted(kw), i)
    # the udp_ping probe batch (src_ip NULL: one source, ports and id from the
    # defaults, a destination per frame), at the full-tile and a ragged count
    for m in (n, 257):
        out = engine.build_udp4(None, p[1][:m], def_src_ip=0xC0A80164, def_src_port=53443, def_dst_port=33435,
                                src_mac=smac, dst_mac=dmac, ttl=64, ip_flags=2)
        torch.cuda.synchronize()
        data = out.cpu().numpy()[: m * 42].reshape(m, 42)
        for i in list(range(0, m, 29)) + [m - 1]:
            want = oracle.build_udp4(smac, dmac, 0xC0A80164, int(host[1][i]) & 0xFFFFFFFF,
                                     53443, 33435, 0, 64, 2, 0, b"")
            assert bytes(data[i]) == want, ("probe", m, i)


@pytest.mark.parametrize("tiles", [3, 8 * 16 * 2 + 5])
def test_probe_stream(engine, tiles):
    """nexg_probe_stream (calibration): both output shapes against numpy, at
    3 tiles (grid order) and at 261 (runs of 16 tiles per XCD + a tail)."""
    import torch
    rng = np.random.default_rng(5)
    host = rng.integers(0, 256, tiles * 16384, dtype=np.uint8)
    data = torch.from_numpy(host).cuda()
    w = host.view("<u4").reshape(tiles, 4, 256, 4)  # tile, k, lane, dword
    lane_x = np.bitwise_xor.reduce(np.bitwise_xor.reduce(w, axis=3), axis=1)  # tile, lane
    o8 = engine.probe_stream(data, True)
    torch.cuda.synchronize()
    got = o8.cpu().numpy().view("<u4").reshape(-1, 2)
    assert (got[:, 0] == lane_x.reshape(-1)).all() and (got[:, 1] == np.arange(tiles * 256)).all()
    o0 = engine.probe_stream(data, False)
    torch.cuda.synchronize()
    assert (o0.cpu().numpy().view("<u4")[:tiles] == np.bitwise_xor.reduce(lane_x, axis=1)).all()
    ow = torch.full((tiles * 16384 + 16,), 0xAB, dtype=torch.uint8, device="cuda")
    engine.probe_write(ow)
    torch.cuda.synchronize()
    got = ow.cpu().numpy()
    want = np.zeros((tiles, 1024, 4), np.uint32)
    want[:, :, 0] = np.arange(tiles)[:, None]
    want[:, :, 1] = np.arange(1024)[None, :]
    assert (got[: tiles * 16384].view("<u4") == want.reshape(-1)).all() and (got[tiles * 16384:] == 0xAB).all()


@pytest.mark.parametrize("workload", [abi.WL_UDP64, abi.WL_IMIX])
def test_logical_shards_equal_whole(engine, workload):
    """SURVEY.md §4 item 5 on one device: the batch regenerated as 8 index-range
    shards (nex_amd.dist.shard, as each bench.py rank does) and parsed shard by
    shard gives exactly the whole batch's records and frame bytes."""
    import torch
    from nex_amd import dist
    total = (1 << 20) + 12345
    whole = engine.gen_batch(workload, total)
    want = engine.parse(whole, out_kind=abi.OUT_RECORD)
    parts, frames = [], []
    for r in range(8):
        b, e = dist.shard(total, r, 8)
        sb = engine.gen_batch(workload, e - b, first_index=b)
        parts.append(engine.parse(sb, out_kind=abi.OUT_RECORD)[: (e - b) * 64])
        frames.append(sb.data[: sb.total_bytes] if sb.offsets is None else
                      sb.data[int(sb.offsets[0]): int(sb.offsets[e - b])])
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(parts), want[: total * 64])
    wb = whole.data[: whole.total_bytes] if whole.offsets is None else whole.data[: int(whole.offsets[total])]
    assert torch.equal(torch.cat(frames), wb)


@pytest.mark.parametrize("flags,ip_offset", [(0, 0), (abi.PARSE_STRICT, 0), (abi.PARSE_FROM_IP, 14),
                                             (abi.PARSE_FROM_IP | abi.PARSE_STRICT, 14),
                                             (abi.PARSE_VLAN, 0)])
def test_large_mutation_sweep(engine, oracle, flags, ip_offset):
    """400k fuzz-style mutations of every fixture family (golden, crafted,
    VLAN, FrameSlice edge cases, IMIX) per parse mode, in the packed
    (SpanTile) and explicit-length (TwoPass) layouts: every record field
    bit-exact against the oracle."""
    import torch
    rng = np.random.default_rng(1000 + flags)
    base = ([bytes.fromhex(v["frame"]) for v in helpers.golden()["frames"]] + helpers.crafted_frames() +
            helpers.vlan_frames() + helpers.slice_frames() +
            [oracle.gen_frame(abi.WL_IMIX, i) for i in range(400)])
    frames = helpers.mutate_frames(rng, base, 400_000)
    want = oracle.parse_packed(*_packed_host(frames), flags=flags, ip_offset=ip_offset, nthreads=16)
    mode = ParseMode.Strict if flags & abi.PARSE_STRICT else ParseMode.Lenient
    opt = ParseOption(bool(flags & abi.PARSE_FROM_IP), ip_offset, bool(flags & abi.PARSE_VLAN))
    for batch in (FrameBatch.from_packed(frames), FrameBatch.from_frames(frames, pad_to=2)):
        got = engine.parse_to_numpy(batch, opt, mode, abi.OUT_RECORD)
        helpers.records_equal(got, want, frames, f"mutation sweep flags={flags}")
    torch.cuda.synchronize()


def _packed_host(frames):
    offs = np.zeros(len(frames) + 1, np.uint64)
    offs[1:] = np.cumsum([len(f) for f in frames])
    data = np.frombuffer(b"".join(frames) + bytes(16), np.uint8)
    return data, offs, None


@pytest.mark.parametrize("flags,ip_offset", [(0, 0), (abi.PARSE_FROM_IP, 14)])
def test_large_mutation_sweep_slices_and_options(engine, oracle, flags, ip_offset):
    """The same 400k-mutation corpus through FrameSlice (NEXG_OUT_SLICE) and
    the device option lists (nexg_decode_options), against the oracle."""
    import torch
    rng = np.random.default_rng(2000 + flags)
    base = ([bytes.fromhex(v["frame"]) for v in helpers.golden()["frames"]] + helpers.crafted_frames() +
            helpers.slice_frames() + [oracle.gen_frame(abi.WL_IMIX, i) for i in range(400)])
    frames = helpers.mutate_frames(rng, base, 400_000)
    data, offs, _ = _packed_host(frames)
    want_s = oracle.slice_packed(data, offs, flags=flags, ip_offset=ip_offset)
    opt = ParseOption(bool(flags & abi.PARSE_FROM_IP), ip_offset)
    batch = FrameBatch.from_packed(frames)
    got_s = engine.parse_to_numpy(batch, opt, ParseMode.Lenient, abi.OUT_SLICE)
    helpers.records_equal(got_s, want_s, frames, f"slice sweep flags={flags}")
    recs = engine.parse(batch, opt, ParseMode.Lenient, abi.OUT_RECORD)
    got_o = engine.decode_options(batch, recs)
    torch.cuda.synchronize()
    got_o = got_o.cpu().numpy()[: len(frames) * 96].view(abi.OPTIONS_DTYPE)
    sel = rng.choice(len(frames), 40_000, replace=False)  # the oracle's option walk is per frame
    want_o = np.array([oracle.decode_options(frames[i], flags, ip_offset) for i in sel], abi.OPTIONS_DTYPE)
    helpers.records_equal(got_o[sel], want_o, [frames[i] for i in sel], f"options sweep flags={flags}")


def test_build_udp4_tuples_aos(engine, oracle):
    """nexg_build_udp4_tuples (one 16-B tuple record per frame): the bytes of
    every frame equal the oracle's udp_ping build (builder/udp.rs:67-95,
    builder/ipv4.rs:94-166) of the same tuple, and equal the SoA build of the
    same arrays, at a full 16M batch (the bench's ser.tuples workload) and at
    ragged counts; per-frame arrays next to the tuples are refused."""
    import ctypes

    import torch
    smac, dmac = bytes([2, 0, 0, 0, 0, 1]), bytes([2, 0, 0, 0, 0, 2])
    for n in (1, 255, 257, 5000, 16 << 20):
        p = engine.gen_udp4_params(n, first_index=3)
        tup = engine.pack_udp4_tuples(*p)
        aos = engine.build_udp4_tuples(tup, src_mac=smac, dst_mac=dmac, ip_flags=2)
        soa = engine.build_udp4(*p, src_mac=smac, dst_mac=dmac, ip_flags=2)
        torch.cuda.synchronize()
        assert torch.equal(aos[: n * 42], soa[: n * 42]), n
        m = min(n, 1 << 16)
        host = [t[:m].cpu().numpy().view(np.uint32 if t.element_size() == 4 else np.uint16) for t in p]
        want = oracle.build_udp4_batch(smac, dmac, *host, 64, 2)
        assert (aos[: m * 42].cpu().numpy().reshape(m, 42) == want).all(), n
    rec = tup[:1].cpu().numpy().view(abi.UDP4_TUPLE_DTYPE)[0]
    assert rec["src_ip"] == int(p[0][0].item()) & 0xFFFFFFFF and rec["dst_port"] == int(p[3][0].item()) & 0xFFFF
    # the other AOS instantiations: a payload (stride 82: the 128-B tile; stride
    # 142: direct global writes) and an output 1 B off 16-B alignment (direct)
    n = 3000
    p = engine.gen_udp4_params(n, first_index=11)
    tup = engine.pack_udp4_tuples(*p)
    for plen, shift in ((40, 0), (100, 0), (0, 1), (40, 1)):
        pay = torch.arange(plen, dtype=torch.uint8, device="cuda") if plen else None
        stride = 42 + plen
        buf_a = torch.zeros(n * stride + 16, dtype=torch.uint8, device="cuda")
        buf_s = torch.zeros(n * stride + 16, dtype=torch.uint8, device="cuda")
        engine.build_udp4_tuples(tup, src_mac=smac, dst_mac=dmac, ip_flags=2, payload=pay,
                                 out=buf_a[shift:], out_stride=stride)
        engine.build_udp4(*p, src_mac=smac, dst_mac=dmac, ip_flags=2, payload=pay, out=buf_s[shift:],
                          out_stride=stride)
        torch.cuda.synchronize()
        assert torch.equal(buf_a, buf_s), (plen, shift)
        host = [t.cpu().numpy().view(np.uint32 if t.element_size() == 4 else np.uint16) for t in p]
        frames = buf_a[shift: shift + n * stride].cpu().numpy().reshape(n, stride)
        for i in list(range(0, n, 97)) + [n - 1]:
            want = oracle.build_udp4(smac, dmac, int(host[0][i]), int(host[1][i]), int(host[2][i]),
                                     int(host[3][i]), int(host[4][i]), 64, 2, 0, bytes(range(plen)))
            assert bytes(frames[i]) == want, (plen, shift, i)
    bad = abi.Udp4Build()
    bad.count, bad.dst_ip = 4, p[1].data_ptr()
    out = torch.empty(4 * 42, dtype=torch.uint8, device="cuda")
    rc = engine.lib.nexg_build_udp4_tuples(engine.ctx, ctypes.byref(bad), ctypes.c_void_p(tup.data_ptr()),
                                           ctypes.c_void_p(out.data_ptr()), 42, None)
    assert rc == abi.EINVAL
