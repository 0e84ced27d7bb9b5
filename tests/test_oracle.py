"""CPU: the oracle (CPU restatement) pinned against the reference's own KATs,
fixtures and quirks (tests/golden/reference_vectors.json)."""
import numpy as np
import pytest

from nex_amd import abi
from nex_amd.frame import frame_from_record, Truncated, BufferTooShort, Malformed
from tests import helpers


G = helpers.golden()


@pytest.mark.parametrize("v", G["util"]["sum_be_words"], ids=lambda v: f"{v['data'][:8]}-{v['skipword']}")
def test_util_sum_be_words_kat(oracle, v):
    # util.rs:190-217
    assert oracle.sum_be_words(bytes.fromhex(v["data"]), v["skipword"]) == v["sum"]


def test_util_joined_kat(oracle):
    # util.rs:244-254
    for v in G["util"]["joined_equals_contiguous"]:
        j = oracle.sum_be_words_joined(bytes.fromhex(v["data"]), 2**63, bytes.fromhex(v["extra"]))
        assert j == oracle.sum_be_words(bytes.fromhex(v["contiguous"]), 2**63)


def test_util_checksum_kat(oracle):
    # util.rs:256-261
    for v in G["util"]["checksum"]:
        assert oracle.checksum(bytes.fromhex(v["data"]), v["skipword"]) == v["checksum"]


def test_checksum_empty_is_zero(oracle):
    # Q19: util.rs:66-68
    assert oracle.checksum(b"", 0) == 0
    assert oracle.checksum(bytes(4), 99) == 0xFFFF


def test_icmpv6_checksum_kat(oracle):
    # icmpv6.rs:606-631
    k = G["icmpv6"]
    pkt = bytes.fromhex(k["packet"])
    src, dst = bytes.fromhex(k["src"]), bytes.fromhex(k["dst"])
    assert oracle.ipv6_checksum(pkt, 1, src, dst, 58) == k["checksum"]
    assert oracle.ipv6_checksum(b"\x81" + pkt[1:], 1, src, dst, 58) == k["checksum_type_0x81"]


@pytest.mark.parametrize("v", G["frames"], ids=lambda v: v["name"])
def test_golden_frames(oracle, v):
    fr = bytes.fromhex(v["frame"])
    rec = oracle.parse_frame(fr, v["parse_flags"], v["ip_offset"])
    helpers.check_expect(rec, fr, v["expect"], v["name"], parse_flags=v["parse_flags"], ip_offset=v["ip_offset"])


def test_survey_crosscheck_values(oracle):
    """Values an independent scratch restatement produced during the survey
    (SURVEY.md §8(c)); not reference-asserted, but a second implementation."""
    g = {v["name"]: bytes.fromhex(v["frame"]) for v in G["frames"]}
    r = oracle.parse_frame(g["ipv4_udp_frame"])
    assert (int(r["ip_csum_calc"]), int(r["l4_csum_calc"])) == (0x8E95, 0x0A92)
    r = oracle.parse_frame(g["bench_ipv4_tcp_frame"])
    assert (int(r["ip_csum_calc"]), int(r["l4_csum_calc"])) == (0x3C5D, 0x3956)
    r = oracle.parse_frame(g["ipv4_round_trip"], abi.PARSE_FROM_IP)
    assert int(r["ip_csum_calc"]) == 0x9C7D and not (int(r["flags"]) & abi.C_IP_OK)


def test_udp_ping_build_golden(oracle):
    b = G["build"][0]
    f = oracle.build_udp4(bytes(6), bytes(6), 0xC0A80164, 0x01010101, b["sport"], b["dport"],
                          ip_flags=b["ip_flags"])
    assert len(f) == b["frame_len"]
    r = oracle.parse_frame(f)
    assert int(r["flags"]) & abi.C_IP_OK and int(r["flags"]) & abi.C_L4_OK
    assert int(r["ip_length"]) == b["ip_total_length"] and int(r["l4_length"]) == b["udp_length"]
    assert (int(r["l4_csum"]), int(r["ip_csum"])) == (0xE870, 0x76C3)  # survey cross-check
    with pytest.raises(ValueError):
        oracle.build_udp4(bytes(6), bytes(6), 1, 2, 3, 4, payload=bytes(65535 - 28 + 1))


def test_udp4_batch_build_equals_single(oracle):
    """The serialize bench's CPU baseline (nexo_build_udp4_batch, threaded)
    builds exactly what the per-tuple restatement builds."""
    rng = np.random.default_rng(3)
    n = 1000
    src, dst = rng.integers(0, 1 << 32, n, dtype=np.uint32), rng.integers(0, 1 << 32, n, dtype=np.uint32)
    sp, dp, ids = (rng.integers(0, 1 << 16, n, dtype=np.uint16) for _ in range(3))
    sm, dm = bytes([2, 0, 0, 0, 0, 1]), bytes([2, 0, 0, 0, 0, 2])
    for th in (1, 3):
        got = oracle.build_udp4_batch(sm, dm, src, dst, sp, dp, ids, 64, 2, nthreads=th)
        for i in range(0, n, 7):
            want = oracle.build_udp4(sm, dm, int(src[i]), int(dst[i]), int(sp[i]), int(dp[i]), int(ids[i]), 64, 2)
            assert bytes(got[i]) == want


# ---- quirks -------------------------------------------

def _rec(oracle, fr, flags=0, off=0):
    return oracle.parse_frame(fr, flags, off)


def test_q2_short_ethernet_is_error(oracle):
    with pytest.raises(BufferTooShort):
        frame_from_record(_rec(oracle, bytes(13)), bytes(13))
    with pytest.raises(Malformed):
        frame_from_record(_rec(oracle, bytes(10), abi.PARSE_FROM_IP, 3), bytes(10))


def test_q4_lenient_ipv4_failure(oracle):
    fr = helpers._eth(bytes([0x44]) + bytes(30))
    f = frame_from_record(_rec(oracle, fr), fr)
    assert f.ip is not None and f.ip.ipv4 is None and f.transport is None and f.payload == b""


def test_q5_effective_total_length(oracle):
    P = bytes(range(20))
    fr = helpers._eth(helpers._ipv4(helpers._udp(P), 17, total=0))
    assert int(_rec(oracle, fr)["ip_length"]) == len(fr) - 14
    fr = helpers._eth(helpers._ipv4(helpers._udp(P), 17)) + bytes(10)  # padding excluded
    f = frame_from_record(_rec(oracle, fr), fr)
    assert f.payload == P
    fr = helpers._eth(helpers._ipv4(helpers._udp(P), 17, total=400))
    assert int(_rec(oracle, fr)["ip_length"]) == len(fr) - 14
    with pytest.raises(Truncated):
        frame_from_record(_rec(oracle, fr, abi.PARSE_STRICT), fr)


def test_q8_reserved_protocol_changes_ip_checksum(oracle):
    fr = bytearray(helpers._eth(helpers._ipv4(bytes(8), 200)))
    r = _rec(oracle, bytes(fr))
    assert int(r["ip_proto"]) == 255
    # the serialised header carries 255, so checksumming the raw bytes differs
    raw = oracle.checksum(bytes(fr[14:34]), 5)
    assert int(r["ip_csum_calc"]) != raw


def test_q10_ipv6_extension_keeps_raw_next_header(oracle):
    P = bytes(range(16))
    fr = helpers._eth(helpers._ipv6(bytes([17, 0]) + bytes(6) + helpers._udp(P), 0), 0x86DD)
    r = _rec(oracle, fr)
    assert int(r["ip_proto"]) == 0 and not (int(r["flags"]) & abi.L_TRANSPORT)
    assert int(r["payload_off"]) == 14 + 48


def test_q13_tcp_failure_keeps_ip_payload(oracle):
    P = bytes(range(30))
    seg = helpers._tcp(P, doff=4)
    fr = helpers._eth(helpers._ipv4(seg, 6))
    f = frame_from_record(_rec(oracle, fr), fr)
    assert f.transport.tcp is None and f.transport.udp is None and f.payload == seg


def test_q15_icmp_needs_8_bytes(oracle):
    fr = helpers._eth(helpers._ipv4(bytes(7), 1))
    f = frame_from_record(_rec(oracle, fr), fr)
    assert f.ip.icmp is None and f.payload == bytes(7) and f.transport is None


def test_q16_tcp_early_eol_reserialises(oracle):
    P = bytes(range(9))
    seg = helpers._tcp(P, opts=b"\x00\x99\x99\x99\x11\x22\x33\x44")
    fr = helpers._eth(helpers._ipv4(seg, 6))
    r = _rec(oracle, fr)
    raw = oracle.ipv4_checksum(seg, 8, bytes([10, 1, 2, 3]), bytes([10, 4, 5, 6]), 6)
    assert int(r["l4_csum_calc"]) != raw  # re-serialised: doff 6, zeroed tail


def test_q17_ipv4_checksum_panic_flagged(oracle):
    fr = helpers._eth(helpers._ipv4(b"", 17, ihl=15, opts=b"\x00" + bytes(39)))
    r = _rec(oracle, fr)
    assert int(r["flags"]) & abi.C_IP_PANIC and not int(r["flags"]) & abi.C_IP_CHECKED


def test_q18_udp_zero_checksum_literal(oracle):
    # a stored 0 is compared literally; no "0 means no checksum" rule
    P = bytes(range(12))
    fr = bytearray(helpers._eth(helpers._ipv4(helpers._udp(P), 17)))
    fr[40:42] = b"\x00\x00"
    r = _rec(oracle, bytes(fr))
    assert int(r["l4_csum"]) == 0 and not (int(r["flags"]) & abi.C_L4_OK)


def test_generator_udp64_properties(oracle):
    recs = np.array([oracle.parse_frame(oracle.gen_frame(abi.WL_UDP64, i)) for i in range(4096)],
                    dtype=abi.RECORD_DTYPE)
    f = recs["flags"]
    assert ((f & abi.L_UDP) != 0).all() and (recs["payload_len"] == 22).all()
    bad = ((f & abi.C_IP_OK) == 0) | ((f & abi.C_L4_OK) == 0)
    assert 0.04 < bad.mean() < 0.09  # 1/16 corrupted
    assert not (((f & abi.C_IP_OK) == 0) & ((f & abi.C_L4_OK) == 0)).any()


def test_generator_imix_properties(oracle):
    n = 6000
    lens = np.array([oracle.gen_length(abi.WL_IMIX, i) for i in range(n)])
    share = [(lens == L).mean() for L in (64, 576, 1500)]
    assert abs(share[0] - 7 / 12) < 0.03 and abs(share[1] - 4 / 12) < 0.03
    recs = np.array([oracle.parse_frame(oracle.gen_frame(abi.WL_IMIX, i)) for i in range(800)],
                    dtype=abi.RECORD_DTYPE)
    f = recs["flags"]
    assert (f & abi.C_L4_CHECKED).all()
    assert ((f & abi.L_IPV6) != 0).mean() > 0.3 and ((f & abi.L_TCP) != 0).mean() > 0.2


def test_oracle_batch_bad_extent(oracle):
    """nexg.h NEXG_ERR_BAD_EXTENT: a frame longer than 65535 B or reaching past
    data_bytes is reported, not parsed (the GPU kernels do the same)."""
    data = np.zeros(70100, np.uint8)
    offs = np.array([0, 64, 64 + 70000, 70100], np.uint64)
    recs = oracle.parse_packed(data, offs, None)
    st = list(abi.status_of(recs["flags"]))
    assert st[1] == abi.ERR_BAD_EXTENT and st[0] != abi.ERR_BAD_EXTENT and st[2] != abi.ERR_BAD_EXTENT
    recs = oracle.parse_packed(data[:100], np.array([0, 64], np.uint64), np.array([64, 40], np.uint32))
    assert abi.status_of(recs["flags"])[1] == abi.ERR_BAD_EXTENT


def _ones_complement(words):
    s = sum(words)
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def test_udp_ping_ipv6_build_kat(oracle):
    """udp_ping's IPv6 branch (udp_ping.rs:83-89): layout per Ipv6Packet::to_bytes
    (ipv6.rs:50-75) and a checksum recomputed here with a plain RFC 1071 sum
    over the IPv6 pseudo-header (util.rs:111-133); the oracle parser then
    verifies it (l4_ok)."""
    import ipaddress
    src = ipaddress.IPv6Address("2001:db8::1").packed
    dst = ipaddress.IPv6Address("2606:4700:4700::1111").packed
    for payload in (b"", b"\x01", b"ping!", bytes(range(200))):
        f = oracle.build_udp6(b"\x02" * 6, b"\x04" * 6, src, dst, 53443, 33435,
                              hop_limit=64, traffic_class=0xA5, flow_label=0x12345, payload=payload)
        ulen = 8 + len(payload)
        assert len(f) == 62 + len(payload)
        assert f[12:14] == b"\x86\xdd"
        assert f[14:18] == bytes([0x6A, 0x51, 0x23, 0x45])      # version 6, tc 0xA5, flow 0x12345
        assert f[18:20] == ulen.to_bytes(2, "big") and f[20] == 17 and f[21] == 64
        assert f[22:38] == src and f[38:54] == dst
        assert f[54:58] == (53443).to_bytes(2, "big") + (33435).to_bytes(2, "big")
        seg = f[54:] + (b"\0" if len(f[54:]) % 2 else b"")
        words = [int.from_bytes(src[i:i + 2], "big") for i in range(0, 16, 2)]
        words += [int.from_bytes(dst[i:i + 2], "big") for i in range(0, 16, 2)]
        words += [17, ulen]
        words += [int.from_bytes(seg[i:i + 2], "big") for i in range(0, len(seg), 2) if i != 6]
        assert int.from_bytes(f[60:62], "big") == _ones_complement(words)
        r = oracle.parse_frame(f)
        assert r["flags"] & abi.C_L4_OK and r["payload_len"] == len(payload)
    with pytest.raises(ValueError):
        oracle.build_udp6(b"\0" * 6, b"\0" * 6, src, dst, 1, 2, payload=bytes(65528))


# ---- FrameSlice (frame.rs:84-287) ------------------------------------------

def _check_slice(s, exp, frame, name):
    assert abi.status_of(np.array([s["flags"]]))[0] == 0, name
    f = int(s["flags"])
    if "datalink" in exp:
        assert f & abi.S_DATALINK and exp["datalink"] == [0, 14], name
    if "network" in exp:
        assert f & abi.S_NETWORK, name
        assert [s["l3_off"], s["l3_off"] + s["l3_len"]] == exp["network"], name
    if "network_len" in exp:
        assert f & abi.S_NETWORK and s["l3_len"] == exp["network_len"], name
    if "transport" in exp:
        a = s["l3_off"] + s["l3_len"]
        assert f & abi.S_TRANSPORT and [a, a + s["l4_len"]] == exp["transport"], name
    if "transport_len" in exp:
        assert f & abi.S_TRANSPORT and s["l4_len"] == exp["transport_len"], name
    if "payload" in exp:
        assert [s["payload_off"], s["payload_off"] + s["payload_len"]] == exp["payload"], name
    if "payload_bytes" in exp:
        p = frame[s["payload_off"]:s["payload_off"] + s["payload_len"]]
        assert p.hex() == exp["payload_bytes"], name
    if "ip_protocol" in exp:
        assert f & abi.S_IP_PROTOCOL and (f >> abi.S_PROTO_SHIFT) & 0xFF == exp["ip_protocol"], name


def test_frame_slice_goldens(oracle):
    n = 0
    for v in helpers.golden()["frames"]:
        if "slice_expect" not in v:
            continue
        fr = bytes.fromhex(v["frame"])
        _check_slice(oracle.slice_frame(fr, v["parse_flags"], v["ip_offset"]), v["slice_expect"], fr,
                     v["name"])
        n += 1
    assert n == 2


def test_frame_slice_semantics(oracle):
    """Where FrameSlice differs from Frame (frame.rs:179-286): hard errors,
    AH walked, ICMP from 4 B, UDP length unchecked, lossy protocol value."""
    P = bytes(range(40))
    st = lambda s: int(abi.status_of(np.array([s["flags"]]))[0])
    # IPv4 with IHL < 5: Frame is lenient (ip all None), FrameSlice errors
    assert st(oracle.slice_frame(helpers._eth(bytes([0x44]) + bytes(19)))) == abi.ERR_INVALID_LENGTH
    assert st(oracle.slice_frame(helpers._eth(P[:19]))) == abi.ERR_BUFFER_TOO_SHORT
    assert st(oracle.slice_frame(helpers._eth(bytes([0x55]) + bytes(19)))) == abi.ERR_MALFORMED
    assert st(oracle.slice_frame(bytes(13))) == abi.ERR_BUFFER_TOO_SHORT
    # UDP length field is not checked: bogus length still yields an 8-B transport
    s = oracle.slice_frame(helpers._eth(helpers._ipv4(helpers._udp(P, length=3), 17)))
    assert st(s) == 0 and s["l4_len"] == 8 and s["payload_len"] == len(P)
    # ICMP header is 4 B and needs only 4 B
    s = oracle.slice_frame(helpers._eth(helpers._ipv4(bytes(5), 1)))
    assert s["l4_len"] == 4 and s["payload_len"] == 1
    # TCP with a bad data offset is an error (Frame keeps going)
    assert st(oracle.slice_frame(helpers._eth(helpers._ipv4(helpers._tcp(P, doff=4), 6)))) == \
        abi.ERR_INVALID_LENGTH
    # TCP shorter than 20 B: no transport, payload = the bytes
    s = oracle.slice_frame(helpers._eth(helpers._ipv4(P[:10], 6)))
    assert st(s) == 0 and not s["flags"] & abi.S_TRANSPORT and s["payload_len"] == 10
    # IPv6 AH (51) is walked: (len + 2) * 4 bytes, then UDP
    ah = bytes([17, 1]) + bytes(10)
    s = oracle.slice_frame(helpers._eth(helpers._ipv6(ah + helpers._udp(b"xyz"), 51), 0x86DD))
    assert st(s) == 0 and s["l3_len"] == 40 + 12 and s["l4_len"] == 8 and s["payload_len"] == 3
    # truncated extension header
    s = oracle.slice_frame(helpers._eth(helpers._ipv6(bytes([17, 3]) + bytes(6), 0), 0x86DD))
    assert st(s) == abi.ERR_TRUNCATED
    # protocol 200 reported as Reserved (255)
    s = oracle.slice_frame(helpers._eth(helpers._ipv4(P, 200)))
    assert (s["flags"] >> abi.S_PROTO_SHIFT) & 0xFF == 255 and s["payload_len"] == len(P)
    # ARP: 28-B network when long enough, nothing otherwise
    s = oracle.slice_frame(helpers._eth(bytes(30), 0x0806))
    assert s["flags"] & abi.S_NETWORK and s["l3_len"] == 28 and s["payload_len"] == 2
    s = oracle.slice_frame(helpers._eth(bytes(20), 0x0806))
    assert not s["flags"] & abi.S_NETWORK and s["payload_len"] == 20
    # from_ip_packet: offset past the end / bad version
    assert st(oracle.slice_frame(bytes(4), abi.PARSE_FROM_IP, 5)) == abi.ERR_INVALID_LENGTH
    assert st(oracle.slice_frame(bytes(4), abi.PARSE_FROM_IP, 4)) == abi.ERR_MALFORMED
    s = oracle.slice_frame(bytes(2) + helpers._ipv4(helpers._udp(b"ab"), 17), abi.PARSE_FROM_IP, 2)
    assert st(s) == 0 and not s["flags"] & abi.S_DATALINK and s["l3_off"] == 2
    assert s["ethertype"] == 0x0800 and s["payload_len"] == 2


def test_frame_slice_materialisation(oracle):
    """nex_amd.frame.frame_slice_from_record rebuilds the reference's borrowed
    views; errors raise the reference's ParseError kind."""
    from nex_amd.frame import frame_slice_from_record, InvalidLength
    v = [x for x in helpers.golden()["frames"] if x["name"] == "frame_slice_ipv4_tcp"][0]
    fr = bytes.fromhex(v["frame"])
    fs = frame_slice_from_record(oracle.slice_frame(fr), fr)
    assert bytes(fs.datalink) == fr[:14] and bytes(fs.network) == fr[14:34]
    assert bytes(fs.transport) == fr[34:54] and bytes(fs.payload) == b"data"
    assert fs.ethertype == 0x0800 and fs.ip_protocol == 6
    with pytest.raises(InvalidLength):
        frame_slice_from_record(oracle.slice_frame(helpers._eth(bytes([0x44]) + bytes(19))), b"")


# ---- tcp_ping / icmp_ping builders (8(f)3) ---------------------------------

def _pseudo_words(src, dst, proto, length):
    w = [int.from_bytes(src[i:i + 2], "big") for i in range(0, len(src), 2)]
    w += [int.from_bytes(dst[i:i + 2], "big") for i in range(0, len(dst), 2)]
    return w + [proto, length]


def _words(b, skip):
    b = b + (b"\0" if len(b) % 2 else b"")
    return [int.from_bytes(b[i:i + 2], "big") for i in range(0, len(b), 2) if i // 2 != skip]


def test_tcp_builder_reference_assertions(oracle):
    import ipaddress
    g = helpers.golden()["build_l4"]
    b = g["tcp_basic"]
    src, dst = ipaddress.IPv4Address(b["src_ip"]).packed, ipaddress.IPv4Address(b["dst_ip"]).packed
    spec = oracle.ip_spec(4, src, dst, ip_flags=2)
    f = oracle.build_tcp(spec, b["sport"], b["dport"], b["seq"], b["ack"], b["flags"], b["window"],
                         b["urg"], payload=bytes.fromhex(b["payload"]))
    t = f[34:]
    assert int.from_bytes(t[0:2], "big") == 1234 and int.from_bytes(t[2:4], "big") == 80
    assert int.from_bytes(t[4:8], "big") == 1 and int.from_bytes(t[8:12], "big") == 2
    assert t[13] == 0x02 and t[12] >> 4 == 5 and t[20:] == b"abc"
    # independent RFC 1071 sum over the IPv4 pseudo-header (util.rs:81-97)
    assert int.from_bytes(t[16:18], "big") == _ones_complement(_pseudo_words(src, dst, 6, len(t)) + _words(t, 8))
    r = oracle.parse_frame(f)
    assert r["flags"] & abi.C_L4_OK and r["flags"] & abi.C_IP_OK
    with pytest.raises(ValueError):  # tcp.rs:211-228
        oracle.build_tcp(spec, 1, 2, options=bytes.fromhex(g["tcp_oversized_options"]["options"]))


@pytest.mark.parametrize("family", [4, 6])
def test_tcp_ping_shape(oracle, family):
    import ipaddress
    g = helpers.golden()["build_l4"]["tcp_ping_options"]
    if family == 4:
        src, dst = ipaddress.IPv4Address("10.0.0.1").packed, ipaddress.IPv4Address("10.0.0.2").packed
    else:
        src, dst = ipaddress.IPv6Address("2001:db8::1").packed, ipaddress.IPv6Address("2001:db8::2").packed
    spec = oracle.ip_spec(family, src, dst, ip_flags=2)
    opts = bytes.fromhex(g["options"])
    f = oracle.build_tcp(spec, g["sport"], 443, 0, 0, g["flags"], g["window"], options=opts)
    l4 = 34 if family == 4 else 54
    t = f[l4:]
    assert t[12] >> 4 == g["data_offset"] and len(t) == 32
    assert t[20:31] == opts and t[31] == 0  # zero padding to the 4-B boundary
    ps = _pseudo_words(src, dst, 6, len(t))
    assert int.from_bytes(t[16:18], "big") == _ones_complement(ps + _words(t, 8))
    r = oracle.parse_frame(f)
    assert r["flags"] & abi.C_L4_OK and r["l4_nopt"] == 6  # the zero pad parses back as EOL


@pytest.mark.parametrize("family", [4, 6])
def test_icmp_ping_shape(oracle, family):
    import ipaddress
    g = helpers.golden()["build_l4"]
    e = g["icmp_ping"]
    if family == 4:
        src, dst = ipaddress.IPv4Address("10.0.0.1").packed, ipaddress.IPv4Address("10.0.0.2").packed
        typ = 8
    else:
        src, dst = ipaddress.IPv6Address("2001:db8::1").packed, ipaddress.IPv6Address("2001:db8::2").packed
        typ = 128
    spec = oracle.ip_spec(family, src, dst, ip_flags=2)
    f = oracle.build_icmp_echo(spec, typ, 0, e["ident"], e["seq"], bytes.fromhex(e["payload"]))
    m = f[34:] if family == 4 else f[54:]
    assert m[0] == typ and m[4:6] == b"\x12\x34" and m[6:8] == b"\x00\x01" and m[8:] == b"hello"
    words = _words(m, 1)
    if family == 6:
        words = _pseudo_words(src, dst, 58, len(m)) + words
    assert int.from_bytes(m[2:4], "big") == _ones_complement(words)
    r = oracle.parse_frame(f)
    assert r["flags"] & abi.C_L4_OK
    with pytest.raises(ValueError):  # builder/icmp.rs:104-117
        oracle.build_icmp_echo(oracle.ip_spec(4, src[:4], dst[:4]), 8, 0, 0, 0,
                               bytes(g["icmp_too_large"]["payload_len"]))


def test_vlan_extension_oracle(oracle):
    """NEXG_PARSE_VLAN: a tagged frame parses like the same frame with the tags
    removed, offsets shifted by 4 per unwrapped tag; without the flag the
    reference behaviour (Q3: no unwrapping) is untouched."""
    shift_fields = ("payload_off", "l3_off", "l4_off")
    for f in helpers.vlan_frames():
        got = oracle.parse_frame(f, abi.PARSE_VLAN)
        plain = oracle.parse_frame(f)
        et = int.from_bytes(f[12:14], "big") if len(f) >= 14 else 0
        ntag = 0
        while ntag < 2 and et in (0x8100, 0x88A8, 0x9100) and len(f) >= 14 + 4 * ntag + 4:
            et = int.from_bytes(f[14 + 4 * ntag + 2:14 + 4 * ntag + 4], "big")
            ntag += 1
        if ntag == 0:
            assert got.tobytes() == plain.tobytes()
            continue
        detag = f[:12] + f[12 + 4 * ntag:]
        want = oracle.parse_frame(detag).copy()
        assert got["flags"] & abi.L_VLAN
        assert (int(got["flags"]) & ~abi.L_VLAN) == int(want["flags"]), f.hex()
        for n in abi.RECORD_DTYPE.names:
            if n == "flags":
                continue
            w = int(want[n])
            if n in shift_fields and (n != "payload_off" or want["payload_len"]) and \
                    (n != "l4_off" or w):
                w += 4 * ntag
            if n == "packet_len":
                w = len(f)
            assert int(got[n]) == w, (n, f.hex())
        if not abi.status_of(int(got["flags"])):  # the Ethernet MACs stay the frame's own
            from nex_amd.frame import frame_from_record
            eth = frame_from_record(got, f).datalink.ethernet
            assert eth.destination == f[0:6] and eth.source == f[6:12] and eth.ethertype == et
    # untagged frames are unchanged by the flag
    for f in helpers.crafted_frames():
        if len(f) >= 14 and f[12:14] in (b"\x81\x00", b"\x88\xa8", b"\x91\x00"):
            continue
        assert oracle.parse_frame(f, abi.PARSE_VLAN).tobytes() == oracle.parse_frame(f).tobytes()


def test_probe_builders(oracle):
    """The arp / ndp probe builders' restatement (examples/arp.rs:59-67,
    examples/ndp.rs:82-108): ARP request layout (arp.rs:385-399) behind a
    broadcast Ethernet header; InvalidFieldLength for hw / proto lengths
    (builder/arp.rs:101-118, arp_builder_rejects_non_ethernet_address_length);
    the NS message is 32 B with a 28-B Icmpv6Packet payload (builder/ndp.rs
    ndp_builder_produces_aligned_source_link_layer_option), its checksum an
    independent RFC 1071 sum, and it parses (oracle) as ICMPv6 135 with the
    checksum verifying."""
    import pytest
    mac = bytes([0x02, 0x42, 0xac, 0x11, 0x00, 0x02])
    f = oracle.build_arp(b"\xff" * 6, mac, bytes([192, 168, 1, 10]), bytes(6), bytes([192, 168, 1, 1]))
    assert f == (b"\xff" * 6 + mac + b"\x08\x06" + bytes([0, 1, 8, 0, 6, 4, 0, 1]) + mac +
                 bytes([192, 168, 1, 10]) + bytes(6) + bytes([192, 168, 1, 1]))
    r = oracle.parse_frame(f)
    assert int(r["flags"]) & 0x3FF == abi.L_ETHERNET | abi.L_ARP
    with pytest.raises(ValueError):
        oracle.build_arp(b"\xff" * 6, mac, bytes(4), bytes(6), bytes(4), hw_len=5)
    with pytest.raises(ValueError):
        oracle.build_arp(b"\xff" * 6, mac, bytes(4), bytes(6), bytes(4), proto_len=6)
    lo = bytes(15) + b"\x01"
    sp = oracle.ip_spec(6, lo, lo, src_mac=bytes(6), dst_mac=bytes([0x33, 0x33, 0, 0, 0, 1]), ttl=255)
    g = oracle.build_ndp_ns(sp)
    assert len(g) == 86 and g[12:14] == b"\x86\xdd" and g[20] == 58 and g[21] == 255
    msg = g[54:]
    assert len(msg) - 4 == 28
    assert msg[0] == 135 and msg[8:24] == lo and msg[24:26] == b"\x01\x01" and msg[26:32] == bytes(6)
    pseudo = lo + lo + (32).to_bytes(4, "big") + bytes([0, 0, 0, 58])
    assert int.from_bytes(msg[2:4], "big") == helpers.rfc1071(pseudo + msg[:2] + b"\0\0" + msg[4:])
    r = oracle.parse_frame(g)
    assert int(r["l4_type"]) == 135 and int(r["flags"]) & abi.C_L4_OK
