"""Shared test helpers: golden vectors, expectation checks, malformed mixes."""
import ipaddress
import json
import os

import numpy as np

from nex_amd import abi
from nex_amd.frame import frame_from_record

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_vectors.json")

LAYER_BITS = {
    "eth": abi.L_ETHERNET, "arp": abi.L_ARP, "ip": abi.L_IP, "ipv4": abi.L_IPV4,
    "ipv6": abi.L_IPV6, "icmp": abi.L_ICMP, "icmpv6": abi.L_ICMPV6,
    "transport": abi.L_TRANSPORT, "tcp": abi.L_TCP, "udp": abi.L_UDP,
}
LAYER_MASK = 0x3FF


def golden():
    with open(GOLDEN) as f:
        return json.load(f)


def rfc1071(data: bytes) -> int:
    """Independent Internet checksum (RFC 1071) of `data` (pure Python)."""
    if len(data) % 2:
        data += b"\0"
    s = sum(int.from_bytes(data[i:i + 2], "big") for i in range(0, len(data), 2))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return ~s & 0xFFFF


def check_expect(rec, frame: bytes, exp: dict, name="", reparse=None, parse_flags=0, ip_offset=0):
    """Assert a record satisfies a reference-test expectation dict.
    `reparse(frame) -> record` re-parses a modified frame (default: the
    oracle; GPU tests pass the engine)."""
    flags = int(rec["flags"])
    if "status" in exp:
        assert (flags >> abi.STATUS_SHIFT) & 7 == exp["status"], name
        if "err_context" in exp:  # the ParseError payload (parse.rs:53-81)
            assert abi.ERR_CONTEXTS[int(rec["l4_type"])] == exp["err_context"], (name, int(rec["l4_type"]))
            assert (int(rec["ip_src"]), int(rec["ip_dst"])) == (exp["err_a"], exp["err_b"]), name
        return
    assert (flags >> abi.STATUS_SHIFT) & 7 == 0, name
    if "layers" in exp:
        want = 0
        for l in exp["layers"]:
            want |= LAYER_BITS[l]
        assert flags & LAYER_MASK == want, (name, hex(flags & LAYER_MASK), hex(want))
    fr = frame_from_record(rec, frame)
    for k, v in exp.items():
        if k in ("layers", "status"):
            continue
        if k == "payload":
            assert fr.payload.hex() == v, (name, fr.payload.hex(), v)
        elif k == "ip_version":
            assert (fr.ip.ipv4 or fr.ip.ipv6).version == v, name
        elif k == "ip_ihl":
            assert int(rec["ip_ver_ihl"]) & 15 == v, name
        elif k in ("ip_src", "ip_dst"):
            assert str(ipaddress.IPv4Address(int(rec[k]))) == v, name
        elif k in ("eth_dst", "eth_src"):
            e = fr.datalink.ethernet
            assert (e.destination if k == "eth_dst" else e.source).hex() == v, name
        elif k == "view" and v["kind"] in NDP_KINDS:
            check_ndp_view(rec, frame, v, name)
        elif k == "view":  # the ICMP / ICMPv6 sub-message the reference test downcasts to
            from nex_amd import views
            kind = v["kind"]
            if kind.startswith("Icmpv6"):
                pkt = views.icmpv6_from_record(rec, frame)
                m = views.Icmpv6EchoPacket.try_from(pkt, reply=kind == "Icmpv6EchoReply")
            else:
                m = views.icmp_message(views.icmp_from_record(rec, frame))
                assert type(m).__name__ == kind + "Packet", (name, type(m).__name__)
            for f, want in v.items():
                if f == "kind":
                    continue
                got = getattr(m, f)
                assert (got.hex() if isinstance(got, bytes) else got) == want, (name, f, got, want)
        elif k == "ip_csum_consistent":
            # ipv4.rs:1073-1095: the computed checksum written back into bytes
            # 10..11 makes a packet whose header verifies and whose bytes are
            # raw_copy; the value itself is an independent RFC 1071 sum.
            assert int(rec["flags"]) & abi.C_IP_CHECKED, name
            calc, l3 = int(rec["ip_csum_calc"]), int(rec["l3_off"])
            hl = (int(rec["ip_ver_ihl"]) & 15) * 4
            hdr = frame[l3:l3 + 10] + b"\0\0" + frame[l3 + 12:l3 + hl]
            assert calc == rfc1071(hdr), (name, hex(calc), hex(rfc1071(hdr)))
            raw_copy = frame[:l3 + 10] + calc.to_bytes(2, "big") + frame[l3 + 12:]
            if reparse is None:
                from oracle import oracle
                r2 = oracle.parse_frame(raw_copy, parse_flags, ip_offset)
            else:
                r2 = reparse(raw_copy)
            assert int(r2["flags"]) & abi.C_IP_OK, name
            assert int(r2["ip_csum"]) == calc == int(r2["ip_csum_calc"]), name
        else:
            assert int(rec[k]) == v, (name, k, int(rec[k]), v)


NDP_KINDS = {"RouterSolicit": 133, "RouterAdvert": 134, "NeighborSolicit": 135, "NeighborAdvert": 136,
             "Redirect": 137}


def ndp_fields_equal(m, v: dict, name=""):
    """An NDP view against an expectation dict (golden "view" / "create":
    integers, addresses as text, options as [type, length, payload hex])."""
    for f, want in v.items():
        if f in ("kind", "cite", "bytes", "try_from", "l4_csum"):
            continue
        got = getattr(m, f)
        if f == "options":
            got = [[o.option_type, o.length, o.payload.hex()] for o in got]
        elif f in ("target_addr", "dest_addr"):
            got = str(got)
        assert got == want, (name, f, got, want)


def check_ndp_view(rec, frame: bytes, v: dict, name=""):
    """icmpv6.rs ndp_tests on a parsed record: the ICMPv6 message located by
    the record decoded with Packet::from_bytes (what the tests call) and the
    Icmpv6Packet of the Frame through TryFrom (what dump.rs calls), each
    asserted as the reference test asserts."""
    from nex_amd import views
    cls = views.NDP_VIEWS[NDP_KINDS[v["kind"]]]
    msg = views.icmpv6_message_bytes(rec, frame)
    assert msg is not None, name
    m = cls.from_bytes(msg)
    assert m.header.icmp_type == NDP_KINDS[v["kind"]] and m.header.icmp_code == 0, name
    assert m.header.checksum == v.get("l4_csum", m.header.checksum), name
    ndp_fields_equal(m, v, name)
    assert m.to_bytes() == msg, name  # the message re-serialises to itself
    tf = v.get("try_from")
    pkt = views.icmpv6_from_record(rec, frame)
    if tf == "same":
        ndp_fields_equal(cls.try_from(pkt), v, name)
    elif tf is not None:
        try:
            cls.try_from(pkt)
        except views.ViewError as e:
            assert str(e) == tf, (name, str(e), tf)
        else:
            raise AssertionError(f"{name}: TryFrom should fail with {tf!r}")


def records_equal(a: np.ndarray, b: np.ndarray, frames=None, what=""):
    """Bit-exact comparison of two record (or desc) arrays with a readable diff."""
    assert a.dtype == b.dtype and a.shape == b.shape, (a.dtype, b.dtype, a.shape, b.shape)
    ab, bb = a.view(np.uint8).reshape(len(a), -1), b.view(np.uint8).reshape(len(b), -1)
    bad = np.nonzero((ab != bb).any(axis=1))[0]
    if len(bad):
        i = int(bad[0])
        diffs = [n for n in a.dtype.names if a[i][n] != b[i][n]]
        detail = {n: (int(a[i][n]), int(b[i][n])) for n in diffs}
        fr = "" if frames is None else bytes(frames[i]).hex()
        raise AssertionError(f"{what}: {len(bad)} of {len(a)} records differ; first #{i}: "
                             f"{detail} frame={fr}")


# ---- malformed / edge-case mixes (SURVEY.md App. C "malformed mix") ---------

def _ipv4(payload, proto, ihl=5, opts=b"", total=None, ident=0x1234, flags_frag=0x4000):
    hl = 20 + len(opts)
    tot = hl + len(payload) if total is None else total
    h = bytes([0x40 | ihl, 0, tot >> 8 & 255, tot & 255, ident >> 8, ident & 255,
               flags_frag >> 8, flags_frag & 255, 64, proto, 0, 0, 10, 1, 2, 3, 10, 4, 5, 6])
    return h + opts + payload


def _eth(p, et=0x0800):
    return bytes(range(1, 13)) + et.to_bytes(2, "big") + p


def _ipv6(payload, nh, plen=None):
    plen = len(payload) if plen is None else plen
    return (bytes([0x6a, 0xbc, 0xde, 0xf1]) + plen.to_bytes(2, "big") + bytes([nh, 64]) +
            bytes(range(16)) + bytes(range(16, 32)) + payload)


def _tcp(payload, opts=b"", doff=None):
    d = (20 + len(opts)) // 4 if doff is None else doff
    return bytes([0x12, 0x34, 0x00, 0x50, 1, 2, 3, 4, 5, 6, 7, 8, (d << 4) | 0x3, 0x18, 0x20, 0,
                  0xAB, 0xCD, 0, 7]) + opts + payload


def _udp(payload, length=None):
    ln = 8 + len(payload) if length is None else length
    return bytes([0x04, 0xd2, 0x00, 0x35, ln >> 8, ln & 255, 0x12, 0x34]) + payload


def crafted_frames():
    """Deterministic edge cases for every quirk in SURVEY.md Appendix A."""
    P = bytes(range(37))
    f = []
    f.append(b"")                                             # Q2 empty
    f.append(bytes(13))                                       # Q2 < 14
    f.append(_eth(b"", 0x0800))                               # IPv4 with 0 bytes
    f.append(_eth(P[:19], 0x0800))                            # Q4 < 20
    f.append(_eth(bytes([0x55]) + bytes(19), 0x0800))         # Q4 version
    f.append(_eth(bytes([0x44]) + bytes(19), 0x0800))         # Q4 ihl < 5
    f.append(_eth(bytes([0x4f]) + bytes(30), 0x0800))         # Q4 ihl*4 > len
    f.append(_eth(_ipv4(_udp(P), 17, total=10)))              # Q4 total < ihl
    f.append(_eth(_ipv4(_udp(P), 17, total=0)))               # Q5 zero total
    f.append(_eth(_ipv4(_udp(P), 17, total=200)))             # Q5 declared > captured
    f.append(_eth(_ipv4(_udp(P), 17)) + bytes(9))             # Q5 Ethernet padding
    f.append(_eth(_ipv4(_udp(P, length=7), 17)))              # Q14 UDP length < 8
    f.append(_eth(_ipv4(_udp(P, length=100), 17)))            # Q14 UDP length > avail
    f.append(_eth(_ipv4(_udp(P, length=20), 17)))             # Q14 bytes beyond UDP length
    f.append(_eth(_ipv4(_udp(P[:3]), 17)))                    # odd UDP length
    f.append(_eth(_ipv4(P[:5], 17)))                          # UDP < 8
    f.append(_eth(_ipv4(_tcp(P), 6)))
    f.append(_eth(_ipv4(_tcp(P, doff=4), 6)))                 # Q13 doff < 5
    f.append(_eth(_ipv4(_tcp(P[:3], doff=15), 6)))            # Q13 doff*4 > len
    f.append(_eth(_ipv4(_tcp(P, opts=b"\x01\x01\x08\x0a" + bytes(8)), 6)))   # NOP NOP TS
    f.append(_eth(_ipv4(_tcp(P, opts=b"\x02\x04\x05\xb4\x00\x13\x22\x33"), 6)))  # MSS EOL junk
    f.append(_eth(_ipv4(_tcp(P, opts=b"\x00\x99\x99\x99\x11\x22\x33\x44"), 6)))  # early EOL
    f.append(_eth(_ipv4(_tcp(P, opts=b"\x01\x01\x01\x02"), 6)))          # kind w/o length
    f.append(_eth(_ipv4(_tcp(P, opts=b"\x05\x01\x00\x00"), 6)))          # len < 2
    f.append(_eth(_ipv4(_tcp(P, opts=b"\x05\x09\x00\x00"), 6)))          # overflow
    f.append(_eth(_ipv4(_tcp(P[:1], opts=b"\x03\x03\x07\x00"), 6)))      # odd payload
    f.append(_eth(_ipv4(P, 1)))                                # ICMP
    f.append(_eth(_ipv4(bytes(7), 1)))                         # Q15 ICMP < 8
    f.append(_eth(_ipv4(bytes(8), 1)))                         # ICMP all-zero (csum 0xFFFF)
    f.append(_eth(_ipv4(P, 200)))                              # Q8 proto 200 -> 255
    f.append(_eth(_ipv4(P, 255)))
    f.append(_eth(_ipv4(P, 50)))                               # Q9 other proto
    f.append(_eth(_ipv4(_udp(P), 17, flags_frag=0x2001)))      # Q7 fragment
    # IPv4 options (Q6, Q16, Q17)
    f.append(_eth(_ipv4(_udp(P), 17, ihl=7, opts=b"\x01\x87\x04\x12\x34\x00\x00\x00")))
    f.append(_eth(_ipv4(_udp(P), 17, ihl=7, opts=b"\x00\x11\x22\x33\x44\x55\x66\x77")))  # EOL first
    f.append(_eth(_ipv4(_udp(P), 17, ihl=8, opts=b"\x01\x00" + bytes(10))))
    f.append(_eth(_ipv4(_udp(P), 17, ihl=6, opts=b"\x07")))   # no room for length
    f.append(_eth(_ipv4(_udp(P), 17, ihl=6, opts=b"\x07\x01\x00\x00")))  # len < 2
    f.append(_eth(_ipv4(_udp(P), 17, ihl=6, opts=b"\x07\x09\x00\x00")))  # overflow
    f.append(_eth(_ipv4(b"", 17, ihl=15, opts=b"\x00" + bytes(39))))       # Q17 panic case
    f.append(_eth(_ipv4(P[:6], 17, ihl=15, opts=b"\x00" + bytes(39))))    # Q17 window into payload
    f.append(_eth(_ipv4(_udp(P), 17, ihl=15, opts=b"\x01" * 40)))
    # IPv6 (Q10-Q12)
    f.append(_eth(_ipv6(_udp(P), 17), 0x86DD))
    f.append(_eth(_ipv6(_tcp(P), 6), 0x86DD))
    f.append(_eth(_ipv6(_tcp(P, opts=b"\x01\x01\x08\x0a" + bytes(8)), 6), 0x86DD))
    f.append(_eth(_ipv6(P, 58), 0x86DD))
    f.append(_eth(_ipv6(P[:7], 58), 0x86DD))
    f.append(_eth(_ipv6(_udp(P), 17, plen=0), 0x86DD))        # Q11 payload_length 0
    f.append(_eth(_ipv6(_udp(P), 17, plen=500), 0x86DD))      # Q11 > captured
    f.append(_eth(_ipv6(bytes([17, 0]) + bytes(6) + _udp(P), 0), 0x86DD))   # HBH
    f.append(_eth(_ipv6(bytes([44, 1]) + bytes(14) + bytes([17, 0]) + bytes(6) + _udp(P), 60), 0x86DD))
    f.append(_eth(_ipv6(bytes([6, 0, 0, 1]) + bytes(4) + _tcp(P), 44), 0x86DD))   # Frag
    f.append(_eth(_ipv6(bytes([17, 0, 0, 0]) + bytes(4) + _udp(P), 43), 0x86DD))  # Route
    f.append(_eth(_ipv6(bytes([17, 9]), 0), 0x86DD))          # Q12 truncated ext
    f.append(_eth(_ipv6(bytes([17]), 0), 0x86DD))             # Q12 no room
    f.append(_eth(_ipv6(bytes([17, 0, 0]), 43), 0x86DD))      # route < 4
    f.append(_eth(_ipv6(bytes([17, 0, 0, 0, 0]), 44), 0x86DD))  # frag < 8
    f.append(_eth(_ipv6(_udp(P), 51), 0x86DD))                # AH not walked
    f.append(_eth(_ipv6(_udp(P), 200), 0x86DD))               # reserved
    f.append(_eth(bytes([0x50]) + bytes(45), 0x86DD))         # version
    f.append(_eth(bytes(39), 0x86DD))                         # < 40
    # ARP / VLAN / misc EtherTypes (Q3)
    f.append(_eth(bytes(range(28)), 0x0806))
    f.append(_eth(bytes(range(27)), 0x0806))
    f.append(_eth(bytes(range(40)), 0x0806))
    f.append(_eth(b"\x20\x01\x08\x00" + _ipv4(_udp(P), 17), 0x8100))
    f.append(_eth(P, 0x88CC))
    f.append(_eth(b"", 0x1234))
    return f


def mutate_frames(rng: np.random.Generator, base, n: int):
    """Random structural mutations of valid frames (fuzz-corpus style)."""
    out = []
    for _ in range(n):
        fr = bytearray(base[int(rng.integers(len(base)))])
        k = int(rng.integers(8))
        if k == 0 and len(fr):                       # truncate
            fr = fr[: int(rng.integers(len(fr) + 1))]
        elif k == 1 and len(fr) > 14:                # flip random header bytes
            for _ in range(int(rng.integers(1, 4))):
                j = int(rng.integers(14, min(len(fr), 80)))
                fr[j] = int(rng.integers(256))
        elif k == 2 and len(fr) > 17:                # random total length / payload length
            j = 16 if fr[12:14] == b"\x08\x00" else 18
            fr[j:j + 2] = int(rng.integers(0, 1 << 16)).to_bytes(2, "big")
        elif k == 3 and len(fr) > 14:                # random IHL / version nibble
            fr[14] = int(rng.integers(256))
        elif k == 4:                                 # append padding / junk
            fr += bytes(rng.integers(0, 256, int(rng.integers(1, 64)), dtype=np.uint8))
        elif k == 5 and len(fr) > 46:                # random L4 length-ish fields
            for j in (38, 39, 46, 47, 58, 59, 66):
                if j < len(fr) and rng.random() < 0.4:
                    fr[j] = int(rng.integers(256))
        elif k == 6:                                 # random bytes frame
            fr = bytearray(rng.integers(0, 256, int(rng.integers(0, 200)), dtype=np.uint8))
        out.append(bytes(fr))
    return out


def slice_frames():
    """Extra edge cases for FrameSlice (frame.rs:84-287): AH walks, extension
    truncation at each check, ARP lengths, tiny transports, from-IP prefixes."""
    P = bytes(range(60))
    f = []
    for ah_len in (0, 1, 4):
        ah = bytes([17, ah_len]) + bytes((ah_len + 2) * 4 - 2)
        f.append(_eth(_ipv6(ah + _udp(P[:9]), 51), 0x86DD))
    hbh = bytes([51, 0]) + bytes(6)
    f.append(_eth(_ipv6(hbh + bytes([6, 1]) + bytes(10) + _tcp(P[:5]), 0), 0x86DD))  # HBH -> AH -> TCP
    f.append(_eth(_ipv6(bytes([17, 0]) + bytes(6) + _udp(b""), 44), 0x86DD))         # fragment
    f.append(_eth(_ipv6(bytes([58, 0]) + bytes(6) + bytes(4), 60), 0x86DD))            # dest opts -> ICMPv6 4 B
    f.append(_eth(_ipv6(bytes([17]), 0), 0x86DD))                                       # ext: cursor+2 > len
    f.append(_eth(_ipv6(bytes([17, 0]) + bytes(3), 43), 0x86DD))                        # ext overruns
    f.append(_eth(_ipv6(bytes([17]), 51), 0x86DD))                                      # AH: cursor+2 > len
    f.append(_eth(_ipv6(bytes([17, 9]) + bytes(4), 51), 0x86DD))                        # AH overruns
    f.append(_eth(_ipv6(bytes(8), 44, plen=4), 0x86DD))                                 # fragment past plen
    f.append(_eth(_ipv6(_udp(P[:3]), 17, plen=0), 0x86DD))                             # plen 0: no transport
    f.append(_eth(_ipv6(_tcp(P[:3], doff=15), 6), 0x86DD))
    f.append(_eth(_ipv4(bytes(3), 1)))                                                 # ICMP < 4
    f.append(_eth(_ipv4(bytes(4), 58)))                                                # ICMPv6 in IPv4
    f.append(_eth(_ipv4(_udp(P, length=2), 17)))
    f.append(_eth(bytes(27), 0x0806))
    f.append(_eth(bytes(28), 0x0806))
    f.append(_eth(bytes(40), 0x0806))
    f.append(_eth(P[:20], 0x8100))
    return f


def vlan(frame: bytes, tags, tpids=None) -> bytes:
    """Insert 802.1Q-style tags (TCI values) after the MAC addresses."""
    tpids = tpids or [0x8100] * len(tags)
    ins = b"".join(t.to_bytes(2, "big") + tci.to_bytes(2, "big") for t, tci in zip(tpids, tags))
    return frame[:12] + ins + frame[12:]


def tcp_ts_frames(oracle, base, rng, fix_checksums=True):
    """Real-traffic TCP shape: NOP, NOP, Timestamps (RFC 7323) inserted after
    the 20-B TCP header of every TCP frame in `base` (IPv4 and IPv6), data
    offset 8, IP lengths grown by 12; with fix_checksums the oracle's computed
    IPv4 / TCP checksums are written back (valid frames), else left stale.
    Plus edge variants: the option bytes perturbed (other layouts), doff 8
    without room for the options, and truncated copies."""
    out = []
    for f in base:
        v4 = f[12:14] == b"\x08\x00"
        l4 = 34 if v4 else 54
        if len(f) < l4 + 20 or f[23 if v4 else 20] != 6:
            continue
        ts = bytes([1, 1, 8, 10]) + bytes(rng.integers(0, 256, 8, dtype=np.uint8))
        g = bytearray(f[:l4 + 20] + ts + f[l4 + 20:])
        g[l4 + 12] = (8 << 4) | (g[l4 + 12] & 0x0F)
        if v4:
            tl = int.from_bytes(g[16:18], "big") + 12
            g[16:18] = tl.to_bytes(2, "big")
        else:
            pl = int.from_bytes(g[18:20], "big") + 12
            g[18:20] = pl.to_bytes(2, "big")
        if fix_checksums:
            r = oracle.parse_frame(bytes(g))
            if v4:
                g[24:26] = int(r["ip_csum_calc"]).to_bytes(2, "big")
            g[l4 + 16:l4 + 18] = int(r["l4_csum_calc"]).to_bytes(2, "big")
        out.append(bytes(g))
        h = bytearray(g)
        h[l4 + 20 + int(rng.integers(4))] = int(rng.choice([0, 1, 2, 3, 8, 10, 255]))
        out.append(bytes(h))
        out.append(bytes(g[: int(rng.integers(l4, len(g)))]))
    return out


def tcp_option_frames(oracle, base, rng):
    """TCP frames of `base` with one-TLV option lists the register path takes
    (MSS alone; NOP NOP SACK with 1-4 blocks; NOP NOP any-kind TLV) and near
    misses (a length one off, EOL / NOP inside, two TLVs), valid checksums."""
    out = []
    lists = [bytes([2, 4, 5, 180]),                                     # MSS (SYN-ACK)
             *[bytes([1, 1, 5, 2 + 8 * k]) + bytes(rng.integers(0, 256, 8 * k, dtype=np.uint8)) for k in (1, 2, 3, 4)],
             bytes([1, 1, 30, 6, 9, 9, 9, 9]),                          # unknown kind, NOP NOP form
             bytes([3, 3, 7, 0]),                                       # WS + EOL pad (not one TLV)
             bytes([1, 1, 5, 11]) + bytes(9),                           # SACK length one off
             bytes([2, 4, 5, 180, 1, 3, 3, 7]),                         # two TLVs
             bytes([1, 1, 1, 1])]                                       # NOPs only
    for i, f in enumerate(base):
        v4 = f[12:14] == b"\x08\x00"
        l4 = 34 if v4 else 54
        if len(f) < l4 + 20 or f[23 if v4 else 20] != 6:
            continue
        opts = lists[i % len(lists)]
        opts = opts + bytes((-len(opts)) % 4)
        g = bytearray(f[:l4 + 20] + opts + f[l4 + 20:])
        g[l4 + 12] = ((5 + len(opts) // 4) << 4) | (g[l4 + 12] & 0x0F)
        k = 16 if v4 else 18
        g[k:k + 2] = (int.from_bytes(g[k:k + 2], "big") + len(opts)).to_bytes(2, "big")
        r = oracle.parse_frame(bytes(g))
        if v4:
            g[24:26] = int(r["ip_csum_calc"]).to_bytes(2, "big")
        g[l4 + 16:l4 + 18] = int(r["l4_csum_calc"]).to_bytes(2, "big")
        out.append(bytes(g))
    return out


def vlan_frames():
    """VLAN-extension cases: single / double / QinQ tags over every inner type,
    truncated tags, three tags (only two unwrapped)."""
    P = bytes(range(40))
    inner = [_eth(_ipv4(_udp(P), 17)), _eth(_ipv4(_tcp(P), 6)), _eth(_ipv4(P[:12], 1)),
             _eth(_ipv6(_udp(P), 17), 0x86DD), _eth(bytes(28), 0x0806), _eth(P[:20], 0x88B5),
             _eth(bytes([0x44]) + bytes(19))]
    f = []
    for x in inner:
        f.append(vlan(x, [0x0064]))
        f.append(vlan(x, [0xE00A, 0x0123], [0x88A8, 0x8100]))
        f.append(vlan(x, [1, 2], [0x9100, 0x8100]))
        f.append(vlan(x, [1, 2, 3]))
    f.append(bytes(12) + b"\x81\x00\x00")            # tag cut short
    f.append(bytes(12) + b"\x81\x00\x00\x01\x08")    # inner EtherType cut short
    f.append(bytes(12) + b"\x81\x00\x00\x01\x08\x00")  # tag complete, nothing after
    return f


def tcp_option_lists(rng):
    """Systematic TCP option lists around the register path's one-TLV branch
    (frame_core.hpp fast_canonical80: `one` = kind >= 2 with length == the
    option bytes; `nnx` = NOP NOP + kind >= 2 with 2 + length == the option
    bytes), for every data offset 6..15: the branch's own shapes (MSS alone,
    SACK 1-4 blocks, timestamps, any kind) and the near misses either side
    (lengths one off, EOL / NOP where the TLV should be, lengths 0 / 1, two
    TLVs, NOPs only). The reference's walk and re-serialisation are
    tcp.rs:731-836 and :521-575."""
    rnd = lambda n: bytes(rng.integers(0, 256, max(0, n), dtype=np.uint8))
    out = []
    for olen in range(4, 41, 4):
        for kind in (2, 3, 4, 5, 8, 30, 254):
            for d in (0, 0, 0, -1, 1, -olen + 2):  # the branch's own shape three times
                ln = olen + d
                if 0 <= ln < 256:
                    out.append(bytes([kind, ln]) + rnd(olen - 2))
        for kind in (5, 8, 19, 2, 255):
            for d in (0, 0, 0, -1, 1):
                ln = olen - 2 + d
                if 0 <= ln < 256:
                    out.append(bytes([1, 1, kind, ln]) + rnd(olen - 4))
        out.append(bytes([1, 1, 0, olen - 2]) + rnd(olen - 4))      # EOL where the kind goes
        out.append(bytes([1, 1, 1, olen - 2]) + rnd(olen - 4))      # a third NOP
        out.append(bytes([1, 1, 5, 1]) + rnd(olen - 4))             # length 1
        out.append(bytes([1, 1, 5, 0]) + rnd(olen - 4))             # length 0
        out.append(bytes([0, olen]) + rnd(olen - 2))                # EOL first (rest is padding)
        out.append(bytes([1, olen - 1]) + rnd(olen - 2))            # one NOP, then junk
        out.append(bytes([1, 2, olen - 2]) + rnd(olen - 3))         # NOP + TLV (not two NOPs)
        out.append(bytes([1]) * olen)                               # NOPs only
        if olen >= 8:
            out.append(bytes([2, 4, 5, 180, 5, olen - 4]) + rnd(olen - 6))        # two TLVs
            out.append(bytes([1, 1, 8, 10]) + rnd(8) + bytes(olen - 12) if olen >= 12 else
                       bytes([1, 1, 8, olen - 2]) + rnd(olen - 4))                  # TS + EOL padding
            out.append(bytes([1, 1, 5, olen - 6]) + rnd(olen - 8) + bytes([1, 1, 1, 0]))  # TLV short, NOPs
    return out


def tcp_option_sweep(oracle, rng, bases):
    """Every list of tcp_option_lists() put behind TCP frames of `bases`
    (IPv4 and IPv6, several payload lengths incl. 0 and odd), data offset and
    IP length set to fit; per frame the checksum-valid form (oracle's computed
    IPv4 / TCP checksums written back), a copy with one payload or option
    byte flipped (L4 verdict false), an IPv4 copy with a stale header
    checksum, and a copy truncated inside the option area (no TcpPacket)."""
    tcp = []
    for f in bases:
        v4 = f[12:14] == b"\x08\x00"
        l4 = 34 if v4 else 54
        if len(f) >= l4 + 20 and f[23 if v4 else 20] == 6:
            tcp.append((f, v4, l4))
    assert len(tcp) >= 4
    out = []
    lists = tcp_option_lists(rng)
    for i, opts in enumerate(lists):
        for j in range(3):
            f, v4, l4 = tcp[(3 * i + j) % len(tcp)]
            g = bytearray(f[:l4 + 20] + opts + f[l4 + 20:])
            g[l4 + 12] = ((5 + len(opts) // 4) << 4) | (g[l4 + 12] & 0x0F)
            k = 16 if v4 else 18
            g[k:k + 2] = (int.from_bytes(g[k:k + 2], "big") + len(opts)).to_bytes(2, "big")
            r = oracle.parse_frame(bytes(g))
            if v4:
                g[24:26] = int(r["ip_csum_calc"]).to_bytes(2, "big")
            if r["l4_csum_calc"] or r["flags"] & abi.C_L4_CHECKED:
                g[l4 + 16:l4 + 18] = int(r["l4_csum_calc"]).to_bytes(2, "big")
            out.append(bytes(g))
            h = bytearray(g)
            h[int(rng.integers(l4 + 20, len(h)))] ^= 0x24
            out.append(bytes(h))
            if v4 and j == 0:
                h = bytearray(g)
                h[25] ^= 0x01
                out.append(bytes(h))
            if j == 1:
                out.append(bytes(g[: l4 + 20 + int(rng.integers(0, len(opts)))]))
    return out


def host_malformed_mix(oracle, count, seed=77, mutate_share=0.5, kinds=None):
    """The bench's malformed mix built on the host: IMIX frames from the
    oracle's generator (the device generator's restatement), mutated by
    nex_amd.workloads.mutate_packed. (bytes, count+1 offsets, counts)."""
    from nex_amd import abi, workloads
    frames = [oracle.gen_frame(abi.WL_IMIX, i, seed=seed) for i in range(count)]
    offs = np.zeros(count + 1, np.int64)
    np.cumsum([len(f) for f in frames], out=offs[1:])
    data = np.frombuffer(b"".join(bytes(f) for f in frames), np.uint8)
    return workloads.mutate_packed(data, offs, seed, mutate_share, kinds or workloads.MUTATIONS)


def fastpath_edge_frames(rng):
    """The register fast path's round-3 shapes and their near misses:
    frames of 0..13 B (Q2); IPv6 with one extension header (hop-by-hop,
    routing, fragment, destination options) of every small length, ahead of
    TCP / UDP / ICMPv6 / no-next-header / another extension, with payload
    lengths that end exactly at, one before and past its end; TCP data offsets
    6..15 whose first option is a TLV of length 0, 1, 2, the list's length,
    one past it and 255 (walk fails or goes on), behind NOP / EOL too; IPv4
    option lists (ipv4_option_frames: declined to the generic walk)."""
    f = [bytes(rng.integers(0, 256, n, dtype=np.uint8)) for n in range(14)]
    f += [bytes(range(12)) + bytes([0x86, 0xDD]) + bytes(rng.integers(0, 256, k, dtype=np.uint8)) for k in (0, 39, 41)]
    for nh in (0, 43, 44, 60):
        for el in (0, 1, 2, 5):
            for nh2 in (6, 17, 58, 59, 0, 60, 200):
                tl = 8 if nh == 44 else 8 + 8 * el
                ext = bytes([nh2, el]) + bytes(rng.integers(0, 256, tl - 2, dtype=np.uint8))
                body = bytes(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8))
                pl = len(ext) + len(body)
                for plen in (pl, tl, tl - 1, 1, 0, pl + 9, 1500):
                    f.append(_eth(_ipv6(ext + body, nh, plen=plen), 0x86DD))
                f.append(_eth(_ipv6(ext[:tl - 3], nh, plen=tl), 0x86DD))  # header cut by the frame end
    for fam in (4, 6):
        for doff in range(6, 16):
            olen = 4 * doff - 20
            for first in (0, 1, 2, 3, 8, 30, 200):
                for ln in sorted({0, 1, 2, 3, olen - 1, olen, olen + 1, 255}):
                    opts = bytes([first, ln & 255]) + bytes(rng.integers(0, 256, olen - 2, dtype=np.uint8))
                    pay = bytes(rng.integers(0, 256, int(rng.choice([0, 5, 40, 600])), dtype=np.uint8))
                    seg = _tcp(pay, opts, doff=doff)
                    f.append(_eth(_ipv4(seg, 6)) if fam == 4 else _eth(_ipv6(seg, 6), 0x86DD))
    f += ipv4_option_frames(rng)
    f += tcp_walk_frames(rng)
    return f


def tcp_walk_frames(rng):
    """TCP option lists the general walk (round 4: tcp.rs:767-818 through the
    span kernel's lane slot) takes or refuses: the SYN lists of common stacks
    (MSS, SACK permitted, timestamps, NOP, window scale; with and without EOL
    padding), lists that stop at an EOL with non-zero bytes after it (dropped
    from the re-serialised header and its checksum), NOP runs, TLVs that cut
    the list later than the first option (Q13), behind IPv4 headers with and
    without options and IPv6, payloads 0..600 B."""
    ts = bytes([8, 10]) + bytes(rng.integers(0, 256, 8, dtype=np.uint8))
    lists = [bytes([2, 4, 5, 0xb4, 4, 2]) + ts + bytes([1, 3, 3, 7]),               # Linux SYN (doff 10)
             bytes([2, 4, 5, 0xb4, 1, 3, 3, 8, 1, 1, 4, 2]),                        # Windows SYN (doff 8)
             bytes([2, 4, 5, 0xb4, 1, 3, 3, 6, 1, 1]) + ts + bytes([4, 2, 0, 0]),   # macOS SYN (doff 11, EOL)
             bytes([2, 4, 5, 0xb4, 0, 9, 9, 9]),                                    # EOL, junk after it
             bytes([1, 1, 0, 0xFF, 0xEE, 0xDD, 0xCC, 0xBB]),                        # NOP NOP EOL junk
             bytes([0]) + bytes([0x5A] * 7),                                        # EOL first
             bytes([1] * 12),                                                       # NOP run
             bytes([3, 3, 7, 1, 2, 4, 5]) + bytes([0]),                             # WS, NOP, MSS, EOL
             bytes([2, 4, 5, 0xb4, 3, 3, 7, 8, 9, 9, 9, 9]),                        # 2nd TLV past the list
             bytes([2, 4, 5, 0xb4, 3, 1, 1, 1]),                                    # 2nd TLV length 1
             bytes([2, 4, 5, 0xb4, 3, 5, 7, 7]),                                    # 2nd TLV one byte past the list
             bytes([2, 4, 5, 0xb4, 3, 4, 7, 7]),                                    # 2nd TLV ends the list exactly
             bytes([2, 4, 5, 0xb4, 1, 1, 1, 3]),                                    # TLV kind at the last byte
             bytes([4, 2, 8, 10]) + bytes(8) + bytes([1, 3, 3, 7, 2, 4, 5, 0xb4, 0, 0, 0, 0])]  # doff 10 / EOL run
    f = []
    for opts in lists:
        for plen in (0, 1, 6, 40, 600):
            body = bytes(rng.integers(0, 256, plen, dtype=np.uint8))
            seg = _tcp(body, opts)
            f.append(_eth(_ipv4(seg, 6)))
            f.append(_eth(_ipv4(seg, 6, ihl=6, opts=bytes([1, 1, 1, 0]))))
            f.append(_eth(_ipv6(seg, 6), 0x86DD))
            f.append(_eth(_ipv4(seg, 6)) + bytes(5))  # Ethernet padding
    return f


def ipv4_option_frames(rng):
    """IPv4 headers with options (IHL 6..15) ahead of UDP / TCP / ICMP / other
    protocols: Router Alert, NOP runs, EOL early (re-serialised header shorter
    than IHL: payload bytes in its checksum, Q17 when the payload is shorter
    still), timestamps, TLVs of length 0 / 1 / past the header / cut by it,
    random bytes; total lengths exact, 0, short of the frame (padding) and
    past it; payloads of 0..600 B."""
    f = []
    for ihl in range(6, 16):
        ol = 4 * (ihl - 5)
        lists = [bytes([0x94, 4, 0, 0]) + bytes([1] * (ol - 4)), bytes([1] * ol), bytes([0]) + bytes([7] * (ol - 1)),
                 bytes([1] * (ol - 1)) + bytes([0x44]), bytes([0x44, ol, 5, 0x10]) + bytes(ol - 4),
                 bytes([0x83, 0]) + bytes(ol - 2), bytes([0x83, 1]) + bytes(ol - 2),
                 bytes([0x83, ol + 1]) + bytes(ol - 2), bytes([1, 0x88, 3, 9, 9]) + bytes([0]) * (ol - 5) if ol >= 8
                 else bytes([0x88, 4, 9, 9]), bytes([1, 1, 0]) + bytes([0xFF]) * (ol - 3),
                 bytes(rng.integers(0, 256, ol, dtype=np.uint8))]
        for opts in lists:
            for proto in (17, 6, 1, 200):
                for plen in (0, 3, 7, 9, 20, 45, 600):
                    body = bytes(rng.integers(0, 256, plen, dtype=np.uint8))
                    seg = (_udp(body) if proto == 17 else _tcp(body) if proto == 6 and plen >= 20 else
                           _tcp(body[:4], bytes([1, 1, 8, 10]) + body[4:12]) if proto == 6 and plen == 9 else
                           bytes([8, 0, 0, 0]) + body if proto == 1 else body)
                    ip = _ipv4(seg, proto, ihl=ihl, opts=opts)
                    f.append(_eth(ip))
                    tot = len(ip)
                    for t in (0, tot - 1, tot + 5, 4 * ihl):
                        f.append(_eth(_ipv4(seg, proto, ihl=ihl, opts=opts, total=t)))
                    f.append(_eth(ip) + bytes(rng.integers(0, 256, int(rng.integers(1, 30)), dtype=np.uint8)))
    return f


def probe_oracle_build(oracle, shape, dst_host, nthreads=1, out=None):
    """The oracle's frames of a nex_amd.probes shape for numpy destinations
    ((count, 4|16) uint8): oracle.build_probe_batch over probes.oracle_args."""
    from nex_amd import probes
    kind, spec, l4 = probes.oracle_args(shape)
    spec = dict(spec)
    fam = spec.pop("family")
    sp = oracle.ip_spec(fam, spec.pop("src"), bytes(16 if fam == 6 else 4), **spec)
    return oracle.build_probe_batch(kind, sp, dst_host, nthreads=nthreads, out=out, **l4)
