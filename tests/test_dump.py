"""examples/dump.rs counterpart (nex_amd.views / nex_amd.dump), on the CPU
over oracle records: the layer-by-layer lines for the reference's own test
packets, the ICMP / ICMPv6 sub-message views with the reference's rules
(icmp.rs:434-700: 4-B minimum; icmpv6 echo: 8-B minimum; NDP fixed parts)
and error strings, and the walk on every crafted / mutated frame without an
exception escaping. The GPU half compares views from GPU and oracle records."""
import numpy as np
import pytest

from nex_amd import abi, views
from nex_amd.frame import IcmpHeader
from tests import helpers


def rec_of(oracle, frame, flags=0, ip_offset=0):
    return oracle.parse_frame(frame, flags, ip_offset)


def golden(name):
    for v in helpers.golden()["frames"]:
        if v["name"] == name:
            return bytes.fromhex(v["frame"])
    raise KeyError(name)


def test_dump_lines_reference_packets(oracle):
    fr = golden("icmp_echo_request")
    assert views.dump_lines(rec_of(oracle, fr), fr) == [
        "ICMP echo request 10.0.0.1 -> 10.0.0.2 (seq=42, id=1234), length: 12"]
    fr = golden("icmp_destination_unreachable")
    assert views.dump_lines(rec_of(oracle, fr), fr) == [
        "ICMP destination unreachable 10.0.0.1 -> 10.0.0.2 (code=IcmpCode(3)), next_hop_mtu=1500, length: 14"]
    fr = golden("icmp_time_exceeded")
    assert views.dump_lines(rec_of(oracle, fr), fr) == [
        "ICMP time exceeded 10.0.0.1 -> 10.0.0.2 (code=IcmpCode(0)), length: 15"]
    fr = golden("udp_basic_parse")
    assert views.dump_lines(rec_of(oracle, fr), fr) == ["UDP Packet: 10.0.0.1:4660 > 10.0.0.2:43981; length: 12"]
    fr = golden("tcp_basic_parse")  # 20 + NOP NOP TS(10) -> 32 + 4 B payload
    assert views.dump_lines(rec_of(oracle, fr), fr) == ["TCP Packet: 10.0.0.1:49511 > 10.0.0.2:9000; length: 36"]
    fr = golden("icmpv6_echo_request_parse")
    assert views.dump_lines(rec_of(oracle, fr), fr) == [
        "ICMPv6 echo request ::1 -> ::1 (type=EchoRequest), length: 13"]


def test_dump_lines_other_layers(oracle):
    P = bytes(range(40))
    cases = [
        (helpers._eth(P, 0x88CC), "LLDP packet: 07:08:09:0a:0b:0c > 01:02:03:04:05:06; ethertype: Lldp length: 54"),
        (helpers._eth(P, 0x1234), "Unknown packet: 07:08:09:0a:0b:0c > 01:02:03:04:05:06; ethertype: Unknown(4660) "
                                  "length: 54"),
        (helpers._eth(bytes([0x44]) + bytes(19)), "Malformed IPv4 Packet"),
        (helpers._eth(bytes(39), 0x86DD), "Malformed IPv6 Packet"),
        (helpers._eth(bytes(27), 0x0806), "Malformed ARP Packet"),
        (helpers._eth(helpers._ipv4(P, 200)), "Unknown IPv4 packet: 10.1.2.3 > 10.4.5.6; protocol: Reserved length: 40"),
        (helpers._eth(helpers._ipv4(helpers._tcp(P, doff=4), 6)), "Malformed TCP Packet"),
        (helpers._eth(helpers._ipv4(helpers._udp(P, length=100), 17)), "Malformed UDP Packet"),
        (helpers._eth(helpers._ipv4(bytes(7), 1)), "Malformed ICMP Packet"),
        (helpers._eth(helpers._ipv4(bytes([8, 0, 0, 0, 1, 2, 3, 4]) + b"x", 58)),  # ICMPv6 inside IPv4 (dump.rs:179)
         "ICMPv6 packet 10.1.2.3 -> 10.4.5.6 (type=Unknown(8)), length: 9"),
    ]
    for fr, want in cases:
        assert views.dump_lines(rec_of(oracle, fr), fr) == [want], fr.hex()
    arp = helpers._eth(bytes([0, 1, 8, 0, 6, 4, 0, 2]) + bytes(range(6)) + bytes([192, 168, 0, 1]) +
                       bytes(range(6, 12)) + bytes([192, 168, 0, 2]), 0x0806)
    assert views.dump_lines(rec_of(oracle, arp), arp) == [
        "ARP packet: 00:01:02:03:04:05(192.168.0.1) > 06:07:08:09:0a:0b(192.168.0.2); operation: Reply"]


def test_icmp_views_rules():
    h = IcmpHeader(8, 0, 0)
    with pytest.raises(views.ViewError, match="Payload too short for Echo Request"):
        views.EchoRequestPacket.try_from(views.IcmpPacket(h, b"\x00\x01\x00"))
    with pytest.raises(views.ViewError, match="Not an Echo Reply"):
        views.EchoReplyPacket.try_from(views.IcmpPacket(h, b"\x00" * 8))
    m = views.TimeExceededPacket.try_from(views.IcmpPacket(IcmpHeader(11, 1, 0), b"\xde\xad\xbe\xefxyz"))
    assert (m.unused, m.payload) == (0xdeadbeef, b"xyz")
    # ICMPv6 echo needs 8 payload bytes where ICMPv4's needs 4 (icmpv6.rs:2282-2284)
    with pytest.raises(views.ViewError, match="Payload too short for Echo Request"):
        views.Icmpv6EchoPacket.try_from(views.Icmpv6Packet(IcmpHeader(128, 0, 0), b"\x00" * 7))
    ns = views.NeighborSolicitPacket.try_from(views.Icmpv6Packet(
        IcmpHeader(135, 0, 0), bytes(4) + bytes(15) + b"\x01" + bytes([1, 1]) + bytes(6)))
    assert str(ns.target_addr) == "::1" and ns.options[0].option_type == 1 and ns.total_len() == 32
    with pytest.raises(views.ViewError, match="panics"):
        views.NeighborAdvertPacket.try_from(views.Icmpv6Packet(IcmpHeader(136, 0, 0), bytes(21)))


def test_dump_walks_every_frame(oracle):
    """No exception escapes the walk on any crafted / VLAN / mutated frame."""
    base = ([bytes.fromhex(v["frame"]) for v in helpers.golden()["frames"]] + helpers.crafted_frames() +
            helpers.vlan_frames() + helpers.slice_frames() + [oracle.gen_frame(abi.WL_IMIX, i) for i in range(100)])
    frames = base + helpers.mutate_frames(np.random.default_rng(8), base, 5000)
    recs = oracle.parse_frames(frames)
    lines = list(views.dump_records(recs, frames, "test"))
    assert sum(1 for ln in lines if ln.startswith("---- Interface: test")) == len(frames)


def test_ndp_option_and_create_vectors():
    """icmpv6.rs ndp_tests on the host: NdpOptionPacket::from_bytes
    (basic_option_parsing: trailing bytes ignored) and every *_create test's
    to_bytes image; the images decode back to the same fields; the
    reference's failure modes (short buffers, length-0 options)."""
    import ipaddress

    from nex_amd import views
    from nex_amd.frame import IcmpHeader
    g = helpers.golden()["ndp"]
    o = g["option"]
    opt = views.NdpOptionPacket.from_bytes(bytes.fromhex(o["bytes"]))
    assert (opt.option_type, opt.length, opt.payload.hex()) == (o["option_type"], o["length"], o["payload"])
    for c in g["create"]:
        t = helpers.NDP_KINDS[c["kind"]]
        cls = views.NDP_VIEWS[t]
        kw = {k: v for k, v in c.items() if k not in ("kind", "cite", "bytes")}
        kw["options"] = [views.NdpOptionPacket(a, b, bytes.fromhex(p)) for a, b, p in kw["options"]]
        for f in ("target_addr", "dest_addr"):
            if f in kw:
                kw[f] = ipaddress.IPv6Address(kw[f])
        m = cls(header=IcmpHeader(t, 0, 0), **kw)
        assert m.to_bytes().hex() == c["bytes"], c["cite"]
        back = cls.from_bytes(bytes.fromhex(c["bytes"])) if len(c["bytes"]) >= 48 else None
        if back is not None:
            helpers.ndp_fields_equal(back, c, c["cite"])
    with pytest.raises(views.ViewError):
        views.NdpOptionPacket.from_bytes(bytes([1]))
    with pytest.raises(views.ViewError):  # length 1 = 8 B, only 4 present
        views.NdpOptionPacket.from_bytes(bytes([1, 1, 0, 0]))
    with pytest.raises(views.ViewError):  # length 0: usize underflow in the reference
        views.NdpOptionPacket.from_bytes(bytes([1, 0]))
    with pytest.raises(views.ViewError):
        views.RouterSolicitPacket.from_bytes(bytes(23))
    with pytest.raises(views.ViewError):  # RS / RA slice [i+2..i] on a length-0 option: panic
        views.RouterSolicitPacket.from_bytes(bytes([133, 0, 0, 0, 0, 0, 0, 0]) + bytes([1, 0]) + bytes(14))
    ns = views.NeighborSolicitPacket.from_bytes(bytes([135]) + bytes(23) + bytes([1, 0, 9, 9]))
    assert ns.options == [] and ns.payload == bytes([1, 0, 9, 9])  # NS stops at a length-0 option
    ra = views.RouterAdvertPacket.from_bytes(bytes([134]) + bytes(15) + bytes([5, 1]) + bytes(6) + bytes([1, 2, 3]))
    assert [(x.option_type, x.length) for x in ra.options] == [(5, 1)] and ra.payload == bytes([1, 2, 3])
    assert ra.options_length() == 8 and ra.total_len() == 8 + 16 + 3
