"""Writes tests/golden/reference_vectors.json.

Every vector is an input and the outputs the REFERENCE's own tests assert for
it (shellrow/nex nex-packet unit tests, fuzz seed corpus, bench fixtures),
transcribed as data with the file:line it comes from. Nothing here is
computed: the oracle and the GPU engine are checked against these values.

Run: python tests/golden/make_golden.py
"""
import json
import os


def h(bs):
    return bytes(bs).hex()


def eth(payload, ethertype=0x0800, dst=bytes(6), src=bytes(6)):
    return bytes(dst) + bytes(src) + ethertype.to_bytes(2, "big") + bytes(payload)


V = []


def add(name, cite, frame, expect, flags=0, ip_offset=0, note="", slice_expect=None):
    v = {"name": name, "cite": cite, "frame": h(frame), "parse_flags": flags,
         "ip_offset": ip_offset, "expect": expect, "note": note}
    if slice_expect is not None:  # what FrameSlice::try_from_buf asserts for the same bytes
        v["slice_expect"] = slice_expect
    V.append(v)


# ---- util.rs:190-261 (checksum arithmetic) --------------------------------
UTIL = {
    "cite": "nex-packet/src/util.rs:190-261",
    "sum_be_words": [
        {"data": h(range(11)), "skipword": 1, "sum": 7190},
        {"data": h(range(11)), "skipword": 2, "sum": 6676},
        {"data": h(range(11)), "skipword": 99, "sum": 7705},
        {"data": h(range(11)), "skipword": 101, "sum": 7705},
        {"data": "", "skipword": 0, "sum": 0},
        {"data": "", "skipword": 10, "sum": 0},
        {"data": "01", "skipword": 1, "sum": 256},
        {"data": "0101", "skipword": 0, "sum": 0},
        {"data": "0101", "skipword": 1, "sum": 257},
        {"data": "040404", "skipword": 0, "sum": 1024},
        {"data": "040404", "skipword": 1, "sum": 1028},
        {"data": "040404", "skipword": 2, "sum": 2052},
        {"data": "040404", "skipword": 3, "sum": 2052},
    ],
    "joined_equals_contiguous": [
        {"data": "01", "extra": "020304", "contiguous": "01020304"},
        {"data": "0102", "extra": "03", "contiguous": "010203"},
    ],
    "checksum": [
        {"data": "ffffffff", "skipword": 2**64 - 1, "checksum": 0},
        {"data": "01", "skipword": 2**64 - 1, "checksum": 0xFEFF},
        {"data": "010203", "skipword": 2**64 - 1, "checksum": 0xFBFD},
    ],
}

# ---- icmpv6.rs:606-631 (ICMPv6 pseudo-header checksum KAT) ----------------
ICMPV6_ECHO = bytes([0x80, 0x00, 0xFF, 0xFF, 0x00, 0x00, 0x00, 0x01]) + bytes([
    0x20, 0x20, 0x75, 0x73, 0x74, 0x20, 0x61, 0x20, 0x66, 0x6c, 0x65, 0x73, 0x68, 0x20,
    0x77, 0x6f, 0x75, 0x6e, 0x64, 0x20, 0x20, 0x74, 0x69, 0x73, 0x20, 0x62, 0x75, 0x74,
    0x20, 0x61, 0x20, 0x73, 0x63, 0x72, 0x61, 0x74, 0x63, 0x68, 0x20, 0x20, 0x6b, 0x6e,
    0x69, 0x67, 0x68, 0x74, 0x73, 0x20, 0x6f, 0x66, 0x20, 0x6e, 0x69, 0x20, 0x20, 0x20])
LO6 = bytes(15) + b"\x01"


def ipv6_hdr(payload, nh, src=LO6, dst=LO6, plen=None, tc_flow=(0x60, 0, 0, 0), hop=64):
    plen = len(payload) if plen is None else plen
    return bytes(tc_flow) + plen.to_bytes(2, "big") + bytes([nh, hop]) + src + dst + bytes(payload)


ICMPV6 = {
    "cite": "nex-packet/src/icmpv6.rs:606-631",
    "packet": h(ICMPV6_ECHO), "src": h(LO6), "dst": h(LO6),
    "checksum": 0x1D2E, "checksum_type_0x81": 0x1C2E,
}
add("icmpv6_echo_request_lo", "icmpv6.rs:606-631 (wrapped in Eth/IPv6 ::1->::1)",
    eth(ipv6_hdr(ICMPV6_ECHO, 58), 0x86DD),
    {"layers": ["eth", "ip", "ipv6", "icmpv6"], "l4_type": 0x80, "l4_csum": 0xFFFF,
     "l4_csum_calc": 0x1D2E})
add("icmpv6_echo_reply_lo", "icmpv6.rs:626-630 (type changed to 0x81)",
    eth(ipv6_hdr(b"\x81" + ICMPV6_ECHO[1:], 58), 0x86DD),
    {"layers": ["eth", "ip", "ipv6", "icmpv6"], "l4_type": 0x81, "l4_csum_calc": 0x1C2E})

# ---- frame.rs:665-784 ----------------------------------------------------
add("unknown_ethertype_keeps_payload", "frame.rs:665-678",
    eth(b"\xde\xad\xbe\xef", 0x88B5),
    {"layers": ["eth"], "payload": "deadbeef"})
raw = bytearray(14 + 20 + 8 + 4)
raw[12:14] = b"\x08\x00"
raw[14:34] = bytes([0x45, 0, 0, 0x20, 0, 1, 0, 0, 64, 17, 0, 0, 192, 0, 2, 1, 198, 51, 100, 2])
raw[34:42] = bytes([0x04, 0xD2, 0x00, 0x35, 0x00, 0x0C, 0x00, 0x00])
raw[42:46] = bytes([1, 2, 3, 4])
add("ipv4_udp_frame", "frame.rs:680-734", raw,
    {"layers": ["eth", "ip", "ipv4", "transport", "udp"], "ip_version": 4, "dst_port": 53,
     "payload": "01020304"})
add("dummy_ethernet_ipv4", "frame.rs:736-745 (ParseOption from_ip_packet, offset 0)",
    bytes([0x45, 0x00, 0x00, 0x14, 0x00, 0x00, 0x00, 0x00, 64, 17, 0, 0, 127, 0, 0, 1, 127, 0, 0, 1]),
    {"layers": ["eth", "ip", "ipv4", "transport"], "ethertype": 0x0800}, flags=2,
    note="UDP over 0 bytes fails -> transport Some(None,None)")
add("frame_slice_ipv4_tcp", "frame.rs:747-762 (FrameSlice boundaries; same bytes via Frame)",
    bytes([0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 0x08, 0x00, 0x45, 0, 0, 44, 0, 0, 0, 0, 64, 6, 0,
           0, 192, 0, 2, 1, 198, 51, 100, 2, 0, 80, 0x04, 0xd2, 0, 0, 0, 0, 0, 0, 0, 0, 0x50,
           0x18, 0, 0, 0, 0, 0, 0]) + b"data",
    {"layers": ["eth", "ip", "ipv4", "transport", "tcp"], "l3_off": 14, "l4_off": 34,
     "payload": b"data".hex(), "ip_proto": 6},
    slice_expect={"cite": "frame.rs:747-762; tests/allocation_behavior.rs:36-49 (is_ok)",
                  "datalink": [0, 14], "network": [14, 34], "transport": [34, 54],
                  "payload": [54, 58], "ip_protocol": 6})
b = bytearray(14 + 40 + 8 + 8 + 3)
b[12:14] = (0x86DD).to_bytes(2, "big")
b[14] = 0x60
b[18:20] = (19).to_bytes(2, "big")
b[20] = 0
b[21] = 64
b[54] = 17
b[55] = 0
b[62:64] = (1234).to_bytes(2, "big")
b[64:66] = (53).to_bytes(2, "big")
b[66:68] = (11).to_bytes(2, "big")
b[70:] = b"dns"
add("frame_slice_ipv6_hbh_udp", "frame.rs:764-784 (Frame path: HBH -> no transport, Q10)", b,
    {"layers": ["eth", "ip", "ipv6"], "ip_nopt": 1, "payload": bytes(b[62:73]).hex()},
    note="FrameSlice reports network 48 B / UDP; Frame keeps raw next_header 0 (Q10) and "
         "exposes the bytes after the extension chain as payload",
    slice_expect={"cite": "frame.rs:764-784", "network_len": 48, "transport_len": 8,
                  "payload_bytes": b"dns".hex(), "ip_protocol": 17})

# ---- ethernet.rs:458-539, ipv6.rs:672-704, icmpv6.rs:2531-2549 (per-protocol
# tests; the asserted bytes as Frames, the asserted values as expectations) ---
add("ethernet_parse_basic", "ethernet.rs:458-476",
    bytes([0xaa, 0xbb, 0xcc, 0xdd, 0xee, 0xff, 0x11, 0x22, 0x33, 0x44, 0x55, 0x66, 0x08, 0x00,
           0xde, 0xad, 0xbe, 0xef]),
    {"layers": ["eth", "ip"], "ethertype": 0x0800, "eth_dst": "aabbccddeeff", "eth_src": "112233445566"},
    note="EtherType Ipv4 with a 4-B payload: IPv4 fails -> ip Some(all None), payload empty (Q4)")
add("ethernet_too_short", "ethernet.rs:510-528 (BufferTooShort, actual 4)", bytes([0, 1, 2, 3]),
    {"status": 1, "err_context": "Ethernet packet", "err_a": 14, "err_b": 4},
    note="ethernet.rs:513-520 asserts BufferTooShort{context 'Ethernet packet', minimum 14, actual 4}")
add("ethernet_unknown_ethertype_dead", "ethernet.rs:530-539 (EtherType::Unknown(0xdead))",
    bytes([0xaa, 0xbb, 0xcc, 0xdd, 0xee, 0xff, 0x11, 0x22, 0x33, 0x44, 0x55, 0x66, 0xde, 0xad,
           0x00, 0x11, 0x22, 0x33]),
    {"layers": ["eth"], "ethertype": 0xdead, "payload": "00112233"})
add("ipv6_basic_header_fields", "ipv6.rs:672-704 (tc 0xaa, flow 0x12345, Udp, hop 64, ::1 -> ::)",
    eth(ipv6_hdr(b"", 17, src=LO6, dst=bytes(16), tc_flow=(0x6a, 0xa1, 0x23, 0x45)), 0x86DD),
    {"layers": ["eth", "ip", "ipv6", "transport"], "ip_tos": 0xaa, "ip_word": 0x12345, "ip_length": 0,
     "ip_proto": 17, "ip_ttl": 64},
    note="UDP over 0 bytes fails -> transport Some(None,None)")
ECHO6 = bytes([0x80, 0x00, 0xbe, 0xef, 0x12, 0x34, 0x56, 0x78]) + b"ping!"
add("icmpv6_echo_request_parse", "icmpv6.rs:2531-2549 (type EchoRequest, code 0, checksum 0xbeef, "
    "id 0x1234, seq 0x5678, payload 'ping!')", eth(ipv6_hdr(ECHO6, 58), 0x86DD),
    {"layers": ["eth", "ip", "ipv6", "icmpv6"], "l4_type": 128, "l4_code": 0, "l4_csum": 0xbeef,
     "payload": (bytes([0x12, 0x34, 0x56, 0x78]) + b"ping!").hex(),
     "view": {"kind": "Icmpv6EchoRequest", "identifier": 0x1234, "sequence_number": 0x5678,
              "payload": b"ping!".hex()}},
    note="Frame.payload of ICMPv6 = bytes after the 4-B header (Q15): identifier, sequence, data")

# ---- ipv4.rs:944-1204 ------------------------------------------------------
IPV4_RT = bytes([0x45, 0x00, 0x00, 0x1c, 0x1c, 0x46, 0x40, 0x00, 0x40, 0x06, 0xb1, 0xe6,
                 0xc0, 0xa8, 0x00, 0x01, 0xc0, 0xa8, 0x00, 0xc7,
                 0xde, 0xad, 0xbe, 0xef, 0xca, 0xfe, 0xba, 0xbe])
add("ipv4_round_trip", "ipv4.rs:944-969 (from_ip_packet)", IPV4_RT,
    {"layers": ["eth", "ip", "ipv4", "transport"], "ip_ihl": 5, "ip_length": 28,
     "ip_src": "192.168.0.1", "ip_dst": "192.168.0.199", "ip_csum": 0xB1E6,
     "payload": "deadbeefcafebabe"},
    flags=2, note="TCP over 8 bytes fails -> transport Some(None,None), payload = IP payload")
IPV4_OPT = bytes([0x47, 0x00, 0x00, 0x20, 0x12, 0x34, 0x40, 0x00, 0x40, 0x11, 0x00, 0x00,
                  0xc0, 0xa8, 0x00, 0x01, 0xc0, 0xa8, 0x00, 0x02,
                  0x01, 0x87, 0x04, 0x12, 0x34, 0x00, 0x00, 0x00,
                  0xde, 0xad, 0xbe, 0xef])
add("ipv4_with_options", "ipv4.rs:971-1020 (from_ip_packet)", IPV4_OPT,
    {"layers": ["eth", "ip", "ipv4", "transport"], "ip_ihl": 7, "ip_length": 32, "ip_nopt": 3,
     "payload": "deadbeef"}, flags=2)
IPV4_CS = bytes([0x45, 0x00, 0x00, 0x14, 0x00, 0x00, 0x40, 0x00, 0x40, 0x06, 0x00, 0x00,
                 0x0a, 0x00, 0x00, 0x01, 0x0a, 0x00, 0x00, 0x02])
add("ipv4_checksum_zero_field", "ipv4.rs:1073-1095 (checksum(&p) then reparse)", IPV4_CS,
    {"layers": ["eth", "ip", "ipv4", "transport"], "ip_csum": 0, "ip_csum_consistent": True},
    flags=2, note="reference asserts checksum(p) round-trips; value pinned by the oracle")
STRICT = bytes([0x45, 0x00, 0x00, 0x28, 0x00, 0x00, 0x00, 0x00, 64, 17, 0, 0, 127, 0, 0, 1, 127,
                0, 0, 1, 1, 2, 3, 4])
add("ipv4_strict_truncation", "ipv4.rs:1176-1187 (strict -> Truncated)", STRICT,
    {"status": 4, "err_context": "IPv4 packet", "err_a": 40, "err_b": 24}, flags=3,
    note="the test asserts the kind; expected/actual follow ipv4.rs:429-435 (total 40, captured 24)")
STRICT6 = bytes([0x60, 0x00, 0x00, 0x00, 0x00, 0x10, 0x11, 0x40] + [0] * 15 + [1] + [0] * 15 + [1, 1, 2, 3, 4])
add("ipv6_strict_truncation", "ipv6.rs:915-928 (strict -> Truncated)", STRICT6,
    {"status": 4, "err_context": "IPv6 payload", "err_a": 56, "err_b": 44}, flags=3,
    note="the test asserts the kind; expected/actual follow ipv6.rs:270-276 (40 + 16 declared, 44 captured)")
add("ipv4_lenient_truncation", "ipv4.rs:1186 (lenient parse succeeds)", STRICT,
    {"layers": ["eth", "ip", "ipv4", "transport"], "ip_length": 24}, flags=2)
ZERO = bytes([0x45, 0x00, 0x00, 0x00, 0x68, 0x23, 0x40, 0x00, 0x80, 0x06, 0x00, 0x00, 192, 168,
              10, 113, 192, 168, 10, 10, 0xde, 0xad, 0xbe, 0xef])
add("ipv4_zero_total_length", "ipv4.rs:1189-1204 (TSO capture: total = captured)", ZERO,
    {"layers": ["eth", "ip", "ipv4", "transport"], "ip_length": 24, "payload": "deadbeef"},
    flags=2)

# ---- ipv6.rs:706-741, :797-802 ---------------------------------------------
IPV6_P = bytes([0x60, 0xA1, 0x23, 0x45, 0x00, 0x08, 0x06, 0x40,
                0xfe, 0x80, 0, 0, 0, 0, 0, 0, 0x02, 0x1a, 0x2b, 0xff, 0xfe, 0x1a, 0x2b, 0x3c,
                0xff, 0x02, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x02]) + b"Hello!!\n"
add("ipv6_from_bytes", "ipv6.rs:706-741 (from_ip_packet)", IPV6_P,
    {"layers": ["eth", "ip", "ipv6", "transport"], "ip_tos": 0x0A, "ip_word": 0x12345,
     "ip_length": 8, "ip_proto": 6, "ip_ttl": 0x40, "payload": b"Hello!!\n".hex()},
    flags=2, note="traffic_class 0xa, flow label 0x12345; TCP over 8 bytes fails")
add("ipv6_too_short", "ipv6.rs:797-802 (20 bytes rejected)", eth(bytes(20), 0x86DD),
    {"layers": ["eth", "ip"]})

# ---- L4 unit fixtures wrapped in IPv4 (tcp.rs, udp.rs, icmp.rs) ------------
def ipv4_hdr(payload, proto, src=(10, 0, 0, 1), dst=(10, 0, 0, 2), ident=0):
    tot = 20 + len(payload)
    return bytes([0x45, 0, tot >> 8, tot & 255, ident >> 8, ident & 255, 0x40, 0, 64, proto, 0, 0,
                  *src, *dst]) + bytes(payload)


# icmp.rs:728-815: EchoReply / DestinationUnreachable / TimeExceeded messages
# as the tests assemble them (checksum field left 0: the tests only assert the
# fields and payloads below), carried as IPv4 protocol 1 in a Frame
# "view": the sub-message the test downcasts to (icmp.rs:434-700) and the
# fields it asserts (echo reply: identifier, sequence, payload; unreachable:
# next_hop_mtu, payload; time exceeded: unused, payload)
for name, cite, msg, typ, code, pl, view in (
        ("icmp_echo_reply_roundtrip", "icmp.rs:728-757 (id 5678, seq 99, payload 'pong')",
         bytes([0, 0, 0, 0, 0x16, 0x2e, 0x00, 0x63]) + b"pong", 0, 0,
         bytes([0x16, 0x2e, 0x00, 0x63]) + b"pong",
         {"kind": "EchoReply", "identifier": 5678, "sequence_number": 99, "payload": b"pong".hex()}),
        ("icmp_destination_unreachable", "icmp.rs:759-787 (code 3, next_hop_mtu 1500, payload 'bad ip')",
         bytes([3, 3, 0, 0, 0, 0, 0x05, 0xdc]) + b"bad ip", 3, 3, bytes([0, 0, 0x05, 0xdc]) + b"bad ip",
         {"kind": "DestinationUnreachable", "next_hop_mtu": 1500, "payload": b"bad ip".hex()}),
        ("icmp_time_exceeded", "icmp.rs:789-815 (unused 0xdeadbeef, payload 'timeout')",
         bytes([11, 0, 0, 0, 0xde, 0xad, 0xbe, 0xef]) + b"timeout", 11, 0,
         bytes([0xde, 0xad, 0xbe, 0xef]) + b"timeout",
         {"kind": "TimeExceeded", "unused": 0xdeadbeef, "payload": b"timeout".hex()})):
    add(name, cite, eth(ipv4_hdr(msg, 1)),
        {"layers": ["eth", "ip", "ipv4", "icmp"], "l4_type": typ, "l4_code": code, "payload": pl.hex(),
         "view": view},
        note="Frame.payload of ICMP = bytes after the 4-B header (Q15)")


# icmpv6.rs ndp_tests (1908-2202). The parse tests decode a bare ICMPv6
# message with Packet::from_bytes (try_from_buf); here each message rides in
# Eth/IPv6 (next header 58) and "view" holds the message type, the fields the
# test asserts ("options": [type, length, payload hex] in order) and what the
# TryFrom<Icmpv6Packet> conversion dump.rs uses gives for the same message
# ("try_from": "same" or the reference's error string).
NDP_RS = bytes([0x85, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
                0x02, 0x01, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x01, 0x01, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00])
NDP_RA = bytes([0x86, 0x00, 0x00, 0x00, 0xff, 0x80, 0x09, 0x00, 0x12, 0x34, 0x56, 0x78, 0x87, 0x65, 0x43, 0x21,
                0x01, 0x01, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x05, 0x01, 0x00, 0x00, 0x57, 0x68, 0x61, 0x74])
NDP_NS = bytes([0x87, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0xff, 0x02] + [0] * 13 + [0x01])
NDP_NA = bytes([0x88, 0x00, 0x00, 0x00, 0x80, 0x00, 0x00, 0x00, 0xff, 0x02] + [0] * 13 + [0x01])
NDP_REDIRECT = bytes([0x89, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0xff, 0x02] + [0] * 13 + [0x01] + [0] * 16)
for name, cite, msg, view in (
        ("icmpv6_ndp_router_solicit", "icmpv6.rs:1922-1956 (basic_rs_parse)", NDP_RS,
         {"kind": "RouterSolicit", "l4_csum": 0, "reserved": 0,
          "options": [[2, 1, "000000000000"], [1, 1, "000000000000"]], "try_from": "same"}),
        ("icmpv6_ndp_router_advert", "icmpv6.rs:1991-2031 (basic_ra_parse)", NDP_RA,
         {"kind": "RouterAdvert", "l4_csum": 0, "hop_limit": 0xff, "flags": 0x80, "lifetime": 0x900,
          "reachable_time": 0x12345678, "retrans_time": 0x87654321,
          "options": [[1, 1, "000000000000"], [5, 1, "000057686174"]], "try_from": "same"}),
        ("icmpv6_ndp_neighbor_solicit", "icmpv6.rs:2071-2083 (basic_ns_parse)", NDP_NS,
         {"kind": "NeighborSolicit", "l4_csum": 0, "reserved": 0, "target_addr": "ff02::1", "options": [],
          "try_from": "Payload too short for Neighbor Solicitation"}),
        ("icmpv6_ndp_neighbor_advert", "icmpv6.rs:2113-2126 (basic_na_parse)", NDP_NA,
         {"kind": "NeighborAdvert", "l4_csum": 0, "reserved": 0, "flags": 0x80, "target_addr": "ff02::1",
          "options": [], "try_from": "same"}),
        ("icmpv6_ndp_redirect", "icmpv6.rs:2157-2171 (basic_redirect_parse)", NDP_REDIRECT,
         {"kind": "Redirect", "l4_csum": 0, "reserved": 0, "target_addr": "ff02::1", "dest_addr": "::",
          "options": [], "try_from": "Payload too short for Redirect"})):
    add(name, cite, eth(ipv6_hdr(msg, 58), 0x86DD),
        {"layers": ["eth", "ip", "ipv6", "icmpv6"], "l4_type": msg[0], "l4_code": 0, "view": view},
        note="NDP message decoded from the GPU record's ICMPv6 bytes (from_bytes) and Icmpv6Packet (TryFrom)")

# NdpOptionPacket::from_bytes (basic_option_parsing, icmpv6.rs:1908-1920) and
# the *_create tests' to_bytes images (icmpv6.rs:1958-1989, 2033-2069,
# 2085-2111, 2128-2155, 2173-2202)
NDP = {
    "option": {"cite": "icmpv6.rs:1908-1920", "bytes": "0201060504030201000000",
               "option_type": 2, "length": 1, "payload": "060504030201"},
    "create": [
        {"kind": "RouterSolicit", "cite": "icmpv6.rs:1958-1989", "reserved": 0,
         "options": [[1, 1, "000000000000"]], "bytes": "8500000000000000" "0101000000000000"},
        {"kind": "RouterAdvert", "cite": "icmpv6.rs:2033-2069", "hop_limit": 0xff, "flags": 0x80,
         "lifetime": 0, "reachable_time": 0, "retrans_time": 0, "options": [[5, 1, "000000000000"]],
         "bytes": "86000000ff800000" "0000000000000000" "0501000000000000"},
        {"kind": "NeighborSolicit", "cite": "icmpv6.rs:2085-2111", "reserved": 0, "target_addr": "ff02::1",
         "options": [], "bytes": "8700000000000000" "ff020000000000000000000000000001"},
        {"kind": "NeighborAdvert", "cite": "icmpv6.rs:2128-2155", "flags": 0x80, "reserved": 0,
         "target_addr": "ff02::1", "options": [], "bytes": "8800000080000000" "ff020000000000000000000000000001"},
        {"kind": "Redirect", "cite": "icmpv6.rs:2173-2202", "reserved": 0, "target_addr": "ff02::1",
         "dest_addr": "::", "options": [],
         "bytes": "8900000000000000" "ff020000000000000000000000000001" "00000000000000000000000000000000"},
    ],
}


TCP_P = bytes([0xc1, 0x67, 0x23, 0x28, 0x90, 0x37, 0xd2, 0xb8, 0x94, 0x4b, 0xb2, 0x76, 0x80, 0x18,
               0x0f, 0xaf, 0xc0, 0x31, 0x00, 0x00, 0x01, 0x01, 0x08, 0x0a, 0x2c, 0x57, 0xcd, 0xa5,
               0x02, 0xa0, 0x41, 0x92]) + b"test"
add("tcp_basic_parse", "tcp.rs:1276-1314 (wrapped in Eth/IPv4)", eth(ipv4_hdr(TCP_P, 6)),
    {"layers": ["eth", "ip", "ipv4", "transport", "tcp"], "src_port": 0xC167,
     "dst_port": 0x2328, "tcp_seq": 0x9037D2B8, "tcp_ack": 0x944BB276, "l4_length": 32,
     "l4_type": 0x18, "tcp_window": 0x0FAF, "l4_csum": 0xC031, "l4_nopt": 3,
     "payload": b"test".hex()})
UDP_P = bytes([0x12, 0x34, 0xab, 0xcd, 0x00, 0x0c, 0x55, 0xaa]) + b"data"
add("udp_basic_parse", "udp.rs:510-527 (wrapped in Eth/IPv4)", eth(ipv4_hdr(UDP_P, 17)),
    {"layers": ["eth", "ip", "ipv4", "transport", "udp"], "src_port": 0x1234,
     "dst_port": 0xABCD, "l4_length": 12, "l4_csum": 0x55AA, "payload": b"data".hex()})
ICMP_P = bytes([8, 0, 0x3a, 0xbc, 0x04, 0xd2, 0x00, 0x2a]) + b"ping"
add("icmp_echo_request", "icmp.rs:708-725 (wrapped in Eth/IPv4)", eth(ipv4_hdr(ICMP_P, 1)),
    {"layers": ["eth", "ip", "ipv4", "icmp"], "l4_type": 8, "l4_code": 0, "l4_csum": 0x3ABC,
     "payload": "04d2002a" + b"ping".hex(),
     "view": {"kind": "EchoRequest", "identifier": 1234, "sequence_number": 42, "payload": b"ping".hex()}})

# ---- bench fixtures (nex-packet/benches) -----------------------------------
BENCH_V4_TCP = bytes([0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 0x08, 0x00, 0x45, 0x00, 0x00, 0x30,
                      0x12, 0x34, 0x40, 0x00, 64, 0x06, 0, 0, 192, 0, 2, 1, 198, 51, 100, 2, 0x04,
                      0xd2, 0x00, 0x50, 0, 0, 0, 1, 0, 0, 0, 0, 0x50, 0x18, 0x20, 0x00, 0, 0, 0,
                      0]) + b"hello!!!"
add("bench_ipv4_tcp_frame", "benches/packet_parse.rs:9-16", BENCH_V4_TCP,
    {"layers": ["eth", "ip", "ipv4", "transport", "tcp"], "payload": b"hello!!!".hex()})
BENCH_V6_UDP = bytes([0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 0x86, 0xdd, 0x60, 0, 0, 0, 0, 16, 17,
                      64, 0xfe, 0x80, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0xfe, 0x80, 0, 0,
                      0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 0x04, 0xd2, 0x00, 0x35, 0x00, 0x10, 0,
                      0]) + b"dns!" + bytes([0, 1, 2, 3])
add("bench_ipv6_udp_frame", "benches/packet_parse.rs:18-24", BENCH_V6_UDP,
    {"layers": ["eth", "ip", "ipv6", "transport", "udp"], "dst_port": 53,
     "payload": (b"dns!" + bytes([0, 1, 2, 3])).hex()})
add("bench_ipv4_udp_packet", "benches/packet_operations.rs:18-21 (ipv4_checksum input)",
    bytes([0x45, 0, 0, 28, 0x12, 0x34, 0x40, 0, 64, 17, 0, 0, 192, 0, 2, 1, 198, 51, 100, 2,
           0x04, 0xd2, 0, 53, 0, 8, 0, 0]),
    {"layers": ["eth", "ip", "ipv4", "transport", "udp"], "payload": ""}, flags=2)

# ---- fuzz seed corpus (fuzz/corpus/*/*.hex) --------------------------------
add("fuzz_ethernet_vlan_ipv4_frame", "fuzz/corpus/ethernet_vlan/ipv4_frame.hex",
    bytes.fromhex("00112233445566778899aabb08004500001c1234400040110000c0000201c633640204d2003500080000"),
    {"layers": ["eth", "ip", "ipv4", "transport", "udp"], "dst_port": 53})
add("fuzz_ipv4_options", "fuzz/corpus/ipv4_options/options.hex",
    bytes.fromhex("470000201234400040110000c0a80001c0a800020187041234000000deadbeef"),
    {"layers": ["eth", "ip", "ipv4", "transport"], "ip_nopt": 3}, flags=2)
add("fuzz_ipv6_hop_by_hop", "fuzz/corpus/ipv6_extensions/hop_by_hop.hex",
    bytes.fromhex("6000000000100040fe800000000000000000000000000001fe800000000000000000000000000002"
                  "110000000000000004d2003500080000"),
    {"layers": ["eth", "ip", "ipv6"], "ip_nopt": 1}, flags=2)
add("fuzz_icmpv6_ndp_rs", "fuzz/corpus/icmpv6_ndp/router_solicitation.hex (in Eth/IPv6)",
    eth(ipv6_hdr(bytes.fromhex("85000000000000000101001122334455"), 58), 0x86DD),
    {"layers": ["eth", "ip", "ipv6", "icmpv6"], "l4_type": 0x85})

# ---- serialize path: udp_ping.rs:68-109 ------------------------------------
BUILD = [{
    "cite": "examples/udp_ping.rs:29-30,68-109; builder/udp.rs:116-130; builder/ipv4.rs:25-47",
    "src_ip": "192.168.1.100", "dst_ip": "1.1.1.1", "sport": 53443, "dport": 33435,
    "ip_flags": 2, "ttl": 64, "ip_id": 0, "udp_length": 8, "ip_total_length": 28,
    "frame_len": 42,
}]

# TCP / ICMP builders (row 8(f)3): what the reference's builder tests assert
BUILD_L4 = {
    "tcp_basic": {
        "cite": "builder/tcp.rs:175-196 (tcp_builder_basic)",
        "src_ip": "192.168.1.100", "dst_ip": "192.168.1.1", "sport": 1234, "dport": 80,
        "seq": 1, "ack": 2, "flags": 0x02, "window": 1024, "urg": 0, "payload": b"abc".hex(),
    },
    "tcp_oversized_options": {
        "cite": "builder/tcp.rs:211-228 (5 x TcpOptionPacket::timestamp(0, 0) -> LengthOverflow)",
        "options": (bytes([8, 10]) + bytes(8)).hex() * 5, "error": "LengthOverflow",
    },
    "tcp_ping_options": {
        "cite": "examples/tcp_ping.rs:111-123 (mss 1460, sack_perm, nop, nop, wscale 7); "
                "tcp.rs:377-407 option encoders, tcp.rs:521-565 to_bytes padding",
        "options": "020405b4" "0402" "01" "01" "030307", "window": 64240, "flags": 0x02,
        "sport": 53443, "data_offset": 8,
    },
    "icmp_too_large": {
        "cite": "builder/icmp.rs:104-117 (payload of 65535 B -> LengthOverflow)",
        "payload_len": 65535, "error": "LengthOverflow",
    },
    "icmp_ping": {
        "cite": "examples/icmp_ping.rs:67-80 (EchoRequest, code 0, echo_fields(0x1234, 0x1), 'hello')",
        "ident": 0x1234, "seq": 1, "payload": b"hello".hex(),
    },
}


def main():
    out = {"util": UTIL, "icmpv6": ICMPV6, "frames": V, "build": BUILD, "build_l4": BUILD_L4, "ndp": NDP,
           "source": "shellrow/nex reference tests (see each 'cite')"}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_vectors.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {len(V)} frame vectors to {path}")


if __name__ == "__main__":
    main()
