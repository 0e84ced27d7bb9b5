"""The probe batches of the reference's three ping callers, as the GPU builds
them: one source host, a destination per frame, every other field the
example's constant.

* ``udp6``: udp_ping's IPv6 branch (examples/udp_ping.rs:29-31, 68-89):
  UdpPacketBuilder SRC_PORT 53443 -> DST_PORT 33435, no payload, inside
  Ipv6PacketBuilder (hop limit 64) and EthernetPacketBuilder: 62 B.
* ``tcp_ping``: examples/tcp_ping.rs:108-163: a SYN from port 53443, window
  64240, options MSS 1460, SACK permitted, NOP, NOP, window scale 7 (11 B,
  padded to 12), IPv4 DontFragment: 66 B (IPv6: 86 B).
* ``icmp_ping``: examples/icmp_ping.rs:67-102: echo request, identifier
  0x1234, sequence 1, payload "hello", IPv4 DontFragment: 47 B (IPv6,
  Icmpv6 echo request type 128: 67 B).

`build` runs a shape through the engine (nexg_build_{udp6,tcp,icmp_echo}_batch
with the source shared: the kernels' probe form, which reads only the
destination per frame); `oracle_args` is the same frames' parameters as plain
data, which the tests and bench.py's cpu_baseline hand to the oracle's
build_probe_batch (nothing here calls the oracle).
"""
SRC_MAC = b"\x02\0\0\0\0\x01"  # synthetic interface / gateway MACs
DST_MAC = b"\x02\0\0\0\0\x02"
SRC_V4 = bytes([192, 168, 1, 100])
SRC_V6 = bytes.fromhex("20010db8000000000000000000000064")
TCP_PING_OPTS = bytes.fromhex("020405b4" "0402" "01" "01" "030307")  # mss, sack_perm, nop, nop, wscale
TCP_PING_DPORT = 80  # the target socket's port (tcp_ping.rs takes it from the command line)
ICMP_PAYLOAD = b"hello"

#: name -> (family, kind, frame length)
SHAPES = {
    "udp6": (6, "udp6", 62),
    "tcp_ping": (4, "tcp", 66),
    "tcp_ping6": (6, "tcp", 86),
    "icmp_ping": (4, "icmp", 47),
    "icmp_ping6": (6, "icmp", 67),
}

NOTE = {
    "udp6": "udp_ping.rs IPv6 branch: UDP 53443 -> 33435, no payload, hop limit 64 (62 B)",
    "tcp_ping": "tcp_ping.rs SYN: port 53443 -> 80, window 64240, MSS/SACK-perm/NOP/NOP/WS options, IPv4 DF (66 B)",
    "tcp_ping6": "tcp_ping.rs SYN over IPv6 (86 B)",
    "icmp_ping": "icmp_ping.rs echo request: id 0x1234, seq 1, payload \"hello\", IPv4 DF (47 B)",
    "icmp_ping6": "icmp_ping.rs ICMPv6 echo request (67 B)",
}


def frame_len(shape):
    return SHAPES[shape][2]


def dst_bytes(shape):
    """Bytes of parameters read per frame by the probe form (the destination)."""
    return 4 if SHAPES[shape][0] == 4 else 16


def source(shape, device):
    import torch
    fam = SHAPES[shape][0]
    return torch.tensor(list(SRC_V4 if fam == 4 else SRC_V6), dtype=torch.uint8, device=device)


def build(eng, shape, dst, src=None, out=None, stream=None, payload_t=None):
    """Build the probe batch `shape` for the (count, 4|16) uint8 device tensor
    `dst` (src: the one source address, default the shape's)."""
    import torch
    fam, kind, _ = SHAPES[shape]
    src = source(shape, dst.device) if src is None else src
    if kind == "udp6":
        return eng.build_udp6(src, dst, def_src_port=53443, def_dst_port=33435, src_mac=SRC_MAC, dst_mac=DST_MAC,
                              hop_limit=64, out=out, stream=stream)
    if kind == "tcp":
        return eng.build_tcp(fam, src, dst, def_src_port=53443, def_dst_port=TCP_PING_DPORT, flags=0x02,
                             window=64240, options=TCP_PING_OPTS, src_mac=SRC_MAC, dst_mac=DST_MAC, ttl=64,
                             ip_flags=2 if fam == 4 else 0, out=out, stream=stream)
    if payload_t is None:
        payload_t = torch.tensor(list(ICMP_PAYLOAD), dtype=torch.uint8, device=dst.device)
    return eng.build_icmp_echo(fam, src, dst, def_identifier=0x1234, def_sequence=1, payload=payload_t,
                               src_mac=SRC_MAC, dst_mac=DST_MAC, ttl=64, ip_flags=2 if fam == 4 else 0, out=out,
                               stream=stream)


def oracle_args(shape):
    """(kind, spec kwargs for oracle.ip_spec without dst, l4 kwargs) of the
    same frames for oracle.build_probe_batch."""
    fam, kind, _ = SHAPES[shape]
    spec = dict(family=fam, src=SRC_V4 if fam == 4 else SRC_V6, src_mac=SRC_MAC, dst_mac=DST_MAC, ttl=64,
                ip_flags=2 if fam == 4 else 0)
    if kind == "udp6":
        return kind, spec, dict(sport=53443, dport=33435)
    if kind == "tcp":
        return kind, spec, dict(sport=53443, dport=TCP_PING_DPORT, flags=0x02, window=64240, urg=0,
                                options=TCP_PING_OPTS)
    return kind, spec, dict(icmp_type=8 if fam == 4 else 128, icmp_code=0, ident=0x1234, seqno=1,
                            payload=ICMP_PAYLOAD)
