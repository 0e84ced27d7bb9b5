"""Host-side mirror of nex-packet's frame API (nex-packet/src/frame.rs).

`ParseOption`, `ParseMode` and `ParseError` keep the reference's names and
meaning (frame.rs:47-50, parse.rs:34-97). `Frame` is materialised from one
engine result (nexg_record, or nexg_desc + the frame bytes) and mirrors the
Option<> layering of frame::Frame (frame.rs:21-60): the device did the parse
and the checksums; this module only reads header fields out of the bytes at
the offsets the device reported.
"""
import enum
import ipaddress
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

from . import abi


class ParseMode(enum.Enum):
    """parse.rs:34-46"""
    Lenient = 0
    Strict = 1


@dataclass(frozen=True)
class ParseOption:
    """frame.rs:47-50 (+ unwrap_vlan: the NEXG_PARSE_VLAN extension, off by
    default; the reference's Frame never unwraps VLAN tags, Q3)"""
    from_ip_packet: bool = False
    offset: int = 0
    unwrap_vlan: bool = False

    def flags(self, mode: ParseMode = ParseMode.Lenient) -> int:
        f = abi.PARSE_FROM_IP if self.from_ip_packet else 0
        if self.unwrap_vlan:
            f |= abi.PARSE_VLAN
        if mode == ParseMode.Strict:
            f |= abi.PARSE_STRICT
        return f


class ParseError(Exception):
    """parse.rs:51-97. The record of a failed frame carries the error's payload
    (include/nexg.h NEXG_CTX_*): `context` is the reference's context string;
    BufferTooShort has minimum / actual, InvalidLength value, Truncated
    expected / actual."""
    kind = None
    fields = ()

    def __init__(self, msg="", context=None, a=0, b=0):
        super().__init__(msg)
        self.context = context
        names = {1: ("minimum", "actual"), 2: ("value",), 4: ("expected", "actual")}.get(self.kind, ())
        for n, v in zip(names, (a, b)):
            setattr(self, n, v)
        self.fields = names


class BufferTooShort(ParseError):
    kind = abi.ERR_BUFFER_TOO_SHORT


class InvalidLength(ParseError):
    kind = abi.ERR_INVALID_LENGTH


class Malformed(ParseError):
    kind = abi.ERR_MALFORMED


class Truncated(ParseError):
    kind = abi.ERR_TRUNCATED


class BadExtent(ParseError):
    kind = abi.ERR_BAD_EXTENT


_ERRORS = {c.kind: c for c in (BufferTooShort, InvalidLength, Malformed, Truncated, BadExtent)}


def parse_error(kind: int, rec=None) -> ParseError:
    """The ParseError of a failed frame; with its record, the payload too."""
    cls = _ERRORS.get(kind, ParseError)
    if rec is None or kind == abi.ERR_BAD_EXTENT:
        return cls(f"ParseError kind {kind}")
    ctx = abi.ERR_CONTEXTS[int(rec["l4_type"])] if int(rec["l4_type"]) < len(abi.ERR_CONTEXTS) else None
    e = cls(f"{cls.__name__} {{ context: {ctx!r} }}", ctx, int(rec["ip_src"]), int(rec["ip_dst"]))
    if e.fields:
        e.args = (f"{cls.__name__} {{ context: {ctx!r}, " +
                  ", ".join(f"{n}: {getattr(e, n)}" for n in e.fields) + " }",)
    return e


# ---- headers (field names follow the reference structs) ------------------

@dataclass
class EthernetHeader:  # ethernet.rs:152-160
    destination: bytes
    source: bytes
    ethertype: int


@dataclass
class ArpHeader:  # arp.rs:300-311
    hardware_type: int
    protocol_type: int
    hw_addr_len: int
    proto_addr_len: int
    operation: int
    sender_hw_addr: bytes
    sender_proto_addr: ipaddress.IPv4Address
    target_hw_addr: bytes
    target_proto_addr: ipaddress.IPv4Address


@dataclass
class Ipv4Header:  # ipv4.rs:187-202
    version: int
    header_length: int
    dscp: int
    ecn: int
    total_length: int
    identification: int
    flags: int
    fragment_offset: int
    ttl: int
    next_level_protocol: int  # IpNextProtocol::value()
    checksum: int
    source: ipaddress.IPv4Address
    destination: ipaddress.IPv4Address
    options: List[Tuple[int, int, int, Optional[int], bytes]] = field(default_factory=list)


@dataclass
class Ipv6Header:  # ipv6.rs:14-23
    version: int
    traffic_class: int
    flow_label: int
    payload_length: int
    next_header: int
    hop_limit: int
    source: ipaddress.IPv6Address
    destination: ipaddress.IPv6Address


@dataclass
class IcmpHeader:  # icmp.rs:172-176 / icmpv6.rs:229-234
    icmp_type: int
    icmp_code: int
    checksum: int


@dataclass
class TcpHeader:  # tcp.rs:482-494
    source: int
    destination: int
    sequence: int
    acknowledgement: int
    data_offset: int
    reserved: int
    flags: int
    window: int
    checksum: int
    urgent_ptr: int
    options: List[Tuple[int, Optional[int], bytes]] = field(default_factory=list)


@dataclass
class UdpHeader:  # udp.rs:22-27
    source: int
    destination: int
    length: int
    checksum: int


@dataclass
class DatalinkLayer:
    ethernet: Optional[EthernetHeader]
    arp: Optional[ArpHeader]


@dataclass
class IpLayer:
    ipv4: Optional[Ipv4Header]
    ipv6: Optional[Ipv6Header]
    icmp: Optional[IcmpHeader]
    icmpv6: Optional[IcmpHeader]


@dataclass
class TransportLayer:
    tcp: Optional[TcpHeader]
    udp: Optional[UdpHeader]


@dataclass
class Checksums:
    """Verification results the engine adds to the Frame path."""
    ip_checked: bool
    ip_ok: bool
    ip_panic: bool
    l4_checked: bool
    l4_ok: bool
    ip_computed: int
    l4_computed: int


@dataclass
class Frame:  # frame.rs:54-60
    datalink: Optional[DatalinkLayer]
    ip: Optional[IpLayer]
    transport: Optional[TransportLayer]
    payload: bytes
    packet_len: int
    checksums: Optional[Checksums] = None


def _be16(b, i):
    return (b[i] << 8) | b[i + 1]


def _ipv4_options(b, l3, ihl):
    """ipv4.rs:442-508 option list (lenient walk) for display."""
    out, i, hl = [], 20, ihl * 4
    while i < hl:
        t = b[l3 + i]
        num = t & 0x1F
        if num in (0, 1):
            out.append(((t >> 7) & 1, (t >> 5) & 3, num, None, b""))
            if num == 0:
                break
            i += 1
            continue
        if i + 2 > hl:
            break
        ln = b[l3 + i + 1]
        if ln < 2 or i + ln > hl:
            break
        out.append(((t >> 7) & 1, (t >> 5) & 3, num, ln, bytes(b[l3 + i + 2:l3 + i + ln])))
        i += ln
    return out


def _tcp_options(b, base, hl):
    """tcp.rs:767-818 option list."""
    out, off = [], 20
    while off < hl:
        kind = b[base + off]
        off += 1
        if kind in (0, 1):
            out.append((kind, None, b""))
            if kind == 0:
                break
            continue
        ln = b[base + off]
        off += 1
        out.append((kind, ln, bytes(b[base + off:base + off + ln - 2])))
        off += ln - 2
    return out


def ipv4_options_at(b, opt_off: int, positions) -> List[Tuple[int, int, int, Optional[int], bytes]]:
    """Ipv4Header.options from nexg_options positions (the device's walk)."""
    out = []
    for p in positions:
        t = b[opt_off + int(p)]
        num = t & 0x1F
        if num in (0, 1):
            out.append(((t >> 7) & 1, (t >> 5) & 3, num, None, b""))
        else:
            ln = b[opt_off + int(p) + 1]
            out.append(((t >> 7) & 1, (t >> 5) & 3, num, ln, bytes(b[opt_off + int(p) + 2:opt_off + int(p) + ln])))
    return out


def tcp_options_at(b, opt_off: int, positions) -> List[Tuple[int, Optional[int], bytes]]:
    """TcpHeader.options from nexg_options positions (the device's walk)."""
    out = []
    for p in positions:
        kind = b[opt_off + int(p)]
        if kind in (0, 1):
            out.append((kind, None, b""))
        else:
            ln = b[opt_off + int(p) + 1]
            out.append((kind, ln, bytes(b[opt_off + int(p) + 2:opt_off + int(p) + ln])))
    return out


def frame_from_record(rec, frame: bytes, options=None) -> Frame:
    """Materialise frame::Frame from a nexg_record and the frame bytes.

    `options` (a nexg_options from Engine.decode_options) supplies the option
    lists as the device decoded them; without it they are walked here.
    Raises the ParseError subclass the reference would return."""
    flags = int(rec["flags"])
    st = (flags >> abi.STATUS_SHIFT) & 7
    if st:
        raise parse_error(st, rec)
    b = frame
    l3 = int(rec["l3_off"])
    eth = None
    if flags & abi.L_ETHERNET:
        if (flags & abi.L_VLAN) or (l3 == 14 and int(rec["ethertype"]) == _be16(b, 12)):
            eth = EthernetHeader(bytes(b[0:6]), bytes(b[6:12]), int(rec["ethertype"]))
        else:  # from_ip_packet: dummy Ethernet (frame.rs:396-400)
            eth = EthernetHeader(b"\0" * 6, b"\0" * 6, int(rec["ethertype"]))
    arp = None
    if flags & abi.L_ARP:
        arp = ArpHeader(_be16(b, l3), _be16(b, l3 + 2), b[l3 + 4], b[l3 + 5], _be16(b, l3 + 6),
                        bytes(b[l3 + 8:l3 + 14]), ipaddress.IPv4Address(bytes(b[l3 + 14:l3 + 18])),
                        bytes(b[l3 + 18:l3 + 24]), ipaddress.IPv4Address(bytes(b[l3 + 24:l3 + 28])))
    datalink = DatalinkLayer(eth, arp) if flags & abi.L_ETHERNET else None
    ip = None
    if flags & abi.L_IP:
        v4 = v6 = icmp = icmpv6 = None
        if flags & abi.L_IPV4:
            w = int(rec["ip_word"])
            ihl = int(rec["ip_ver_ihl"]) & 15
            v4 = Ipv4Header(4, ihl, int(rec["ip_tos"]) >> 2, int(rec["ip_tos"]) & 3,
                            int(rec["ip_length"]), w >> 16, (w >> 13) & 7, w & 0x1FFF,
                            int(rec["ip_ttl"]), int(rec["ip_proto"]), int(rec["ip_csum"]),
                            ipaddress.IPv4Address(int(rec["ip_src"])),
                            ipaddress.IPv4Address(int(rec["ip_dst"])),
                            _ipv4_options(b, l3, ihl) if options is None else
                            ipv4_options_at(b, int(options["ip_opt_off"]),
                                            options["ip_pos"][:int(options["n_ip"])]))
        if flags & abi.L_IPV6:
            v6 = Ipv6Header(6, int(rec["ip_tos"]), int(rec["ip_word"]), int(rec["ip_length"]),
                            int(rec["ip_proto"]), int(rec["ip_ttl"]),
                            ipaddress.IPv6Address(bytes(b[l3 + 8:l3 + 24])),
                            ipaddress.IPv6Address(bytes(b[l3 + 24:l3 + 40])))
        ic = IcmpHeader(int(rec["l4_type"]), int(rec["l4_code"]), int(rec["l4_csum"]))
        if flags & abi.L_ICMP:
            icmp = ic
        if flags & abi.L_ICMPV6:
            icmpv6 = ic
        ip = IpLayer(v4, v6, icmp, icmpv6)
    transport = None
    if flags & abi.L_TRANSPORT:
        tcp = udp = None
        l4 = int(rec["l4_off"])
        if flags & abi.L_TCP:
            oc = int(rec["l4_code"])
            tcp = TcpHeader(int(rec["src_port"]), int(rec["dst_port"]), int(rec["tcp_seq"]),
                            int(rec["tcp_ack"]), oc >> 4, oc & 15, int(rec["l4_type"]),
                            int(rec["tcp_window"]), int(rec["l4_csum"]), int(rec["tcp_urg"]),
                            _tcp_options(b, l4, int(rec["l4_length"])) if options is None else
                            tcp_options_at(b, int(options["tcp_opt_off"]),
                                           options["tcp_pos"][:int(options["n_tcp"])]))
        if flags & abi.L_UDP:
            udp = UdpHeader(int(rec["src_port"]), int(rec["dst_port"]), int(rec["l4_length"]),
                            int(rec["l4_csum"]))
        transport = TransportLayer(tcp, udp)
    po, pl = int(rec["payload_off"]), int(rec["payload_len"])
    cs = Checksums(bool(flags & abi.C_IP_CHECKED), bool(flags & abi.C_IP_OK),
                   bool(flags & abi.C_IP_PANIC), bool(flags & abi.C_L4_CHECKED),
                   bool(flags & abi.C_L4_OK), int(rec["ip_csum_calc"]), int(rec["l4_csum_calc"]))
    return Frame(datalink, ip, transport, bytes(b[po:po + pl]), int(rec["packet_len"]), cs)


def frame_view_payload(frame: bytes, payload_len: int, option: ParseOption = ParseOption()) -> bytes:
    """FrameView payload quirk (frame.rs:609-622): the LAST payload_len bytes
    after the link header, not the Frame.payload slice."""
    start = option.offset if option.from_ip_packet else 14
    avail = frame[start:] if start <= len(frame) else b""
    if payload_len > len(avail):
        return b""
    return bytes(avail[len(avail) - payload_len:])


@dataclass
class FrameView:  # frame.rs:345-379
    """Frame's decoded layers with the payload borrowed from the input (Q27)."""
    datalink: Optional[DatalinkLayer]
    ip: Optional[IpLayer]
    transport: Optional[TransportLayer]
    payload: bytes
    packet_len: int


def frame_view_from_record(rec, frame: bytes, option: ParseOption = ParseOption()) -> FrameView:
    """FrameView::try_from_buf (frame.rs:360-372) from a NEXG_OUT_RECORD record."""
    f = frame_from_record(rec, frame)
    return FrameView(f.datalink, f.ip, f.transport,
                     frame_view_payload(frame, int(rec["payload_len"]), option), f.packet_len)


@dataclass
class FrameSlice:  # frame.rs:62-83
    """Borrowed layer boundaries (as memoryviews of the input)."""
    packet: memoryview
    datalink: Optional[memoryview]
    network: Optional[memoryview]
    transport: Optional[memoryview]
    payload: memoryview
    ethertype: Optional[int]
    ip_protocol: Optional[int]


def frame_slice_from_record(s, frame) -> FrameSlice:
    """FrameSlice::try_from_buf (frame.rs:84-136) from a NEXG_OUT_SLICE entry;
    raises the ParseError kind the reference returns."""
    flags = int(s["flags"])
    status = (flags >> abi.STATUS_SHIFT) & 7
    if status:
        raise parse_error(status)
    mv = memoryview(bytes(frame))
    l3, l3n, l4n = int(s["l3_off"]), int(s["l3_len"]), int(s["l4_len"])
    po, pn = int(s["payload_off"]), int(s["payload_len"])
    return FrameSlice(
        packet=mv,
        datalink=mv[:14] if flags & abi.S_DATALINK else None,
        network=mv[l3:l3 + l3n] if flags & abi.S_NETWORK else None,
        transport=mv[l3 + l3n:l3 + l3n + l4n] if flags & abi.S_TRANSPORT else None,
        payload=mv[po:po + pn],
        ethertype=int(s["ethertype"]) if flags & abi.S_ETHERTYPE else None,
        ip_protocol=(flags >> abi.S_PROTO_SHIFT) & 0xFF if flags & abi.S_IP_PROTOCOL else None,
    )
