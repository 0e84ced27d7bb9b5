"""Typed per-layer views over engine results: the per-protocol packet API
`examples/dump.rs` walks layer by layer (dump.rs:96-350) and the ICMP /
ICMPv6 sub-message conversions it downcasts to (icmp.rs:434-700;
icmpv6.rs echo_request / echo_reply / ndp).

The GPU parse (NEXG_OUT_RECORD) locates every layer; these views read the
fields out of the frame bytes at those offsets, with the reference's
validation rules and error strings, so the dump counterpart (`dump_lines`)
prints what dump.rs prints for the same frames.
"""
import ipaddress
from dataclasses import dataclass, field
from typing import List, Optional, Union

from . import abi
from .frame import IcmpHeader, _be16
from .parse_frame import _mac, ethertype_debug, ipproto_debug, ipv6_display

ICMP_TYPE_NAMES = {0: "EchoReply", 3: "DestinationUnreachable", 4: "SourceQuench", 5: "RedirectMessage",
                   8: "EchoRequest", 9: "RouterAdvertisement", 10: "RouterSolicitation", 11: "TimeExceeded",
                   12: "ParameterProblem", 13: "TimestampRequest", 14: "TimestampReply",
                   15: "InformationRequest", 16: "InformationReply", 17: "AddressMaskRequest",
                   18: "AddressMaskReply", 30: "Traceroute", 31: "DatagramConversionError",
                   32: "MobileHostRedirect", 33: "IPv6WhereAreYou", 34: "IPv6IAmHere",
                   35: "MobileRegistrationRequest", 36: "MobileRegistrationReply", 37: "DomainNameRequest",
                   38: "DomainNameReply", 39: "SKIP", 40: "Photuris"}  # icmp.rs:59-89
ICMPV6_TYPE_NAMES = {1: "DestinationUnreachable", 2: "PacketTooBig", 3: "TimeExceeded", 4: "ParameterProblem",
                     128: "EchoRequest", 129: "EchoReply", 130: "MulticastListenerQuery",
                     131: "MulticastListenerReport", 132: "MulticastListenerDone", 133: "RouterSolicitation",
                     134: "RouterAdvertisement", 135: "NeighborSolicitation", 136: "NeighborAdvertisement",
                     137: "RedirectMessage", 138: "RouterRenumbering", 139: "NodeInformationQuery",
                     140: "NodeInformationResponse", 141: "InverseNeighborDiscoverySolicitation",
                     142: "InverseNeighborDiscoveryAdvertisement", 143: "Version2MulticastListenerReport",
                     144: "HomeAgentAddressDiscoveryRequest", 145: "HomeAgentAddressDiscoveryReply",
                     146: "MobilePrefixSolicitation", 147: "MobilePrefixAdvertisement",
                     148: "CertificationPathSolicitationMessage", 149: "CertificationPathAdvertisementMessage",
                     150: "ExperimentalMobilityProtocols", 151: "MulticastRouterAdvertisement",
                     152: "MulticastRouterSolicitation", 153: "MulticastRouterTermination",
                     154: "FMIPv6Messages", 155: "RPLControlMessage", 156: "ILNPv6LocatorUpdateMessage",
                     157: "DuplicateAddressRequest", 158: "DuplicateAddressConfirmation",
                     159: "MPLControlMessage", 160: "ExtendedEchoRequest", 161: "ExtendedEchoReply"}  # icmpv6.rs:74-116
ARP_OP_NAMES = {1: "Request", 2: "Reply"}


def icmp_type_debug(t: int) -> str:
    return ICMP_TYPE_NAMES.get(t, f"Unknown({t})")


def icmpv6_type_debug(t: int) -> str:
    return ICMPV6_TYPE_NAMES.get(t, f"Unknown({t})")


class ViewError(ValueError):
    """A TryFrom conversion failed; the message is the reference's error string."""


# ---- ICMP (icmp.rs) --------------------------------------------------------

@dataclass
class IcmpPacket:  # icmp.rs:178-248
    header: IcmpHeader
    payload: bytes

    @classmethod
    def try_from_bytes(cls, b: bytes) -> "IcmpPacket":
        """icmp.rs:188-214: >= 8 B (ICMPV4_HEADER_LEN), payload = bytes[4..]."""
        if len(b) < 8:
            raise ViewError("Malformed")
        return cls(IcmpHeader(b[0], b[1], _be16(b, 2)), bytes(b[4:]))

    def total_len(self) -> int:  # icmp.rs:241-243
        return 4 + len(self.payload)


@dataclass
class EchoRequestPacket:  # icmp.rs:478-504
    header: IcmpHeader
    identifier: int
    sequence_number: int
    payload: bytes

    @classmethod
    def try_from(cls, pkt: IcmpPacket) -> "EchoRequestPacket":
        if pkt.header.icmp_type != 8:
            raise ViewError("Not an Echo Request")
        if len(pkt.payload) < 4:
            raise ViewError("Payload too short for Echo Request")
        return cls(pkt.header, _be16(pkt.payload, 0), _be16(pkt.payload, 2), pkt.payload[4:])


@dataclass
class EchoReplyPacket:  # icmp.rs:547-573
    header: IcmpHeader
    identifier: int
    sequence_number: int
    payload: bytes

    @classmethod
    def try_from(cls, pkt: IcmpPacket) -> "EchoReplyPacket":
        if pkt.header.icmp_type != 0:
            raise ViewError("Not an Echo Reply")
        if len(pkt.payload) < 4:
            raise ViewError("Payload too short for Echo Reply")
        return cls(pkt.header, _be16(pkt.payload, 0), _be16(pkt.payload, 2), pkt.payload[4:])


@dataclass
class DestinationUnreachablePacket:  # icmp.rs:618-647
    header: IcmpHeader
    unused: int
    next_hop_mtu: int
    payload: bytes

    @classmethod
    def try_from(cls, pkt: IcmpPacket) -> "DestinationUnreachablePacket":
        if pkt.header.icmp_type != 3:
            raise ViewError("Not a Destination Unreachable")
        if len(pkt.payload) < 4:
            raise ViewError("Payload too short for Destination Unreachable")
        return cls(pkt.header, _be16(pkt.payload, 0), _be16(pkt.payload, 2), pkt.payload[4:])


@dataclass
class TimeExceededPacket:  # icmp.rs:664-699
    header: IcmpHeader
    unused: int
    payload: bytes

    @classmethod
    def try_from(cls, pkt: IcmpPacket) -> "TimeExceededPacket":
        if pkt.header.icmp_type != 11:
            raise ViewError("Not a Time Exceeded")
        if len(pkt.payload) < 4:
            raise ViewError("Payload too short for Time Exceeded")
        return cls(pkt.header, int.from_bytes(pkt.payload[:4], "big"), pkt.payload[4:])


# ---- ICMPv6 (icmpv6.rs) ----------------------------------------------------

@dataclass
class Icmpv6Packet:  # icmpv6.rs:236-300
    header: IcmpHeader
    payload: bytes

    @classmethod
    def try_from_bytes(cls, b: bytes) -> "Icmpv6Packet":
        """icmpv6.rs:248-272: >= 8 B (ICMPV6_HEADER_LEN), payload = bytes[4..]."""
        if len(b) < 8:
            raise ViewError("Malformed")
        return cls(IcmpHeader(b[0], b[1], _be16(b, 2)), bytes(b[4:]))

    def total_len(self) -> int:
        return 4 + len(self.payload)


@dataclass
class Icmpv6EchoPacket:  # icmpv6.rs:2268-2294 (echo_request) / 2427-2453 (echo_reply)
    header: IcmpHeader
    identifier: int
    sequence_number: int
    payload: bytes

    @classmethod
    def try_from(cls, pkt: Icmpv6Packet, reply: bool = False) -> "Icmpv6EchoPacket":
        kind = "Echo Reply" if reply else "Echo Request"
        if pkt.header.icmp_type != (129 if reply else 128):
            raise ViewError(f"Not an {kind} packet")
        if len(pkt.payload) < 8:  # the v6 conversions ask for 8 B (the v4 ones for 4)
            raise ViewError(f"Payload too short for {kind}")
        return cls(pkt.header, _be16(pkt.payload, 0), _be16(pkt.payload, 2), pkt.payload[4:])

    def total_len(self) -> int:  # header 8 B (type, code, checksum, id, seq) + data
        return 8 + len(self.payload)


@dataclass
class NdpOptionPacket:  # icmpv6.rs:776-857
    option_type: int
    length: int  # unit: 8 bytes
    payload: bytes

    @classmethod
    def from_bytes(cls, b: bytes) -> "NdpOptionPacket":
        """Packet::try_from_buf (icmpv6.rs:784-810): >= 2 B, length * 8 B
        present, payload = bytes[2 .. length * 8] (trailing bytes ignored)."""
        if len(b) < 2:
            raise ViewError("Malformed")
        total = b[1] * 8
        if len(b) < total:
            raise ViewError("Malformed")
        if total < 2:  # total_len - 2 underflows in the reference (usize)
            raise ViewError("NDP option of length 0: the reference panics (usize underflow)")
        return cls(b[0], b[1], bytes(b[2:total]))

    def to_bytes(self) -> bytes:  # icmpv6.rs:817-823
        return bytes([self.option_type, self.length]) + self.payload

    def option_payload_length(self) -> int:  # icmpv6.rs:852-856, as written (payload.len() * 8 - 2)
        n = len(self.payload)
        return n * 8 - 2 if n > 0 else 0


def _ndp_options(b: bytes) -> List[NdpOptionPacket]:
    """The TryFrom<Icmpv6Packet> option split (e.g. icmpv6.rs:1295-1307 /
    1510-1522): the bytes after the fixed part in 8-B chunks (the last one
    possibly shorter), type = chunk[0], length = chunk[1] (a 1-byte trailing
    chunk makes the reference index out of range)."""
    out = []
    for k in range(0, len(b), 8):
        c = b[k:k + 8]
        if len(c) < 2:
            raise ViewError("NDP option chunk of 1 byte: the reference panics (chunk[1])")
        out.append(NdpOptionPacket(c[0], c[1], bytes(c[2:])))
    return out


def _ndp_options_buf(b: bytes, i: int, skip_short: bool):
    """The Packet::try_from_buf option walk from byte i (e.g. icmpv6.rs:
    937-957): while two bytes remain, an option of length * 8 bytes that fits
    is taken, else the walk stops; the rest is the payload. NS / NA /
    Redirect also stop at a length-0 option (skip_short, icmpv6.rs:1347);
    RS / RA slice bytes[i+2 .. i] there, which panics."""
    opts = []
    while i + 2 <= len(b):
        ol = b[i + 1] * 8
        if skip_short and ol < 2:
            break
        if i + ol > len(b):
            break
        if ol < 2:
            raise ViewError("NDP option of length 0: the reference panics (slice i+2..i)")
        opts.append(NdpOptionPacket(b[i], b[i + 1], bytes(b[i + 2:i + ol])))
        i += ol
    return opts, bytes(b[i:])


def _opts_bytes(opts: List[NdpOptionPacket]) -> bytes:
    return b"".join(o.to_bytes() for o in opts)


def _hdr_bytes(h: IcmpHeader) -> bytes:
    return bytes([h.icmp_type, h.icmp_code]) + h.checksum.to_bytes(2, "big")


def _hdr(b: bytes) -> IcmpHeader:
    return IcmpHeader(b[0], b[1], _be16(b, 2))


@dataclass
class RouterSolicitPacket:  # icmpv6.rs:872-1023
    header: IcmpHeader
    reserved: int
    options: List[NdpOptionPacket] = field(default_factory=list)
    payload: bytes = b""

    @classmethod
    def try_from(cls, pkt: Icmpv6Packet) -> "RouterSolicitPacket":  # icmpv6.rs:879-917
        if pkt.header.icmp_type != 133:
            raise ViewError("Not a Router Solicitation packet")
        if len(pkt.payload) < 8:
            raise ViewError("Payload too short for Router Solicitation")
        p = pkt.payload
        return cls(pkt.header, int.from_bytes(p[:4], "big"), _ndp_options(p[4:]))

    @classmethod
    def from_bytes(cls, b: bytes) -> "RouterSolicitPacket":  # icmpv6.rs:921-969: >= 24 B (NDP_SOL_PACKET_LEN)
        if len(b) < 24:
            raise ViewError("Malformed")
        opts, rest = _ndp_options_buf(b, 8, False)
        return cls(_hdr(b), int.from_bytes(b[4:8], "big"), opts, rest)

    def to_bytes(self) -> bytes:  # icmpv6.rs:976-988
        return _hdr_bytes(self.header) + self.reserved.to_bytes(4, "big") + _opts_bytes(self.options)

    def total_len(self) -> int:  # ICMPV6_HEADER_LEN + 4 + payload, icmpv6.rs:998-1008
        return 8 + 4 + len(self.payload)

    def options_length(self) -> int:  # icmpv6.rs:1016-1022
        n = len(self.to_bytes())
        return n - 8 if n > 8 else 0


@dataclass
class RouterAdvertPacket:  # icmpv6.rs:1055-1234
    header: IcmpHeader
    hop_limit: int
    flags: int
    lifetime: int
    reachable_time: int
    retrans_time: int
    options: List[NdpOptionPacket] = field(default_factory=list)
    payload: bytes = b""

    @classmethod
    def try_from(cls, pkt: Icmpv6Packet) -> "RouterAdvertPacket":  # icmpv6.rs:1066-1117
        if pkt.header.icmp_type != 134:
            raise ViewError("Not a Router Advertisement packet")
        if len(pkt.payload) < 16:
            raise ViewError("Payload too short for Router Advertisement")
        p = pkt.payload
        return cls(pkt.header, p[0], p[1], _be16(p, 2), int.from_bytes(p[4:8], "big"),
                   int.from_bytes(p[8:12], "big"), _ndp_options(p[12:]))

    @classmethod
    def from_bytes(cls, b: bytes) -> "RouterAdvertPacket":  # icmpv6.rs:1120-1177: >= 24 B (NDP_ADV_PACKET_LEN)
        if len(b) < 24:
            raise ViewError("Malformed")
        opts, rest = _ndp_options_buf(b, 16, False)
        return cls(_hdr(b), b[4], b[5], _be16(b, 6), int.from_bytes(b[8:12], "big"),
                   int.from_bytes(b[12:16], "big"), opts, rest)

    def to_bytes(self) -> bytes:  # icmpv6.rs:1185-1201
        return (_hdr_bytes(self.header) + bytes([self.hop_limit, self.flags]) + self.lifetime.to_bytes(2, "big") +
                self.reachable_time.to_bytes(4, "big") + self.retrans_time.to_bytes(4, "big") +
                _opts_bytes(self.options))

    def total_len(self) -> int:  # ICMPV6_HEADER_LEN + 16 + payload, icmpv6.rs:1209-1219
        return 8 + 16 + len(self.payload)

    def options_length(self) -> int:  # icmpv6.rs:1227-1233
        n = len(self.to_bytes())
        return n - 16 if n > 16 else 0


@dataclass
class NeighborSolicitPacket:  # icmpv6.rs:1258-1434
    header: IcmpHeader
    reserved: int
    target_addr: ipaddress.IPv6Address
    options: List[NdpOptionPacket] = field(default_factory=list)
    payload: bytes = b""

    @classmethod
    def try_from(cls, pkt: Icmpv6Packet) -> "NeighborSolicitPacket":  # icmpv6.rs:1266-1315
        if pkt.header.icmp_type != 135:
            raise ViewError("Not a Neighbor Solicitation packet")
        if len(pkt.payload) < 24:  # asks 24 B though the fixed part is 20 (a 24-B message fails)
            raise ViewError("Payload too short for Neighbor Solicitation")
        p = pkt.payload
        return cls(pkt.header, int.from_bytes(p[:4], "big"), ipaddress.IPv6Address(bytes(p[4:20])),
                   _ndp_options(p[20:]))

    @classmethod
    def from_bytes(cls, b: bytes) -> "NeighborSolicitPacket":  # icmpv6.rs:1319-1377: >= 24 B
        if len(b) < 24:
            raise ViewError("Malformed")
        opts, rest = _ndp_options_buf(b, 24, True)
        return cls(_hdr(b), int.from_bytes(b[4:8], "big"), ipaddress.IPv6Address(bytes(b[8:24])), opts, rest)

    def to_bytes(self) -> bytes:  # icmpv6.rs:1385-1400
        return (_hdr_bytes(self.header) + self.reserved.to_bytes(4, "big") + self.target_addr.packed +
                _opts_bytes(self.options))

    def total_len(self) -> int:  # ICMPV6_HEADER_LEN + 24 + payload (empty after try_from), icmpv6.rs:1407-1417
        return 8 + 24 + len(self.payload)

    def options_length(self) -> int:  # icmpv6.rs:1426-1433
        n = len(self.to_bytes())
        return n - 24 if n > 24 else 0


@dataclass
class NeighborAdvertPacket:  # icmpv6.rs:1472-1664
    header: IcmpHeader
    flags: int
    reserved: int
    target_addr: ipaddress.IPv6Address
    options: List[NdpOptionPacket] = field(default_factory=list)
    payload: bytes = b""

    @classmethod
    def try_from(cls, pkt: Icmpv6Packet) -> "NeighborAdvertPacket":  # icmpv6.rs:1481-1535
        if pkt.header.icmp_type != 136:
            raise ViewError("Not a Neighbor Advert packet")
        if len(pkt.payload) < 20:
            raise ViewError("Payload too short for Neighbor Advert")
        p = pkt.payload
        return cls(pkt.header, p[0], int.from_bytes(p[1:4], "big"), ipaddress.IPv6Address(bytes(p[4:20])),
                   _ndp_options(p[20:]))

    @classmethod
    def from_bytes(cls, b: bytes) -> "NeighborAdvertPacket":  # icmpv6.rs:1539-1603: >= 24 B
        if len(b) < 24:
            raise ViewError("Malformed")
        opts, rest = _ndp_options_buf(b, 24, True)
        return cls(_hdr(b), b[4], int.from_bytes(b[5:8], "big"), ipaddress.IPv6Address(bytes(b[8:24])), opts, rest)

    def to_bytes(self) -> bytes:  # icmpv6.rs:1610-1631: flags << 24 | reserved & 0xFFFFFF
        fr = (self.flags << 24) | (self.reserved & 0xFFFFFF)
        return _hdr_bytes(self.header) + fr.to_bytes(4, "big") + self.target_addr.packed + _opts_bytes(self.options)

    def total_len(self) -> int:  # icmpv6.rs:1638-1648
        return 8 + 24 + len(self.payload)

    def options_length(self) -> int:  # icmpv6.rs:1656-1663
        n = len(self.to_bytes())
        return n - 24 if n > 24 else 0


@dataclass
class RedirectPacket:  # icmpv6.rs:1696-1901
    header: IcmpHeader
    reserved: int
    target_addr: ipaddress.IPv6Address
    dest_addr: ipaddress.IPv6Address
    options: List[NdpOptionPacket] = field(default_factory=list)
    payload: bytes = b""

    @classmethod
    def try_from(cls, pkt: Icmpv6Packet) -> "RedirectPacket":  # icmpv6.rs:1705-1765
        if pkt.header.icmp_type != 137:
            raise ViewError("Not a Redirect packet")
        if len(pkt.payload) < 40:  # asks 40 B though the fixed part is 36 (a 40-B message fails)
            raise ViewError("Payload too short for Redirect")
        p = pkt.payload
        return cls(pkt.header, int.from_bytes(p[:4], "big"), ipaddress.IPv6Address(bytes(p[4:20])),
                   ipaddress.IPv6Address(bytes(p[20:36])), _ndp_options(p[36:]))

    @classmethod
    def from_bytes(cls, b: bytes) -> "RedirectPacket":  # icmpv6.rs:1769-1843: >= 40 B
        if len(b) < 40:
            raise ViewError("Malformed")
        opts, rest = _ndp_options_buf(b, 40, True)
        return cls(_hdr(b), int.from_bytes(b[4:8], "big"), ipaddress.IPv6Address(bytes(b[8:24])),
                   ipaddress.IPv6Address(bytes(b[24:40])), opts, rest)

    def to_bytes(self) -> bytes:  # icmpv6.rs:1849-1867
        return (_hdr_bytes(self.header) + self.reserved.to_bytes(4, "big") + self.target_addr.packed +
                self.dest_addr.packed + _opts_bytes(self.options))

    def total_len(self) -> int:  # ICMPV6_HEADER_LEN + 40 + payload, icmpv6.rs:1874-1884
        return 8 + 40 + len(self.payload)

    def options_length(self) -> int:  # icmpv6.rs:1893-1900
        n = len(self.to_bytes())
        return n - 40 if n > 40 else 0


NDP_VIEWS = {133: RouterSolicitPacket, 134: RouterAdvertPacket, 135: NeighborSolicitPacket,
             136: NeighborAdvertPacket, 137: RedirectPacket}


def icmpv6_message_bytes(rec, frame: bytes) -> Optional[bytes]:
    """The ICMPv6 message a GPU record located: from its L4 offset to the end
    of the Frame's IP payload (what Packet::try_from_buf of an NDP message
    takes, icmpv6.rs ndp); None without an ICMPv6 layer."""
    if not int(rec["flags"]) & abi.L_ICMPV6:
        return None
    l4, po, pl = int(rec["l4_off"]), int(rec["payload_off"]), int(rec["payload_len"])
    end = po + pl if pl else l4 + 4
    return bytes(frame[l4:end])


IcmpView = Union[EchoRequestPacket, EchoReplyPacket, DestinationUnreachablePacket, TimeExceededPacket]


def icmp_from_record(rec, frame: bytes) -> Optional[IcmpPacket]:
    """Frame.ip.icmp plus its payload (Q15: bytes after the 4-B header) as
    the IcmpPacket the GPU parse located; None when the Frame has no ICMP."""
    if not int(rec["flags"]) & abi.L_ICMP:
        return None
    l4, po, pl = int(rec["l4_off"]), int(rec["payload_off"]), int(rec["payload_len"])
    return IcmpPacket(IcmpHeader(int(rec["l4_type"]), int(rec["l4_code"]), int(rec["l4_csum"])),
                      bytes(frame[po:po + pl]) if pl else bytes(frame[l4 + 4:l4 + 4]))


def icmpv6_from_record(rec, frame: bytes) -> Optional[Icmpv6Packet]:
    if not int(rec["flags"]) & abi.L_ICMPV6:
        return None
    po, pl = int(rec["payload_off"]), int(rec["payload_len"])
    return Icmpv6Packet(IcmpHeader(int(rec["l4_type"]), int(rec["l4_code"]), int(rec["l4_csum"])),
                        bytes(frame[po:po + pl]))


def icmp_message(pkt: IcmpPacket) -> IcmpView:
    """The typed ICMP message by type, as dump.rs:226-288 downcasts."""
    t = pkt.header.icmp_type
    conv = {8: EchoRequestPacket, 0: EchoReplyPacket, 3: DestinationUnreachablePacket,
            11: TimeExceededPacket}.get(t)
    if conv is None:
        raise ViewError(f"no typed view for ICMP type {t}")
    return conv.try_from(pkt)


# ---- the layer walk of examples/dump.rs ------------------------------------

def ip_payload_from_record(rec, frame: bytes) -> Optional[bytes]:
    """Ipv4Packet / Ipv6Packet.payload of the Frame's IP layer (lenient, the
    mode dump.rs's try_from_bytes uses): IPv4 [IHL*4, effective total);
    IPv6 after the extension chain up to min(40 + payload_length, captured)."""
    f = int(rec["flags"])
    l3 = int(rec["l3_off"])
    if f & abi.L_IPV4:
        return bytes(frame[l3 + 4 * (int(rec["ip_ver_ihl"]) & 15):l3 + int(rec["ip_length"])])
    if f & abi.L_IPV6:
        end = l3 + min(40 + int(rec["ip_length"]), len(frame) - l3)
        if f & (abi.L_TCP | abi.L_UDP | abi.L_ICMPV6):
            start = int(rec["l4_off"])
        elif int(rec["payload_len"]):
            start = int(rec["payload_off"])
        else:
            start = end
        return bytes(frame[start:end])
    return None


def _tcp_total_len(seg: bytes) -> Optional[int]:
    """TcpPacket::try_from_bytes + total_len (tcp.rs:585-617): None if it fails."""
    from .frame import _tcp_options
    if len(seg) < 20:
        return None
    hl = (seg[12] >> 4) * 4
    if hl < 20 or hl > len(seg):
        return None
    off, ok = 20, True
    while off < hl:
        kind = seg[off]
        off += 1
        if kind == 0:
            break
        if kind == 1:
            continue
        if off >= hl:
            ok = False
            break
        ln = seg[off]
        off += 1
        if ln < 2 or off + ln - 2 > hl:
            ok = False
            break
        off += ln - 2
    if not ok:
        return None
    opt = sum(1 if k in (0, 1) else (ln or 2) for k, ln, _ in _tcp_options(seg, 0, hl))
    return ((20 + opt + 3) & ~3) + (len(seg) - hl)


def _transport_lines(src: str, dst: str, fam: str, proto: int, p: bytes) -> List[str]:
    """dump.rs:166-350 handle_transport_protocol and the handle_* it calls."""
    if proto == 6:
        tl = _tcp_total_len(p)
        if tl is None:
            return ["Malformed TCP Packet"]
        return [f"TCP Packet: {src}:{_be16(p, 0)} > {dst}:{_be16(p, 2)}; length: {tl}"]
    if proto == 17:
        ul = _be16(p, 4) if len(p) >= 8 else 0
        if len(p) < 8 or ul < 8 or ul > len(p):
            return ["Malformed UDP Packet"]
        return [f"UDP Packet: {src}:{_be16(p, 0)} > {dst}:{_be16(p, 2)}; length: {ul}"]
    if proto == 1:
        try:
            pkt = IcmpPacket.try_from_bytes(p)
        except ViewError:
            return ["Malformed ICMP Packet"]
        t, tl = pkt.header.icmp_type, pkt.total_len()
        try:
            if t == 8:
                m = EchoRequestPacket.try_from(pkt)
                return [f"ICMP echo request {src} -> {dst} (seq={m.sequence_number}, id={m.identifier}), "
                        f"length: {tl}"]
            if t == 0:
                m = EchoReplyPacket.try_from(pkt)
                return [f"ICMP echo reply {src} -> {dst} (seq={m.sequence_number}, id={m.identifier}), "
                        f"length: {tl}"]
            if t == 3:
                m = DestinationUnreachablePacket.try_from(pkt)
                return [f"ICMP destination unreachable {src} -> {dst} (code=IcmpCode({m.header.icmp_code})), "
                        f"next_hop_mtu={m.next_hop_mtu}, length: {tl}"]
            if t == 11:
                m = TimeExceededPacket.try_from(pkt)
                return [f"ICMP time exceeded {src} -> {dst} (code=IcmpCode({m.header.icmp_code})), length: {tl}"]
        except ViewError as e:  # dump.rs unwraps the conversion: the reference panics here
            return [f"panic: {e}"]
        return [f"ICMP packet {src} -> {dst} (type={icmp_type_debug(t)}), length: {tl}"]
    if proto == 58:
        try:
            pkt = Icmpv6Packet.try_from_bytes(p)
        except ViewError:
            return ["Malformed ICMPv6 Packet"]
        t = pkt.header.icmp_type
        try:
            if t in (128, 129):
                m = Icmpv6EchoPacket.try_from(pkt, reply=t == 129)
                what = "echo reply" if t == 129 else "echo request"
                return [f"ICMPv6 {what} {src} -> {dst} (type={icmpv6_type_debug(t)}), length: {m.total_len()}"]
            if t == 135:
                m = NeighborSolicitPacket.try_from(pkt)
                return [f"ICMPv6 neighbor solicitation {src} -> {dst} (type={icmpv6_type_debug(t)}), "
                        f"length: {m.total_len()}"]
            if t == 136:
                m = NeighborAdvertPacket.try_from(pkt)
                return [f"ICMPv6 neighbor advertisement {src} -> {dst} (type={icmpv6_type_debug(t)}), "
                        f"length: {m.total_len()}"]
        except ViewError as e:
            return [f"panic: {e}"]
        return [f"ICMPv6 packet {src} -> {dst} (type={icmpv6_type_debug(t)}), length: {pkt.total_len()}"]
    return [f"Unknown {fam} packet: {src} > {dst}; protocol: {ipproto_debug(proto)} length: {len(p)}"]


def dump_lines(rec, frame: bytes) -> List[str]:
    """dump.rs:96-350 handle_ethernet_frame for one frame from its GPU record
    (NEXG_OUT_RECORD, lenient mode) and bytes."""
    f = int(rec["flags"])
    if abi.status_of(f):  # EthernetPacket::try_from_buf(..).unwrap() (dump.rs:88) would panic
        return ["panic: Ethernet packet shorter than 14 bytes"]
    et = int(rec["ethertype"])
    l3 = int(rec["l3_off"])
    if et == 0x0800 or et == 0x86DD:
        fam = "IPv4" if et == 0x0800 else "IPv6"
        if not f & (abi.L_IPV4 | abi.L_IPV6):
            return [f"Malformed {fam} Packet"]
        if f & abi.L_IPV4:
            src, dst = str(ipaddress.IPv4Address(int(rec["ip_src"]))), str(ipaddress.IPv4Address(int(rec["ip_dst"])))
        else:
            src = ipv6_display(ipaddress.IPv6Address(bytes(frame[l3 + 8:l3 + 24])))
            dst = ipv6_display(ipaddress.IPv6Address(bytes(frame[l3 + 24:l3 + 40])))
        return _transport_lines(src, dst, fam, int(rec["ip_proto"]), ip_payload_from_record(rec, frame))
    if et == 0x0806:
        if not f & abi.L_ARP:
            return ["Malformed ARP Packet"]
        b = frame
        return [f"ARP packet: {_mac(b[l3 + 8:l3 + 14])}({ipaddress.IPv4Address(int(rec['ip_src']))}) > "
                f"{_mac(b[l3 + 18:l3 + 24])}({ipaddress.IPv4Address(int(rec['ip_dst']))}); operation: "
                f"{ARP_OP_NAMES.get(int(rec['l4_length']), 'Unknown(%d)' % int(rec['l4_length']))}"]
    disp = _ETHERTYPE_DISPLAY.get(et, "Unknown")
    return [f"{disp} packet: {_mac(frame[6:12])} > {_mac(frame[0:6])}; ethertype: {ethertype_debug(et)} "
            f"length: {len(frame)}"]


# EtherType::name (ethernet.rs:86-113): the display names dump.rs prints
_ETHERTYPE_DISPLAY = {0x0800: "IPv4", 0x0806: "ARP", 0x0842: "WakeOnLan", 0x22F3: "Trill", 0x6003: "DECnet",
                      0x8035: "RARP", 0x809B: "AppleTalk", 0x80F3: "AARP", 0x8137: "IPX", 0x8204: "QNX",
                      0x86DD: "IPv6", 0x8808: "FlowControl", 0x8819: "CobraNet", 0x8847: "MPLS",
                      0x8848: "MPLS Multicast", 0x8863: "PPPoE Discovery", 0x8864: "PPPoE Session",
                      0x8100: "VLAN", 0x88A8: "Provider Bridging", 0x88CC: "LLDP", 0x88F7: "PTP",
                      0x8902: "CFM", 0x9100: "QinQ", 0x8899: "RLDP"}


def dump_records(records, frames, source: str, first_no: int = 1):
    """The dump.rs:54-93 loop over one parsed batch: a header line per frame,
    then its layer lines."""
    for k, (rec, fr) in enumerate(zip(records, frames)):
        yield f"---- Interface: {source}, No.: {first_no + k}, Total Length: {len(fr)} bytes ----"
        yield from dump_lines(rec, fr)
