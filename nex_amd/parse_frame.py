"""Batched counterpart of the reference's `examples/parse_frame.rs`.

The reference receives one frame per `rx.next()` and calls
`Frame::try_from_buf` on it (parse_frame.rs:43-73), then prints it with
`display_frame` (parse_frame.rs:76-131). Here frames come from a capture file
(the datalink source that needs no privileges; nex-datalink's `pcap::from_file`
channel, pcap.rs:95-109), are moved to the GPU a batch at a time and parsed by
`nexg_parse_batch` (NEXG_OUT_RECORD); each record is materialised as a
`Frame` (frame.py::frame_from_record) and printed in display_frame's layout.

    python -m nex_amd.parse_frame capture.pcap [--batch N] [--limit N]

Enum names follow the reference's `Debug` output for the common values
(EtherType::new, ethernet.rs:56-80; IpNextProtocol, ip.rs:308-456); other
EtherTypes print as the derived Debug does (`Unknown(<decimal>)`); IP protocol
numbers outside the table print as `IpNextProtocol(n)` — display only, the
parsed values are exact.
"""
import argparse
import sys
from typing import Iterator, List

import numpy as np

from . import abi
from .frame import Frame, ParseMode, ParseOption, frame_from_record

ETHERTYPE_NAMES = {0x0800: "Ipv4", 0x0806: "Arp", 0x0842: "WakeOnLan", 0x22F3: "Trill",
                   0x6003: "DECnet", 0x8035: "Rarp", 0x809B: "AppleTalk", 0x80F3: "Aarp",
                   0x8137: "Ipx", 0x8204: "Qnx", 0x86DD: "Ipv6", 0x8808: "FlowControl",
                   0x8819: "CobraNet", 0x8847: "Mpls", 0x8848: "MplsMcast",
                   0x8863: "PppoeDiscovery", 0x8864: "PppoeSession", 0x8100: "Vlan",
                   0x88A8: "PBridge", 0x88CC: "Lldp", 0x88F7: "Ptp", 0x8902: "Cfm",
                   0x9100: "QinQ", 0x8899: "Rldp"}
IPPROTO_NAMES = {0: "Hopopt", 1: "Icmp", 2: "Igmp", 4: "Ipv4", 6: "Tcp", 17: "Udp",
                 41: "Ipv6", 43: "Ipv6Route", 44: "Ipv6Frag", 47: "Gre", 50: "Esp", 51: "Ah",
                 58: "Icmpv6", 59: "Ipv6NoNxt", 60: "Ipv6Opts", 132: "Sctp", 255: "Reserved"}
ARP_OPS = {1: "Request", 2: "Reply"}


def _mac(b: bytes) -> str:
    return ":".join(f"{x:02x}" for x in b)


def ethertype_debug(v: int) -> str:
    """EtherType's derived Debug: the variant name, or Unknown(<decimal u16>)."""
    return ETHERTYPE_NAMES.get(v, f"Unknown({v})")


def ipv6_display(a) -> str:
    """std::net::Ipv6Addr's Display: IPv4-mapped addresses in dotted form,
    otherwise RFC 5952 (what ipaddress prints)."""
    return f"::ffff:{a.ipv4_mapped}" if a.ipv4_mapped is not None else str(a)


def ipproto_debug(v: int) -> str:
    return IPPROTO_NAMES.get(v, f"IpNextProtocol({v})")


def display_frame(frame: Frame) -> List[str]:
    """parse_frame.rs:76-131, as lines."""
    out = [f"Packet Frame ({frame.packet_len} bytes)"]
    dl = frame.datalink
    if dl is not None:
        if dl.ethernet is not None:
            e = dl.ethernet
            out.append(f"  Ethernet: {_mac(e.source)} > {_mac(e.destination)} ({ethertype_debug(e.ethertype)})")
        if dl.arp is not None:
            a = dl.arp
            out.append(f"  ARP: {_mac(a.sender_hw_addr)}({a.sender_proto_addr}) > "
                       f"{_mac(a.target_hw_addr)}({a.target_proto_addr}); operation: "
                       f"{ARP_OPS.get(a.operation, f'Unknown({a.operation})')}")
    ip = frame.ip
    if ip is not None:
        if ip.ipv4 is not None:
            out.append(f"  IPv4: {ip.ipv4.source} -> {ip.ipv4.destination} "
                       f"(protocol: {ipproto_debug(ip.ipv4.next_level_protocol)})")
        if ip.ipv6 is not None:
            out.append(f"  IPv6: {ipv6_display(ip.ipv6.source)} -> {ipv6_display(ip.ipv6.destination)} "
                       f"(next header: {ipproto_debug(ip.ipv6.next_header)})")
        if ip.icmp is not None:
            out.append("  ICMP: present")
        if ip.icmpv6 is not None:
            out.append("  ICMPv6: present")
    tp = frame.transport
    if tp is not None:
        if tp.tcp is not None:
            out.append(f"  TCP: {tp.tcp.source} -> {tp.tcp.destination}")
        if tp.udp is not None:
            out.append(f"  UDP: {tp.udp.source} -> {tp.udp.destination}")
    if len(frame.payload):
        out.append(f"  Payload: {len(frame.payload)} bytes")
    return out


def display_records(records: np.ndarray, frames: List[bytes], first_no: int, source: str) -> Iterator[str]:
    """The per-frame print loop of parse_frame.rs:45-70 over one parsed batch."""
    for k, (rec, fr) in enumerate(zip(records, frames)):
        yield (f"---- Interface: {source}, No.: {first_no + k}, "
               f"Total Length: {len(fr)} bytes ----")
        status = abi.status_of(int(rec["flags"]))
        if status != 0:
            yield "Failed to parse packet as Frame"
            continue
        yield from display_frame(frame_from_record(rec, fr))


def parse_capture(path: str, engine=None, batch_frames: int = 1 << 16, limit: int = 0,
                  option: ParseOption = ParseOption(), mode: ParseMode = ParseMode.Lenient
                  ) -> Iterator[str]:
    """Capture file -> GPU batches -> display lines (frames numbered from 1)."""
    import torch

    from .engine import Engine, FrameBatch
    from .ingest import LINKTYPE_RAW, PcapReader
    eng = engine or Engine(0)
    rd = PcapReader(path)
    if rd.linktype == LINKTYPE_RAW and not option.from_ip_packet:
        option = ParseOption(True, 0)
    data = np.empty(batch_frames * 2048, np.uint8)
    offs = np.empty(batch_frames + 1, np.uint64)
    no = 1
    while True:
        n = rd.read_into(data, offs)
        if n == 0:
            break
        if limit:
            n = min(n, limit - no + 1)
        end = int(offs[n])
        frames = [bytes(data[int(offs[i]):int(offs[i + 1])]) for i in range(n)]
        dev = torch.from_numpy(data[:max(end, 16)].copy()).to(eng.torch_device)
        doffs = torch.from_numpy(offs[:n + 1].astype(np.int64)).to(eng.torch_device)
        recs = eng.parse_to_numpy(FrameBatch(data=dev, count=n, offsets=doffs), option, mode,
                                  abi.OUT_RECORD)
        yield from display_records(recs, frames, no, path)
        no += n
        if limit and no > limit:
            break


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("capture", help="pcap / pcapng file")
    ap.add_argument("--batch", type=int, default=1 << 16, help="frames per GPU batch")
    ap.add_argument("--limit", type=int, default=0, help="stop after N frames")
    ap.add_argument("--strict", action="store_true", help="ParseMode::Strict")
    args = ap.parse_args(argv)
    mode = ParseMode.Strict if args.strict else ParseMode.Lenient
    for line in parse_capture(args.capture, batch_frames=args.batch, limit=args.limit, mode=mode):
        print(line)


if __name__ == "__main__":
    sys.exit(main())
