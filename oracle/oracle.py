"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU restatement
(oracle/nex_oracle.c, built into oracle/liboracle.so by oracle/Makefile).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module. Parity status: pinned by the reference's own KATs and fixtures
(tests/golden/); the Rust reference itself cannot be built here.
"""
import ctypes
import os
import subprocess

import numpy as np

from nex_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        P, S, U16, U32, U64, I = (ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint16,
                                  ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int)
        L.nexo_checksum.restype = U16
        L.nexo_checksum.argtypes = [P, S, S]
        L.nexo_sum_be_words.restype = U32
        L.nexo_sum_be_words.argtypes = [P, S, S]
        L.nexo_sum_be_words_joined.restype = U32
        L.nexo_sum_be_words_joined.argtypes = [P, S, S, P, S]
        L.nexo_ipv4_checksum.restype = U16
        L.nexo_ipv4_checksum.argtypes = [P, S, S, P, S, P, P, ctypes.c_uint8]
        L.nexo_ipv6_checksum.restype = U16
        L.nexo_ipv6_checksum.argtypes = [P, S, S, P, S, P, P, ctypes.c_uint8]
        L.nexo_parse_frame.restype = None
        L.nexo_parse_frame.argtypes = [P, S, U32, U32, P]
        L.nexo_parse_batch.restype = I
        L.nexo_parse_batch.argtypes = [ctypes.POINTER(abi.Frames), U32, U32, P, P, I]
        L.nexo_build_udp4.restype = I
        L.nexo_build_udp4.argtypes = [P, P, U32, U32, U16, U16, U16, ctypes.c_uint8, ctypes.c_uint8,
                                      ctypes.c_uint8, P, U32, P]
        L.nexo_build_udp4_batch.restype = I
        L.nexo_build_udp4_batch.argtypes = [ctypes.POINTER(Udp4Tuples), P, I]
        L.nexo_slice_frame.restype = None
        L.nexo_decode_options.argtypes = [P, ctypes.c_size_t, U32, U32, P]
        L.nexo_decode_options.restype = None
        L.nexo_slice_frame.argtypes = [P, ctypes.c_size_t, U32, U32, P]
        L.nexo_slice_batch.restype = None
        L.nexo_slice_batch.argtypes = [ctypes.POINTER(abi.Frames), U32, U32, P]
        L.nexo_build_tcp.restype = I
        L.nexo_build_tcp.argtypes = [ctypes.POINTER(IpSpec), U16, U16, U32, U32, ctypes.c_uint8, U16,
                                     U16, P, U32, P, U32, P]
        L.nexo_build_icmp_echo.restype = I
        L.nexo_build_icmp_echo.argtypes = [ctypes.POINTER(IpSpec), ctypes.c_uint8, ctypes.c_uint8,
                                           U16, U16, P, U32, P]
        L.nexo_build_arp.restype = I
        L.nexo_build_arp.argtypes = [P, P, P, P, P, U16, U16, U16, ctypes.c_uint8, ctypes.c_uint8, P]
        L.nexo_build_ndp_ns.restype = I
        L.nexo_build_ndp_ns.argtypes = [ctypes.POINTER(IpSpec), P]
        L.nexo_build_udp6.restype = I
        L.nexo_build_udp6.argtypes = [P, P, P, P, U16, U16, ctypes.c_uint8, ctypes.c_uint8, U32, P,
                                      U32, P]
        L.nexo_build_probe_batch.restype = I
        L.nexo_build_probe_batch.argtypes = [ctypes.POINTER(ProbeBatch), P, I]
        L.nexo_recompute_frame.restype = None
        L.nexo_recompute_frame.argtypes = [P, S, U32, U32, U32, P]
        L.nexo_gen_length.restype = U32
        L.nexo_gen_length.argtypes = [I, U64, U64]
        L.nexo_gen_frame.restype = None
        L.nexo_gen_frame.argtypes = [I, U64, U64, P]
        L.nexo_gen_udp4_params.restype = None
        L.nexo_gen_udp4_params.argtypes = [U64, U64, P, P, P, P, P]
        _lib = L
    return _lib


def _buf(b):
    b = bytes(b)
    return ctypes.create_string_buffer(b, max(len(b), 1)), len(b)


def checksum(data, skipword):
    buf, n = _buf(data)
    return lib().nexo_checksum(buf, n, min(skipword, 2**63))


def sum_be_words(data, skipword):
    buf, n = _buf(data)
    return lib().nexo_sum_be_words(buf, n, min(skipword, 2**63))


def sum_be_words_joined(data, skipword, extra):
    b1, n1 = _buf(data)
    b2, n2 = _buf(extra)
    return lib().nexo_sum_be_words_joined(b1, n1, min(skipword, 2**63), b2, n2)


def ipv6_checksum(data, skipword, src, dst, proto):
    buf, n = _buf(data)
    return lib().nexo_ipv6_checksum(buf, n, skipword, None, 0, bytes(src), bytes(dst), proto)


def ipv4_checksum(data, skipword, src, dst, proto):
    buf, n = _buf(data)
    return lib().nexo_ipv4_checksum(buf, n, skipword, None, 0, bytes(src), bytes(dst), proto)


def parse_frame(frame, flags=0, ip_offset=0):
    rec = np.zeros(1, dtype=abi.RECORD_DTYPE)
    buf, n = _buf(frame)
    lib().nexo_parse_frame(buf, n, flags, ip_offset, rec.ctypes.data)
    return rec[0]


def parse_packed(data: np.ndarray, offsets=None, lengths=None, stride=0, flags=0, ip_offset=0,
                 nthreads=1):
    """Parse a host-memory batch laid out as nexg_frames; returns records."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    count = (len(lengths) if lengths is not None else
             (len(offsets) - 1 if offsets is not None else len(data) // stride))
    offs = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    lens = None if lengths is None else np.ascontiguousarray(lengths, dtype=np.uint32)
    fr = abi.Frames(data=data.ctypes.data, data_bytes=data.nbytes,
                    offsets=None if offs is None else offs.ctypes.data,
                    lengths=None if lens is None else lens.ctypes.data,
                    stride=stride, reserved=0, count=count)
    recs = np.zeros(count, dtype=abi.RECORD_DTYPE)
    lib().nexo_parse_batch(ctypes.byref(fr), flags, ip_offset, recs.ctypes.data, None, nthreads)
    return recs


def decode_options(frame: bytes, flags=0, ip_offset=0):
    """Option lists of the Frame (ipv4.rs:442-508, tcp.rs:767-818) -> one nexg_options."""
    out = np.zeros(1, dtype=abi.OPTIONS_DTYPE)
    b, n = _buf(frame)
    lib().nexo_decode_options(b, n, flags, ip_offset, out.ctypes.data)
    return out[0]


def slice_frame(frame: bytes, flags=0, ip_offset=0):
    """FrameSlice::try_from_buf (frame.rs:84-287) -> one nexg_slice."""
    out = np.zeros(1, dtype=abi.SLICE_DTYPE)
    b, n = _buf(frame)
    lib().nexo_slice_frame(b, n, flags, ip_offset, out.ctypes.data)
    return out[0]


def slice_packed(data: np.ndarray, offsets=None, lengths=None, stride=0, flags=0, ip_offset=0):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    count = (len(lengths) if lengths is not None else
             (len(offsets) - 1 if offsets is not None else len(data) // stride))
    offs = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    lens = None if lengths is None else np.ascontiguousarray(lengths, dtype=np.uint32)
    fr = abi.Frames(data=data.ctypes.data, data_bytes=data.nbytes,
                    offsets=None if offs is None else offs.ctypes.data,
                    lengths=None if lens is None else lens.ctypes.data,
                    stride=stride, reserved=0, count=count)
    out = np.zeros(count, dtype=abi.SLICE_DTYPE)
    lib().nexo_slice_batch(ctypes.byref(fr), flags, ip_offset, out.ctypes.data)
    return out


def parse_frames(frames, flags=0, ip_offset=0):
    return np.array([parse_frame(f, flags, ip_offset) for f in frames], dtype=abi.RECORD_DTYPE)


def build_udp4(src_mac, dst_mac, src_ip, dst_ip, sport, dport, ip_id=0, ttl=64, ip_flags=0,
               dscp_ecn=0, payload=b""):
    out = ctypes.create_string_buffer(42 + len(payload) + 64)
    pb, pn = _buf(payload)
    n = lib().nexo_build_udp4(bytes(src_mac), bytes(dst_mac), src_ip, dst_ip, sport, dport, ip_id,
                              ttl, ip_flags, dscp_ecn, pb, pn, out)
    if n < 0:
        raise ValueError("BuildError::LengthOverflow")
    return out.raw[:n]


class Udp4Tuples(ctypes.Structure):
    _fields_ = [("src_mac", ctypes.c_void_p), ("dst_mac", ctypes.c_void_p), ("src_ip", ctypes.c_void_p),
                ("dst_ip", ctypes.c_void_p), ("src_port", ctypes.c_void_p), ("dst_port", ctypes.c_void_p),
                ("ip_id", ctypes.c_void_p), ("count", ctypes.c_uint64), ("ttl", ctypes.c_uint8),
                ("ip_flags", ctypes.c_uint8)]


def build_udp4_batch(src_mac, dst_mac, src_ip, dst_ip, sport, dport, ip_id, ttl=64, ip_flags=0,
                     nthreads=1, out=None):
    """udp_ping IPv4 builds (empty payload) over numpy tuple arrays: a
    (count, 42) uint8 array; `nthreads` static index-range shards."""
    src_ip = np.ascontiguousarray(src_ip, np.uint32)
    dst_ip = np.ascontiguousarray(dst_ip, np.uint32)
    sport = np.ascontiguousarray(sport, np.uint16)
    dport = np.ascontiguousarray(dport, np.uint16)
    ip_id = np.ascontiguousarray(ip_id, np.uint16)
    n = len(src_ip)
    if out is None:
        out = np.empty((n, 42), np.uint8)
    sm, dm = _buf(src_mac)[0], _buf(dst_mac)[0]
    t = Udp4Tuples(ctypes.cast(sm, ctypes.c_void_p), ctypes.cast(dm, ctypes.c_void_p), src_ip.ctypes.data,
                   dst_ip.ctypes.data, sport.ctypes.data, dport.ctypes.data, ip_id.ctypes.data, n, ttl, ip_flags)
    lib().nexo_build_udp4_batch(ctypes.byref(t), out.ctypes.data, nthreads)
    return out


def build_udp6(src_mac, dst_mac, src_ip: bytes, dst_ip: bytes, sport, dport, hop_limit=64,
               traffic_class=0, flow_label=0, payload=b""):
    """udp_ping IPv6 branch (examples/udp_ping.rs:83-89): Eth/IPv6/UDP bytes."""
    out = ctypes.create_string_buffer(62 + len(payload) + 64)
    pb, pn = _buf(payload)
    n = lib().nexo_build_udp6(bytes(src_mac), bytes(dst_mac), bytes(src_ip), bytes(dst_ip), sport,
                              dport, hop_limit, traffic_class, flow_label, pb, pn, out)
    if n < 0:
        raise ValueError("BuildError::LengthOverflow")
    return out.raw[:n]


class IpSpec(ctypes.Structure):
    """struct nexo_ip_spec (oracle/nex_oracle.h)"""
    _fields_ = [("family", ctypes.c_int), ("src", ctypes.c_uint8 * 16), ("dst", ctypes.c_uint8 * 16),
                ("src_mac", ctypes.c_uint8 * 6), ("dst_mac", ctypes.c_uint8 * 6),
                ("ip_id", ctypes.c_uint16), ("ttl", ctypes.c_uint8), ("ip_flags", ctypes.c_uint8),
                ("dscp_ecn", ctypes.c_uint8), ("flow_label", ctypes.c_uint32)]


def ip_spec(family, src: bytes, dst: bytes, src_mac=bytes(6), dst_mac=bytes(6), ip_id=0, ttl=64,
            ip_flags=0, dscp_ecn=0, flow_label=0):
    sp = IpSpec(family=family, ip_id=ip_id, ttl=ttl, ip_flags=ip_flags, dscp_ecn=dscp_ecn,
                flow_label=flow_label)
    sp.src[:len(src)] = list(src)
    sp.dst[:len(dst)] = list(dst)
    sp.src_mac[:] = list(src_mac)
    sp.dst_mac[:] = list(dst_mac)
    return sp


def build_tcp(spec, sport, dport, seq=0, ack=0, flags=0, window=0xFFFF, urg=0, options=b"",
              payload=b""):
    """TcpPacketBuilder -> Ipv4/Ipv6PacketBuilder -> EthernetPacketBuilder (tcp_ping.rs)."""
    out = ctypes.create_string_buffer(54 + 60 + len(payload) + 64)
    ob, on = _buf(options)
    pb, pn = _buf(payload)
    n = lib().nexo_build_tcp(ctypes.byref(spec), sport, dport, seq, ack, flags, window, urg, ob, on,
                             pb, pn, out)
    if n < 0:
        raise ValueError("BuildError::LengthOverflow")
    return out.raw[:n]


class ProbeBatch(ctypes.Structure):
    """struct nexo_probe_batch (oracle/nex_oracle.h)"""
    _fields_ = [("kind", ctypes.c_int), ("ip", IpSpec), ("dst", ctypes.c_void_p), ("count", ctypes.c_uint64),
                ("sport", ctypes.c_uint16), ("dport", ctypes.c_uint16), ("window", ctypes.c_uint16),
                ("urg", ctypes.c_uint16), ("seq", ctypes.c_uint32), ("ack", ctypes.c_uint32),
                ("tcp_flags", ctypes.c_uint8), ("icmp_type", ctypes.c_uint8), ("icmp_code", ctypes.c_uint8),
                ("pad0", ctypes.c_uint8), ("ident", ctypes.c_uint16), ("seqno", ctypes.c_uint16),
                ("opts", ctypes.c_void_p), ("opt_len", ctypes.c_uint32),
                ("payload", ctypes.c_void_p), ("payload_len", ctypes.c_uint32)]


PROBE_KIND = {"tcp": 0, "icmp": 1, "udp6": 2}


def build_probe_batch(kind, spec, dst, nthreads=1, out=None, **l4):
    """A probe batch (nexo_build_probe_batch): every frame built from `spec`
    and the L4 fields `l4` (tcp: sport, dport, seq, ack, flags, window, urg,
    options, payload; icmp: icmp_type, icmp_code, ident, seqno, payload; udp6:
    sport, dport, payload) with destination dst[i] ((count, 4|16) uint8).
    Returns a (count, flen) uint8 array."""
    dst = np.ascontiguousarray(dst, np.uint8)
    n = dst.shape[0]
    ob, on = _buf(l4.get("options", b""))
    pb, pn = _buf(l4.get("payload", b""))
    p = ProbeBatch(kind=PROBE_KIND[kind], ip=spec, dst=dst.ctypes.data, count=n,
                   sport=l4.get("sport", 0), dport=l4.get("dport", 0), window=l4.get("window", 0xFFFF),
                   urg=l4.get("urg", 0), seq=l4.get("seq", 0), ack=l4.get("ack", 0),
                   tcp_flags=l4.get("flags", 0), icmp_type=l4.get("icmp_type", 8),
                   icmp_code=l4.get("icmp_code", 0), ident=l4.get("ident", 0), seqno=l4.get("seqno", 0),
                   opts=ctypes.cast(ob, ctypes.c_void_p), opt_len=on,
                   payload=ctypes.cast(pb, ctypes.c_void_p), payload_len=pn)
    first = ctypes.create_string_buffer(70000)
    p.count = min(n, 1)  # one build first: the frame length (or the overflow)
    flen = lib().nexo_build_probe_batch(ctypes.byref(p), first, 1) if n else 0
    p.count = n
    if flen < 0:
        raise ValueError("BuildError::LengthOverflow")
    if out is None:
        out = np.empty((n, max(flen, 1)), np.uint8)
    if n:
        lib().nexo_build_probe_batch(ctypes.byref(p), out.ctypes.data, nthreads)
    return out


def build_icmp_echo(spec, icmp_type, code, ident, seqno, payload=b""):
    """Icmp(v6)PacketBuilder.echo_fields -> IP -> Ethernet (icmp_ping.rs)."""
    out = ctypes.create_string_buffer(62 + len(payload) + 64)
    pb, pn = _buf(payload)
    n = lib().nexo_build_icmp_echo(ctypes.byref(spec), icmp_type, code, ident, seqno, pb, pn, out)
    if n < 0:
        raise ValueError("BuildError::LengthOverflow")
    return out.raw[:n]


def build_arp(eth_dst: bytes, sender_mac: bytes, sender_ip: bytes, target_mac: bytes, target_ip: bytes,
              hardware_type=1, protocol_type=0x0800, operation=1, hw_len=6, proto_len=4):
    """ArpPacketBuilder -> EthernetPacketBuilder (examples/arp.rs:59-67)."""
    out = ctypes.create_string_buffer(64)
    n = lib().nexo_build_arp(bytes(eth_dst), bytes(sender_mac), bytes(sender_ip), bytes(target_mac),
                             bytes(target_ip), hardware_type, protocol_type, operation, hw_len, proto_len, out)
    if n < 0:
        raise ValueError("BuildError::InvalidFieldLength")
    return out.raw[:n]


def build_ndp_ns(spec):
    """NdpPacketBuilder -> Ipv6PacketBuilder -> EthernetPacketBuilder
    (examples/ndp.rs:82-108); spec.dst is the target, spec.dst_mac the
    Ethernet destination."""
    out = ctypes.create_string_buffer(128)
    n = lib().nexo_build_ndp_ns(ctypes.byref(spec), out)
    if n < 0:
        raise ValueError("NDP needs IPv6")
    return out.raw[:n]


def recompute_frame(frame: bytes, which=abi.FIX_IP | abi.FIX_L4, flags=0, ip_offset=0):
    """(fixed frame bytes, nexg_fixup) — the mutable views' recompute_checksum
    chained as examples/mutable_chaining.rs does (nexo_recompute_frame)."""
    buf, n = _buf(frame)
    out = np.zeros(1, abi.FIXUP_DTYPE)
    lib().nexo_recompute_frame(buf, n, flags, ip_offset, which, out.ctypes.data)
    return buf.raw[:n], out[0]


def gen_length(workload, index, seed=abi.DEFAULT_SEED):
    return lib().nexo_gen_length(workload, seed, index)


def gen_frame(workload, index, seed=abi.DEFAULT_SEED):
    n = gen_length(workload, index, seed)
    out = ctypes.create_string_buffer(max(n, 1504))
    lib().nexo_gen_frame(workload, seed, index, out)
    return out.raw[:n]


def gen_udp4_params(index, seed=abi.DEFAULT_SEED):
    v = [ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint16(), ctypes.c_uint16(), ctypes.c_uint16()]
    lib().nexo_gen_udp4_params(seed, index, *[ctypes.byref(x) for x in v])
    return tuple(x.value for x in v)
