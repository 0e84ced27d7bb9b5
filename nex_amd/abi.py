"""Python mirror of include/nexg.h: constants, ctypes structs, numpy dtypes.

Layouts here must match include/nexg.h byte for byte; tests/test_abi.py checks
the sizes against the C compiler's view.
"""
import ctypes

import numpy as np

ABI_VERSION = 1

# call status
OK, EINVAL, ENOMEM, EDEVICE, ELAUNCH, ERANGE, EPERM, EIO = 0, -1, -2, -3, -4, -5, -6, -7

# per-frame status: ParseError kind (nex-packet/src/parse.rs:51-97)
FRAME_OK = 0
ERR_BUFFER_TOO_SHORT = 1
ERR_INVALID_LENGTH = 2
ERR_MALFORMED = 3
ERR_TRUNCATED = 4
ERR_BAD_EXTENT = 7

PARSE_STRICT = 0x1
PARSE_FROM_IP = 0x2
PARSE_VLAN = 0x4  # extension: unwrap up to two 802.1Q/802.1ad/QinQ tags (not Frame semantics)

L_ETHERNET = 1 << 0
L_ARP = 1 << 1
L_IP = 1 << 2
L_IPV4 = 1 << 3
L_IPV6 = 1 << 4
L_ICMP = 1 << 5
L_ICMPV6 = 1 << 6
L_TRANSPORT = 1 << 7
L_TCP = 1 << 8
L_UDP = 1 << 9
C_IP_CHECKED = 1 << 10
C_IP_OK = 1 << 11
C_IP_PANIC = 1 << 12
C_L4_CHECKED = 1 << 13
C_L4_OK = 1 << 14
L_VLAN = 1 << 15
STATUS_SHIFT = 24
VERDICT_ERR = L_ARP | L_IP  # NEXG_VERDICT_ERR: never both in a parsed Frame

OUT_DESC = 1
OUT_RECORD = 2
OUT_SLICE = 3
OUT_FLAGS = 4  # nexg_desc.flags only (include/nexg.h)
OUT_VERDICT = 5  # lossless 2-B form of the flags word (include/nexg.h)
OUT_SPARSE = 6  # 1-B shape codes + per-64-frame exception slots (include/nexg.h)
OUT_GROUPED = 7  # SPARSE with uniform 64-frame groups as a head byte + 2 verdict masks
GROUPED_TILE_RUN = 0x80  # NEXG_GROUPED_TILE_RUN: a mixed group whose exceptions run per 256-frame tile

# NEXG_FRAMES_* hints (nexg_frames.hints)
FRAMES_MONOTONE = 0x1
FRAMES_OFFSETS32 = 0x2  # u32 offset table (+ 64-bit group bases over 4 GiB)


def offsets32_layout(count, with_bases):
    """(u32 entries, byte offset of the u64 group bases, base count, total
    bytes) of a NEXG_FRAMES_OFFSETS32 table for `count` frames whose table
    starts 8-B aligned (include/nexg.h nexg_offsets32_bytes)."""
    n = count + 1
    base_off = (4 * n + 7) // 8 * 8
    nb = (n + 255) // 256 if with_bases else 0
    return n, base_off, nb, (base_off + 8 * nb) if with_bases else 4 * n


def offsets32_table(offsets64, data_bytes):
    """numpy u64 offsets (count + 1 entries) -> the NEXG_FRAMES_OFFSETS32
    table as a uint8 array: offsets mod 2^32, then (data_bytes > 0xFFFFFFFF)
    the full offset of every 256th frame."""
    o = np.asarray(offsets64, dtype=np.uint64)
    count = len(o) - 1
    with_bases = data_bytes > 0xFFFFFFFF
    n, base_off, nb, total = offsets32_layout(count, with_bases)
    buf = np.zeros(total, np.uint8)
    buf[: 4 * n].view(np.uint32)[:] = (o & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    if with_bases:
        buf[base_off:].view(np.uint64)[:] = o[::256]
    return buf


def offsets32_decode(table, count, data_bytes):
    """The full u64 offsets (count + 1) of a NEXG_FRAMES_OFFSETS32 table
    (uint8 array), as the kernels read it."""
    t = np.asarray(table, np.uint8)
    with_bases = data_bytes > 0xFFFFFFFF
    n, base_off, nb, _ = offsets32_layout(count, with_bases)
    lo = t[: 4 * n].view(np.uint32).astype(np.uint64)
    if not with_bases:
        return lo
    b = t[base_off: base_off + 8 * nb].view(np.uint64)[np.arange(n) >> 8]
    return b + ((lo - (b & np.uint64(0xFFFFFFFF))) & np.uint64(0xFFFFFFFF))

# NEXG_OUT_SPARSE code byte
SPARSE_IP_OK = 0x10
SPARSE_L4_OK = 0x20
SPARSE_TAG_SHIFT = 6
SHAPE_EXCEPTION, SHAPE_IP_NONE = 0, 10
_V4 = L_ETHERNET | L_IP | L_IPV4 | C_IP_CHECKED
_V6 = L_ETHERNET | L_IP | L_IPV6
#: NEXG_SHAPE_FLAGS / NEXG_SHAPE_HDR (include/nexg.h), indexed by shape 0..15
SHAPE_FLAGS = np.array([
    0,
    _V4 | L_TRANSPORT | L_UDP | C_L4_CHECKED, _V4 | L_TRANSPORT | L_TCP | C_L4_CHECKED, _V4 | L_ICMP | C_L4_CHECKED,
    _V6 | L_TRANSPORT | L_UDP | C_L4_CHECKED, _V6 | L_TRANSPORT | L_TCP | C_L4_CHECKED, _V6 | L_ICMPV6 | C_L4_CHECKED,
    L_ETHERNET, _V4, _V6, L_ETHERNET | L_IP,
    1 << STATUS_SHIFT, 2 << STATUS_SHIFT, 3 << STATUS_SHIFT, 4 << STATUS_SHIFT, 7 << STATUS_SHIFT], np.uint32)
SHAPE_HDR = np.array([0, 28, 40, 24, 48, 60, 44, 0, 20, 40, 0, 0, 0, 0, 0, 0], np.int64)


def sparse_exc_offset(count):
    """NEXG_SPARSE_EXC_OFFSET: byte offset of the exception slots."""
    return (int(count) + 15) & ~15


def sparse_bytes(count):
    """NEXG_SPARSE_BYTES: size of a NEXG_OUT_SPARSE output."""
    return sparse_exc_offset(count) + 8 * int(count)


def grouped_offsets(count):
    """NEXG_GROUPED_{MASK,CODE,EXC}_OFFSET and NEXG_GROUPED_BYTES."""
    g = (int(count) + 63) >> 6
    mask = (g + 15) & ~15
    code = mask + 16 * g
    exc = (code + int(count) + 15) & ~15
    return mask, code, exc, exc + 8 * int(count)


def grouped_codes(buf, count):
    """Every frame's NEXG_OUT_SPARSE code from a NEXG_OUT_GROUPED output
    (nexg_grouped_code, vectorised)."""
    buf = np.asarray(buf, np.uint8)
    mask, code, _, _ = grouped_offsets(count)
    G = (count + 63) >> 6
    i = np.arange(count)
    g = i >> 6
    head = buf[:G].astype(np.int64)[g]
    m = buf[mask:mask + 16 * G].copy().view("<u8").reshape(-1, 2)
    b = (i & 63).astype(np.uint64)
    ip = (m[g, 0] >> b) & np.uint64(1)
    l4 = (m[g, 1] >> b) & np.uint64(1)
    uni = head | np.where(ip != 0, SPARSE_IP_OK, 0) | np.where(l4 != 0, SPARSE_L4_OK, 0)
    mixed = (head == 0) | (head == GROUPED_TILE_RUN)
    return np.where(mixed, buf[code:code + count].astype(np.int64), uni)


def grouped_to_desc(buf, count, lengths, parse_flags=0, ip_offset=0):
    """nexg_desc[count] from a NEXG_OUT_GROUPED output (uint8 host array)."""
    buf = np.asarray(buf, np.uint8)
    _, _, exc, _ = grouped_offsets(count)
    G = (count + 63) >> 6
    run = buf[:G][np.arange(count) >> 6] == GROUPED_TILE_RUN
    return codes_to_desc(grouped_codes(buf, count), buf[exc:exc + 8 * count].view(DESC_DTYPE), count, lengths,
                         parse_flags, ip_offset, tile_run=run)


def sparse_to_desc(buf, count, lengths, parse_flags=0, ip_offset=0):
    """nexg_desc[count] from a NEXG_OUT_SPARSE output (uint8 host array):
    nexg_sparse_decode per code, exceptions looked up per 64-frame group.
    `lengths` = every frame's length (int array)."""
    buf = np.asarray(buf, np.uint8)
    return codes_to_desc(buf[:count].astype(np.int64),
                         buf[sparse_exc_offset(count):sparse_exc_offset(count) + 8 * count].view(DESC_DTYPE),
                         count, lengths, parse_flags, ip_offset)


def codes_to_desc(codes, exc, count, lengths, parse_flags=0, ip_offset=0, tile_run=None):
    """nexg_sparse_decode over every code; code-0 frames take the k-th
    exception of their 64-frame group (exc = the exception slots), or of
    their 256-frame tile where `tile_run` (per frame) is set
    (NEXG_GROUPED_TILE_RUN groups)."""
    lengths = np.asarray(lengths, np.int64)[:count]
    shape, tags = codes & 0xF, (codes >> SPARSE_TAG_SHIFT) & 3
    out = np.zeros(count, DESC_DTYPE)
    fl = SHAPE_FLAGS[shape].astype(np.int64)
    pay = (shape >= 1) & (shape < SHAPE_IP_NONE)
    fl |= np.where(pay & ((codes & SPARSE_IP_OK) != 0), C_IP_OK, 0)
    fl |= np.where(pay & ((codes & SPARSE_L4_OK) != 0), C_L4_OK, 0)
    fl |= np.where((pay | (shape == SHAPE_IP_NONE)) & (tags > 0), L_VLAN, 0)
    base = ip_offset if parse_flags & PARSE_FROM_IP else 14
    h = base + 4 * tags + SHAPE_HDR[shape]
    plen = np.where(pay, lengths - h, 0)
    out["flags"] = fl.astype(np.uint32)
    out["payload_len"] = (plen & 0xFFFF).astype(np.uint16)
    out["payload_off"] = np.where(pay & (lengths > h), h, 0).astype(np.uint16)
    ex = np.nonzero(shape == SHAPE_EXCEPTION)[0]
    if len(ex):
        unit = np.full(len(ex), 64, np.int64) if tile_run is None else np.where(tile_run[ex], 256, 64)
        start = ex // unit * unit  # the first frame of the exception's group or tile
        first = np.searchsorted(ex, start)  # index in ex of that run's first exception
        rank = np.arange(len(ex)) - first
        out[ex] = exc[start + rank]
    return out

# FrameSlice presence bits (nexg_slice.flags)
S_DATALINK = 1 << 0
S_NETWORK = 1 << 1
S_TRANSPORT = 1 << 2
S_ETHERTYPE = 1 << 3
S_IP_PROTOCOL = 1 << 4
S_PROTO_SHIFT = 8

WL_UDP64 = 1
WL_IMIX = 2

#: seed of the synthetic workloads ("nex")
DEFAULT_SEED = 0x6E6578


#: NEXG_CTX_* -> the reference's ParseError context string (include/nexg.h)
ERR_CONTEXTS = (None, "Ethernet packet", "Frame dummy Ethernet classification", "IPv4 packet",
                "IPv4 packet version", "IPv4 header length", "IPv4 header", "IPv4 total length",
                "IPv4 options", "IPv4 option length", "IPv6 packet", "IPv6 packet version", "IPv6 payload",
                "IPv6 extension header", "IPv6 routing header", "IPv6 fragment header")


def status_of(flags):
    return (np.asarray(flags) >> STATUS_SHIFT) & 0x7


DESC_DTYPE = np.dtype([("flags", "<u4"), ("payload_off", "<u2"), ("payload_len", "<u2")])
assert DESC_DTYPE.itemsize == 8

SLICE_DTYPE = np.dtype([("flags", "<u4"), ("l3_off", "<u2"), ("l3_len", "<u2"), ("l4_len", "<u2"),
                        ("payload_off", "<u2"), ("payload_len", "<u2"), ("ethertype", "<u2")])
assert SLICE_DTYPE.itemsize == 16
FLAGS_DTYPE = np.dtype([("flags", "<u4")])
VERDICT_DTYPE = np.dtype([("verdict", "<u2")])


def verdict_to_flags(v):
    """NEXG_VERDICT_FLAGS (include/nexg.h): the flags words of 2-B verdicts."""
    v = np.asarray(v).astype(np.uint32)
    err = (v & VERDICT_ERR) == VERDICT_ERR
    return np.where(err, ((v >> 3) & 7) << STATUS_SHIFT, v).astype(np.uint32)
OPTIONS_DTYPE = np.dtype([("n_ip", "u1"), ("n_tcp", "u1"), ("ip_opt_off", "<u2"), ("tcp_opt_off", "<u2"),
                          ("reserved", "<u2"), ("ip_pos", "u1", 40), ("tcp_pos", "u1", 40), ("pad", "u1", 8)])
assert OPTIONS_DTYPE.itemsize == 96

RECORD_DTYPE = np.dtype([
    ("flags", "<u4"), ("payload_off", "<u2"), ("payload_len", "<u2"),
    ("packet_len", "<u2"), ("ethertype", "<u2"), ("l3_off", "<u2"), ("l4_off", "<u2"),
    ("ip_ver_ihl", "u1"), ("ip_tos", "u1"), ("ip_length", "<u2"),
    ("ip_word", "<u4"),
    ("ip_ttl", "u1"), ("ip_proto", "u1"), ("ip_nopt", "u1"), ("l4_nopt", "u1"),
    ("ip_src", "<u4"), ("ip_dst", "<u4"),
    ("ip_csum", "<u2"), ("ip_csum_calc", "<u2"), ("l4_csum", "<u2"), ("l4_csum_calc", "<u2"),
    ("src_port", "<u2"), ("dst_port", "<u2"), ("l4_length", "<u2"),
    ("l4_type", "u1"), ("l4_code", "u1"),
    ("tcp_seq", "<u4"), ("tcp_ack", "<u4"), ("tcp_window", "<u2"), ("tcp_urg", "<u2"),
])
assert RECORD_DTYPE.itemsize == 64


class Frames(ctypes.Structure):
    """struct nexg_frames"""
    _fields_ = [
        ("data", ctypes.c_void_p),
        ("data_bytes", ctypes.c_uint64),
        ("offsets", ctypes.c_void_p),
        ("lengths", ctypes.c_void_p),
        ("stride", ctypes.c_uint32),
        ("hints", ctypes.c_uint32),
        ("count", ctypes.c_uint64),
    ]


class ParseOptionC(ctypes.Structure):
    """struct nexg_parse_option"""
    _fields_ = [("flags", ctypes.c_uint32), ("ip_offset", ctypes.c_uint32)]


class Udp4Build(ctypes.Structure):
    """struct nexg_udp4_build"""
    _fields_ = [
        ("src_ip", ctypes.c_void_p),
        ("dst_ip", ctypes.c_void_p),
        ("src_port", ctypes.c_void_p),
        ("dst_port", ctypes.c_void_p),
        ("ip_id", ctypes.c_void_p),
        ("src_mac", ctypes.c_void_p),
        ("dst_mac", ctypes.c_void_p),
        ("payload", ctypes.c_void_p),
        ("payload_len", ctypes.c_uint32),
        ("def_src_port", ctypes.c_uint16),
        ("def_dst_port", ctypes.c_uint16),
        ("def_ip_id", ctypes.c_uint16),
        ("def_src_mac", ctypes.c_uint8 * 6),
        ("def_dst_mac", ctypes.c_uint8 * 6),
        ("ttl", ctypes.c_uint8),
        ("ip_flags", ctypes.c_uint8),
        ("dscp_ecn", ctypes.c_uint8),
        ("reserved", ctypes.c_uint8),
        ("def_src_ip", ctypes.c_uint32),
        ("count", ctypes.c_uint64),
    ]


#: struct nexg_udp4_tuple (16 B): the AoS per-frame tuple of nexg_build_udp4_tuples
UDP4_TUPLE_DTYPE = np.dtype([("src_ip", "<u4"), ("dst_ip", "<u4"), ("src_port", "<u2"), ("dst_port", "<u2"),
                             ("ip_id", "<u2"), ("reserved", "<u2")])


class Udp6Build(ctypes.Structure):
    """struct nexg_udp6_build"""
    _fields_ = [
        ("src_ip", ctypes.c_void_p),
        ("dst_ip", ctypes.c_void_p),
        ("src_port", ctypes.c_void_p),
        ("dst_port", ctypes.c_void_p),
        ("src_mac", ctypes.c_void_p),
        ("dst_mac", ctypes.c_void_p),
        ("payload", ctypes.c_void_p),
        ("payload_len", ctypes.c_uint32),
        ("flow_label", ctypes.c_uint32),
        ("def_src_port", ctypes.c_uint16),
        ("def_dst_port", ctypes.c_uint16),
        ("def_src_mac", ctypes.c_uint8 * 6),
        ("def_dst_mac", ctypes.c_uint8 * 6),
        ("hop_limit", ctypes.c_uint8),
        ("traffic_class", ctypes.c_uint8),
        ("src_shared", ctypes.c_uint8),
        ("reserved", ctypes.c_uint8),
        ("count", ctypes.c_uint64),
    ]


class IpBuild(ctypes.Structure):
    """struct nexg_ip_build"""
    _fields_ = [
        ("src_ip", ctypes.c_void_p), ("dst_ip", ctypes.c_void_p), ("ip_id", ctypes.c_void_p),
        ("src_mac", ctypes.c_void_p), ("dst_mac", ctypes.c_void_p),
        ("family", ctypes.c_uint32), ("flow_label", ctypes.c_uint32), ("def_ip_id", ctypes.c_uint16),
        ("def_src_mac", ctypes.c_uint8 * 6), ("def_dst_mac", ctypes.c_uint8 * 6),
        ("ttl", ctypes.c_uint8), ("ip_flags", ctypes.c_uint8), ("tos", ctypes.c_uint8),
        ("src_shared", ctypes.c_uint8), ("reserved", ctypes.c_uint8 * 2),
    ]


class TcpBuild(ctypes.Structure):
    """struct nexg_tcp_build"""
    _fields_ = [
        ("ip", IpBuild),
        ("src_port", ctypes.c_void_p), ("dst_port", ctypes.c_void_p), ("seq", ctypes.c_void_p),
        ("ack", ctypes.c_void_p), ("payload", ctypes.c_void_p), ("payload_len", ctypes.c_uint32),
        ("def_seq", ctypes.c_uint32), ("def_ack", ctypes.c_uint32),
        ("def_src_port", ctypes.c_uint16), ("def_dst_port", ctypes.c_uint16),
        ("window", ctypes.c_uint16), ("urgent_ptr", ctypes.c_uint16),
        ("flags", ctypes.c_uint8), ("options_len", ctypes.c_uint8), ("options", ctypes.c_uint8 * 40),
        ("reserved", ctypes.c_uint8 * 2), ("count", ctypes.c_uint64),
    ]


class IcmpEchoBuild(ctypes.Structure):
    """struct nexg_icmp_echo_build"""
    _fields_ = [
        ("ip", IpBuild),
        ("identifier", ctypes.c_void_p), ("sequence", ctypes.c_void_p), ("payload", ctypes.c_void_p),
        ("payload_len", ctypes.c_uint32), ("def_identifier", ctypes.c_uint16),
        ("def_sequence", ctypes.c_uint16), ("icmp_type", ctypes.c_uint8), ("icmp_code", ctypes.c_uint8),
        ("reserved", ctypes.c_uint8 * 2), ("count", ctypes.c_uint64),
    ]


class ArpBuild(ctypes.Structure):
    """struct nexg_arp_build"""
    _fields_ = [
        ("sender_ip", ctypes.c_void_p), ("target_ip", ctypes.c_void_p), ("sender_mac", ctypes.c_void_p),
        ("target_mac", ctypes.c_void_p), ("eth_dst", ctypes.c_void_p),
        ("def_sender_ip", ctypes.c_uint8 * 4), ("def_sender_mac", ctypes.c_uint8 * 6),
        ("def_target_mac", ctypes.c_uint8 * 6), ("def_eth_dst", ctypes.c_uint8 * 6),
        ("hardware_type", ctypes.c_uint16), ("protocol_type", ctypes.c_uint16), ("operation", ctypes.c_uint16),
        ("hw_addr_len", ctypes.c_uint8), ("proto_addr_len", ctypes.c_uint8), ("count", ctypes.c_uint64),
    ]


class NdpNsBuild(ctypes.Structure):
    """struct nexg_ndp_ns_build"""
    _fields_ = [("ip", IpBuild), ("eth_dst_multicast", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("count", ctypes.c_uint64)]


# in-place checksum fix-up (nexg_recompute_checksums_batch)
FIX_IP = 0x1
FIX_L4 = 0x2
FIXUP_DTYPE = np.dtype([("done", "u1"), ("proto", "u1"), ("ip_csum", "<u2"), ("l4_csum", "<u2"),
                        ("l4_off", "<u2")])
assert FIXUP_DTYPE.itemsize == 8

#: static inline helpers of include/nexg.h (header-only, not exported)
HEADER_INLINE = ("nexg_sparse_decode", "nexg_grouped_code", "nexg_grouped_exc_slot", "nexg_offsets32_bases",
                 "nexg_offsets32_bytes")

#: every symbol include/nexg.h declares (tests check the .so exports them)
EXPORTED_SYMBOLS = (
    "nexg_abi_version", "nexg_strerror", "nexg_ctx_create", "nexg_ctx_destroy",
    "nexg_ctx_last_error", "nexg_ctx_cu_count", "nexg_parse_batch", "nexg_checksum_batch", "nexg_decode_options", "nexg_probe_stream",
    "nexg_probe_span_clock", "nexg_probe_latency",
    "nexg_sparse_expand", "nexg_grouped_expand", "nexg_recompute_checksums_batch",
    "nexg_rx_config_default", "nexg_rx_open", "nexg_rx_next_batch", "nexg_rx_stats", "nexg_rx_close",
    "nexg_tpacket3_walk", "nexg_tx_open", "nexg_tx_send_batch", "nexg_tx_close",
    "nexg_build_udp4_batch", "nexg_build_udp4_tuples", "nexg_build_udp6_batch", "nexg_build_tcp_batch",
    "nexg_build_icmp_echo_batch", "nexg_build_arp_batch", "nexg_build_ndp_ns_batch", "nexg_pcap_open", "nexg_pcap_linktype", "nexg_pcap_last_error",
    "nexg_pcap_read_batch", "nexg_pcap_read_raw", "nexg_pcap_map", "nexg_pcap_walk_mapped", "nexg_pcap_set_read_threads", "nexg_pcap_close", "nexg_gen_lengths", "nexg_gen_frames", "nexg_gen_udp4_params",
)
