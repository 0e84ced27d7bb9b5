/*
 * nexg.h — C ABI of the MI355X-native batched packet-dissect + checksum engine.
 *
 * This is the drop-in boundary for nex-packet's per-frame hot path
 * (shellrow/nex, reference mounted at /root/reference). The reference exposes
 * only a Rust API; each entry point below replaces a family of Rust calls that
 * the callers (examples/parse_frame.rs, examples/dump.rs, examples/udp_ping.rs)
 * make one frame at a time:
 *
 *   nexg_parse_batch      <- frame::Frame::try_from_buf / try_from_buf_with_mode
 *                            (nex-packet/src/frame.rs:299, :309) evaluated on N
 *                            frames, fused with the verification checksums
 *                            ipv4::checksum (ipv4.rs:932), udp::checksum
 *                            (udp.rs:443), tcp::checksum (tcp.rs:1207),
 *                            icmp::checksum (icmp.rs:429), icmpv6::checksum
 *                            (icmpv6.rs:589).
 *   nexg_checksum_batch   <- util::checksum (nex-packet/src/util.rs:65) on N
 *                            independent buffers.
 *   nexg_build_udp4_batch <- UdpPacketBuilder::build (builder/udp.rs:67) +
 *                            Ipv4PacketBuilder::to_bytes (builder/ipv4.rs:94,168)
 *                            + EthernetPacketBuilder::to_bytes
 *                            (builder/ethernet.rs:68), the udp_ping.rs:68-109
 *                            composition, on N parameter tuples.
 *   nexg_gen_frames       <- synthetic workload synthesis;
 *                            no reference counterpart (bench/test inputs).
 *
 * Conventions:
 *   - Plain C: no exceptions cross the ABI; every call returns an int status
 *     (NEXG_OK = 0, negative on error) and never aborts.
 *   - All frame / output buffers are DEVICE pointers owned by the caller;
 *     work is enqueued on `stream` (a hipStream_t, NULL = default stream) and
 *     is stream-ordered: the call returns before the kernels finish. Calls
 *     on one context may use different streams: the context's one device
 *     scratch (TwoPass tail sums) is handed between streams with an event.
 *   - One context per device; a context is not thread-safe (the reference's
 *     RawReceiver is likewise single-consumer, nex-datalink/src/lib.rs:363).
 *   - Frame-level parse failures are data, not call errors: they are reported
 *     per frame in the status field (ParseError kinds, parse.rs:51-97).
 */
#ifndef NEXG_H
#define NEXG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NEXG_ABI_VERSION 1

/* ---- call status ------------------------------------------------------ */
enum {
    NEXG_OK = 0,
    NEXG_EINVAL = -1,  /* bad argument (NULL pointer, unsupported layout) */
    NEXG_ENOMEM = -2,  /* host allocation failed                          */
    NEXG_EDEVICE = -3, /* HIP device error / not a gfx950 device          */
    NEXG_ELAUNCH = -4, /* kernel launch failed                            */
    NEXG_ERANGE = -5,  /* BuildError::LengthOverflow (builder/error.rs:8)  */
    NEXG_EPERM = -6,   /* datalink socket: no CAP_NET_RAW                 */
    NEXG_EIO = -7      /* datalink socket / ring system call failed       */
};

/* ---- per-frame status: ParseError kind (parse.rs:51-97) --------------- */
enum {
    NEXG_FRAME_OK = 0,
    NEXG_ERR_BUFFER_TOO_SHORT = 1, /* ParseError::BufferTooShort */
    NEXG_ERR_INVALID_LENGTH = 2,   /* ParseError::InvalidLength  */
    NEXG_ERR_MALFORMED = 3,        /* ParseError::Malformed      */
    NEXG_ERR_TRUNCATED = 4,        /* ParseError::Truncated      */
    NEXG_ERR_BAD_EXTENT = 7        /* caller error: frame extent past data_bytes
                                      or longer than 65535 bytes (no Frame)   */
};

/* ---- ParseOption / ParseMode (frame.rs:47-50, parse.rs:34-46) ---------- */
#define NEXG_PARSE_STRICT 0x1u  /* ParseMode::Strict (default Lenient)        */
#define NEXG_PARSE_FROM_IP 0x2u /* ParseOption.from_ip_packet (ip_offset used) */
/* Extension (Frame itself never unwraps VLAN, Q3): before
 * dispatching on the EtherType, unwrap up to two 802.1Q / 802.1ad / QinQ tags
 * (EtherType 0x8100 / 0x88A8 / 0x9100) as VlanPacket::try_from_buf reads one
 * (vlan.rs:102-127: 2-B TCI, inner EtherType), when all 4 bytes are present.
 * The record's ethertype is the inner one, l3_off moves by 4 per tag, the
 * tags stay readable at frame bytes [12, l3_off - 2); NEXG_L_VLAN is set. */
#define NEXG_PARSE_VLAN 0x4u

typedef struct nexg_parse_option {
    uint32_t flags;     /* NEXG_PARSE_* */
    uint32_t ip_offset; /* ParseOption.offset, used with NEXG_PARSE_FROM_IP */
} nexg_parse_option;

/* ---- per-frame flags word (shared by nexg_desc and nexg_record) --------
 * Layer bits mirror the Option<> structure of frame::Frame (frame.rs:21-60).
 * Checksum bits record the verify semantics DESIGN.md §3 states:
 *   ip ok  := ipv4::checksum(&Ipv4Packet) == header.checksum
 *   l4 ok  := {tcp,udp}::checksum(&pkt,&src,&dst) == header.checksum,
 *             icmp::checksum(&pkt) / icmpv6::checksum(&pkt,&src,&dst) likewise.
 * Bits 24..26 hold the frame status (NEXG_FRAME_OK / NEXG_ERR_*). */
#define NEXG_L_ETHERNET (1u << 0)  /* datalink.ethernet is Some            */
#define NEXG_L_ARP (1u << 1)       /* datalink.arp is Some                 */
#define NEXG_L_IP (1u << 2)        /* frame.ip is Some (maybe all-None)    */
#define NEXG_L_IPV4 (1u << 3)      /* ip.ipv4 is Some                      */
#define NEXG_L_IPV6 (1u << 4)      /* ip.ipv6 is Some                      */
#define NEXG_L_ICMP (1u << 5)      /* ip.icmp is Some                      */
#define NEXG_L_ICMPV6 (1u << 6)    /* ip.icmpv6 is Some                    */
#define NEXG_L_TRANSPORT (1u << 7) /* frame.transport is Some              */
#define NEXG_L_TCP (1u << 8)       /* transport.tcp is Some                */
#define NEXG_L_UDP (1u << 9)       /* transport.udp is Some                */
#define NEXG_C_IP_CHECKED (1u << 10) /* IPv4 header checksum evaluated     */
#define NEXG_C_IP_OK (1u << 11)      /* ... and equals the stored field    */
#define NEXG_C_IP_PANIC (1u << 12)   /* ipv4::checksum would panic (Q17)   */
#define NEXG_C_L4_CHECKED (1u << 13) /* L4 checksum evaluated              */
#define NEXG_C_L4_OK (1u << 14)      /* ... and equals the stored field    */
#define NEXG_L_VLAN (1u << 15)       /* NEXG_PARSE_VLAN unwrapped >= 1 tag  */
#define NEXG_STATUS_SHIFT 24
#define NEXG_STATUS(flags) (((flags) >> NEXG_STATUS_SHIFT) & 0x7u)

/* Compact 8-byte result per frame (out_kind NEXG_OUT_DESC). Together with the
 * frame bytes it determines the whole frame::Frame (nex_amd/frame.py
 * materialises it): header fields sit at fixed offsets of their layer.
 * payload_off/len locate Frame.payload inside the frame; an empty payload is
 * reported as (0, 0). */
typedef struct nexg_desc {
    uint32_t flags;
    uint16_t payload_off;
    uint16_t payload_len;
} nexg_desc;

/* Full decoded record per frame (out_kind NEXG_OUT_RECORD), 64 bytes.
 * Field values are the reference's parsed values (ipv4.rs:510-528,
 * ipv6.rs:259-268, tcp.rs:820-835, udp.rs:227-235, icmp.rs:188-204,
 * arp.rs:340-371). Fields of absent layers are 0.
 *
 * A frame whose status is a ParseError kind carries the error's payload
 * (parse.rs:53-81) and nothing else:
 *   l4_type = NEXG_CTX_* (which reference check failed: its context string)
 *   ip_src  = BufferTooShort.minimum | InvalidLength.value | Truncated.expected
 *   ip_dst  = BufferTooShort.actual  | Truncated.actual       (else 0) */
enum {
    NEXG_CTX_NONE = 0,
    NEXG_CTX_ETHERNET_PACKET = 1,     /* "Ethernet packet"  ethernet.rs:310-316           */
    NEXG_CTX_DUMMY_ETHERNET = 2,      /* "Frame dummy Ethernet classification" frame.rs:585 */
    NEXG_CTX_IPV4_PACKET = 3,         /* "IPv4 packet"  BufferTooShort ipv4.rs:380-386,
                                         Truncated (strict) ipv4.rs:429-435                */
    NEXG_CTX_IPV4_VERSION = 4,        /* "IPv4 packet version"  ipv4.rs:388-393           */
    NEXG_CTX_IPV4_HEADER_LENGTH = 5,  /* "IPv4 header length"  ipv4.rs:395-401            */
    NEXG_CTX_IPV4_HEADER = 6,         /* "IPv4 header"  ipv4.rs:403-410                   */
    NEXG_CTX_IPV4_TOTAL_LENGTH = 7,   /* "IPv4 total length" (value = declared) 421-427   */
    NEXG_CTX_IPV4_OPTIONS = 8,        /* "IPv4 options" (strict)  ipv4.rs:476-481          */
    NEXG_CTX_IPV4_OPTION_LENGTH = 9,  /* "IPv4 option length" (strict)  ipv4.rs:485-491    */
    NEXG_CTX_IPV6_PACKET = 10,        /* "IPv6 packet"  ipv6.rs:225-231                   */
    NEXG_CTX_IPV6_VERSION = 11,       /* "IPv6 packet version"  ipv6.rs:235-239           */
    NEXG_CTX_IPV6_PAYLOAD = 12,       /* "IPv6 payload" (strict)  ipv6.rs:271-277          */
    NEXG_CTX_IPV6_EXTENSION = 13,     /* "IPv6 extension header"  ipv6.rs:288-308         */
    NEXG_CTX_IPV6_ROUTING = 14,       /* "IPv6 routing header"  ipv6.rs:319-335           */
    NEXG_CTX_IPV6_FRAGMENT = 15       /* "IPv6 fragment header"  ipv6.rs:346-352          */
};
typedef struct nexg_record {
    uint32_t flags;          /* as nexg_desc.flags                              */
    uint16_t payload_off;    /* Frame.payload offset in the frame               */
    uint16_t payload_len;    /* Frame.payload length                            */
    uint16_t packet_len;     /* Frame.packet_len (frame.rs:575)                 */
    uint16_t ethertype;      /* EtherType value (dummy value when FROM_IP)      */
    uint16_t l3_off;         /* offset of the IP / ARP header                   */
    uint16_t l4_off;         /* offset of the TCP/UDP/ICMP header (0 if none)   */
    uint8_t ip_ver_ihl;      /* v4: version<<4|ihl  v6: version<<4  arp: hlen    */
    uint8_t ip_tos;          /* v4: dscp<<2|ecn     v6: traffic_class arp: plen  */
    uint16_t ip_length;      /* v4: total_length (effective, Q5) v6: payload_length */
    uint32_t ip_word;        /* v4: identification<<16 | flags<<13 | frag_off    */
                             /* v6: flow_label                                   */
    uint8_t ip_ttl;          /* v4: ttl   v6: hop_limit                          */
    uint8_t ip_proto;        /* IpNextProtocol::value() of v4 proto / v6 nh (Q8) */
    uint8_t ip_nopt;         /* v4: options.len()  v6: extensions.len()          */
    uint8_t l4_nopt;         /* tcp: options.len()                               */
    uint32_t ip_src;         /* v4 / arp sender proto addr, as a BE u32 value   */
    uint32_t ip_dst;         /* v4 / arp target proto addr                       */
    uint16_t ip_csum;        /* v4 header checksum field                         */
    uint16_t ip_csum_calc;   /* ipv4::checksum(&pkt) (0 if not evaluated)        */
    uint16_t l4_csum;        /* tcp/udp/icmp/icmpv6 checksum field               */
    uint16_t l4_csum_calc;   /* reference checksum of the L4 packet              */
    uint16_t src_port;       /* tcp/udp source      arp: hardware_type           */
    uint16_t dst_port;       /* tcp/udp destination arp: protocol_type           */
    uint16_t l4_length;      /* udp: length  tcp: data_offset*4  arp: operation  */
    uint8_t l4_type;         /* icmp(v6) type   tcp: flags                       */
    uint8_t l4_code;         /* icmp(v6) code   tcp: data_offset<<4|reserved     */
    uint32_t tcp_seq;
    uint32_t tcp_ack;
    uint16_t tcp_window;
    uint16_t tcp_urg;
} nexg_record;

#define NEXG_OUT_DESC 1
#define NEXG_OUT_RECORD 2
#define NEXG_OUT_SLICE 3
/* Flags-only result per frame (out_kind NEXG_OUT_FLAGS), 4 bytes: exactly
 * nexg_desc.flags (layer presence, checksum verdicts, status) without the
 * payload location — for consumers that only classify and verify. On HBM the
 * 8-B descriptor stream costs ~18 % of the read rate at 64-B frames; 4 B
 * halves that. */
#define NEXG_OUT_FLAGS 4
/* Verdict per frame (out_kind NEXG_OUT_VERDICT), 2 bytes, lossless for the
 * flags word: a parsed frame stores flags & 0xFFFF (layer and checksum bits;
 * bits 16..23 are never set), a frame with a nonzero status (no layers) stores
 * NEXG_VERDICT_ERR | status << 3. NEXG_L_ARP together with NEXG_L_IP marks it:
 * a Frame never holds both datalink.arp and ip (frame.rs:596-607). Output
 * alignment 2 B. Explicit-length batches (TwoPass layout) run the lane-window
 * kernel for this output. */
#define NEXG_OUT_VERDICT 5
#define NEXG_VERDICT_ERR (NEXG_L_ARP | NEXG_L_IP)
#define NEXG_VERDICT_FLAGS(v)                                                        \
    ((((v) & NEXG_VERDICT_ERR) == NEXG_VERDICT_ERR) ? ((((uint32_t)(v) >> 3) & 0x7u) \
                                                       << NEXG_STATUS_SHIFT)         \
                                                    : (uint32_t)(v))

/* Sparse descriptors (out_kind NEXG_OUT_SPARSE): lossless for nexg_desc at
 * 1 B per frame whenever the frame has one of the canonical shapes below
 * (every frame of the synthetic 64-B and IMIX workloads does), plus the full
 * 8-B descriptor for every other frame. `out` (16-B aligned) holds
 *   codes : uint8_t[count]                 at out
 *   exc   : nexg_desc[count] (capacity)    at out + NEXG_SPARSE_EXC_OFFSET(count)
 * The k-th exception (code 0) of the 64-frame group g = i / 64, counted in
 * frame order, is stored at exc[64 * g + k]; nothing else of exc is written.
 * Code byte: bits 0..3 shape, bit 4 NEXG_C_IP_OK, bit 5 NEXG_C_L4_OK, bits
 * 6..7 number of VLAN tags unwrapped (NEXG_PARSE_VLAN). With L = l3 offset
 * = (FROM_IP ? ip_offset : 14) + 4 * tags, h = L + NEXG_SHAPE_HDR(shape):
 *   flags       = NEXG_SHAPE_FLAGS(shape) | ok bits | (tags ? NEXG_L_VLAN : 0)
 *   payload_len = len - h, payload_off = payload_len ? h : 0
 * for shapes 1..9; shape 10 (IP layer present but all None, Q4/Q12) has an
 * empty payload; shapes 11..15 are error statuses 1..4, 7 (no layers, empty
 * payload). The device encoder stores a code only when this decodes to the
 * frame's exact descriptor, so the output is lossless by construction;
 * nexg_sparse_expand (below) or nexg_sparse_decode restores nexg_desc. */
#define NEXG_OUT_SPARSE 6
#define NEXG_SPARSE_EXC_OFFSET(count) ((((uint64_t)(count)) + 15u) & ~(uint64_t)15u)
#define NEXG_SPARSE_BYTES(count) (NEXG_SPARSE_EXC_OFFSET(count) + 8u * (uint64_t)(count))
#define NEXG_SPARSE_IP_OK 0x10u
#define NEXG_SPARSE_L4_OK 0x20u
#define NEXG_SPARSE_TAG_SHIFT 6
enum {
    NEXG_SHAPE_EXCEPTION = 0,
    NEXG_SHAPE_V4_UDP = 1,   /* IPv4 IHL 5 + UDP, datagram to the frame end   */
    NEXG_SHAPE_V4_TCP = 2,   /* IPv4 IHL 5 + TCP data offset 5                */
    NEXG_SHAPE_V4_ICMP = 3,  /* IPv4 IHL 5 + ICMP                             */
    NEXG_SHAPE_V6_UDP = 4,   /* IPv6 without extensions + UDP                 */
    NEXG_SHAPE_V6_TCP = 5,   /* IPv6 + TCP data offset 5                      */
    NEXG_SHAPE_V6_ICMP = 6,  /* IPv6 + ICMPv6                                 */
    NEXG_SHAPE_ETH_ONLY = 7, /* EtherType not IPv4/IPv6/ARP (Q3)              */
    NEXG_SHAPE_V4_OTHER = 8, /* IPv4 IHL 5, no L4 layer (Q9, Q15)             */
    NEXG_SHAPE_V6_OTHER = 9, /* IPv6 without extensions, no L4 layer          */
    NEXG_SHAPE_IP_NONE = 10, /* ip = Some(all None), payload empty (Q4, Q12)  */
    NEXG_SHAPE_ERR_FIRST = 11 /* 11..14 = status 1..4, 15 = NEXG_ERR_BAD_EXTENT */
};
#define NEXG_SHAPE_V4_ (NEXG_L_ETHERNET | NEXG_L_IP | NEXG_L_IPV4 | NEXG_C_IP_CHECKED)
#define NEXG_SHAPE_V6_ (NEXG_L_ETHERNET | NEXG_L_IP | NEXG_L_IPV6)
#define NEXG_SHAPE_FLAGS(s)                                                                     \
    ((s) == 1 ? NEXG_SHAPE_V4_ | NEXG_L_TRANSPORT | NEXG_L_UDP | NEXG_C_L4_CHECKED            \
   : (s) == 2 ? NEXG_SHAPE_V4_ | NEXG_L_TRANSPORT | NEXG_L_TCP | NEXG_C_L4_CHECKED            \
   : (s) == 3 ? NEXG_SHAPE_V4_ | NEXG_L_ICMP | NEXG_C_L4_CHECKED                              \
   : (s) == 4 ? NEXG_SHAPE_V6_ | NEXG_L_TRANSPORT | NEXG_L_UDP | NEXG_C_L4_CHECKED            \
   : (s) == 5 ? NEXG_SHAPE_V6_ | NEXG_L_TRANSPORT | NEXG_L_TCP | NEXG_C_L4_CHECKED            \
   : (s) == 6 ? NEXG_SHAPE_V6_ | NEXG_L_ICMPV6 | NEXG_C_L4_CHECKED                            \
   : (s) == 7 ? NEXG_L_ETHERNET                                                               \
   : (s) == 8 ? NEXG_SHAPE_V4_                                                                \
   : (s) == 9 ? NEXG_SHAPE_V6_                                                                \
   : (s) == 10 ? NEXG_L_ETHERNET | NEXG_L_IP                                                  \
   : (s) >= 11 && (s) <= 14 ? (uint32_t)((s) - 10) << NEXG_STATUS_SHIFT                       \
   : (s) == 15 ? (uint32_t)NEXG_ERR_BAD_EXTENT << NEXG_STATUS_SHIFT : 0u)
/* bytes from the l3 offset to the payload: IP header + L4 header */
#define NEXG_SHAPE_HDR(s)                                                                       \
    ((s) == 1 ? 28u : (s) == 2 ? 40u : (s) == 3 ? 24u : (s) == 4 ? 48u : (s) == 5 ? 60u       \
   : (s) == 6 ? 44u : (s) == 8 ? 20u : (s) == 9 ? 40u : 0u)

/* nexg_desc of a frame from its sparse code (host side; the device encoder
 * uses the same table). len = the frame's length, flags/ip_offset = the
 * batch's parse option. Returns 0 for an exception code (look the descriptor
 * up in exc), 1 otherwise. */
static inline int nexg_sparse_decode(uint8_t code, uint32_t len, uint32_t parse_flags,
                                     uint32_t ip_offset, nexg_desc* d) {
    const uint32_t shape = code & 0xFu, tags = (uint32_t)code >> NEXG_SPARSE_TAG_SHIFT;
    if (shape == NEXG_SHAPE_EXCEPTION) return 0;
    d->flags = NEXG_SHAPE_FLAGS(shape);
    d->payload_off = 0;
    d->payload_len = 0;
    if (shape >= NEXG_SHAPE_IP_NONE) {
        if (shape == NEXG_SHAPE_IP_NONE && tags) d->flags |= NEXG_L_VLAN;
        return 1;
    }
    d->flags |= ((code & NEXG_SPARSE_IP_OK) ? NEXG_C_IP_OK : 0u) | ((code & NEXG_SPARSE_L4_OK) ? NEXG_C_L4_OK : 0u) |
                (tags ? NEXG_L_VLAN : 0u);
    const uint32_t h = ((parse_flags & NEXG_PARSE_FROM_IP) ? ip_offset : 14u) + 4u * tags + NEXG_SHAPE_HDR(shape);
    d->payload_len = (uint16_t)(len - h);
    d->payload_off = (uint16_t)(len > h ? h : 0u);
    return 1;
}

/* Grouped sparse descriptors (out_kind NEXG_OUT_GROUPED): NEXG_OUT_SPARSE's
 * codes with the common part of each 64-frame group g = i / 64 stored once.
 * A group whose frames all share one non-exception code up to its two
 * verdict bits is "uniform": heads[g] = that code with bits 4..5 clear, and
 * its verdicts are two 64-bit masks (bit i % 64 = NEXG_SPARSE_IP_OK /
 * NEXG_SPARSE_L4_OK of frame i); nothing else of the group is written
 * (17 B per 64 frames on single-shape traffic). Any other group is mixed and
 * stores its 1-B codes and exceptions as NEXG_OUT_SPARSE does, with heads[g]
 * = 0; or heads[g] = NEXG_GROUPED_TILE_RUN (the packed-batch kernel's form):
 * then the exceptions of its 256-frame tile T = i / 256 sit in one run, frame
 * i's at exc[256 T + k], k = the code-0 frames of [256 T, i) (one write burst
 * per tile instead of one per group: DESIGN.md §6 round 6). Every
 * area is written densely (a head byte per group, 16 B of masks per group):
 * interleaving them with the codes costs partial-line writes.
 * `out` (16-B aligned) holds
 *   heads : uint8_t[G]                     at out            (G = groups)
 *   masks : uint32_t[G][4] {ip lo, ip hi, l4 lo, l4 hi} at out + NEXG_GROUPED_MASK_OFFSET(count)
 *   codes : uint8_t[count]                 at out + NEXG_GROUPED_CODE_OFFSET(count)
 *   exc   : nexg_desc[count] (capacity)    at out + NEXG_GROUPED_EXC_OFFSET(count)
 * nexg_grouped_code gives frame i's NEXG_OUT_SPARSE code (then
 * nexg_sparse_decode), nexg_grouped_exc_slot the exc index of a code-0
 * frame; nexg_grouped_expand restores nexg_desc[count] on the device. */
#define NEXG_OUT_GROUPED 7
#define NEXG_GROUPED_GROUPS(count) ((((uint64_t)(count)) + 63u) >> 6)
#define NEXG_GROUPED_MASK_OFFSET(count) ((NEXG_GROUPED_GROUPS(count) + 15u) & ~(uint64_t)15u)
#define NEXG_GROUPED_CODE_OFFSET(count) (NEXG_GROUPED_MASK_OFFSET(count) + 16u * NEXG_GROUPED_GROUPS(count))
#define NEXG_GROUPED_EXC_OFFSET(count) ((NEXG_GROUPED_CODE_OFFSET(count) + (uint64_t)(count) + 15u) & ~(uint64_t)15u)
#define NEXG_GROUPED_BYTES(count) (NEXG_GROUPED_EXC_OFFSET(count) + 8u * (uint64_t)(count))
/* head of a mixed group whose exceptions are kept per 256-frame tile (its
 * shape bits are 0, so it is never a uniform group's head) */
#define NEXG_GROUPED_TILE_RUN 0x80u

/* frame i's NEXG_OUT_SPARSE code from a NEXG_OUT_GROUPED output (host side) */
static inline uint8_t nexg_grouped_code(const void* out, uint64_t count, uint64_t i) {
    const uint8_t* o = (const uint8_t*)out;
    const uint64_t g = i >> 6;
    const uint8_t head = o[g];
    if (!head || head == NEXG_GROUPED_TILE_RUN) return o[NEXG_GROUPED_CODE_OFFSET(count) + i];
    const uint8_t* m = o + NEXG_GROUPED_MASK_OFFSET(count) + 16u * g;
    /* the masks are little-endian words: bit b of a 64-bit mask is bit b % 8
     * of its byte b / 8 */
    const uint32_t b = (uint32_t)(i & 63u), byte = b >> 3, sh = b & 7u;
    const uint32_t ip = (m[byte] >> sh) & 1u, l4 = (m[8u + byte] >> sh) & 1u;
    return (uint8_t)(head | (ip ? NEXG_SPARSE_IP_OK : 0u) | (l4 ? NEXG_SPARSE_L4_OK : 0u));
}

/* index in the exc area of frame i's descriptor when its code is 0 (host
 * side): its group's run (heads[g] = 0) or its tile's (NEXG_GROUPED_TILE_RUN) */
static inline uint64_t nexg_grouped_exc_slot(const void* out, uint64_t count, uint64_t i) {
    const uint8_t* o = (const uint8_t*)out;
    const uint64_t first = o[i >> 6] == NEXG_GROUPED_TILE_RUN ? (i & ~(uint64_t)255u) : (i & ~(uint64_t)63u);
    uint64_t k = 0;
    for (uint64_t j = first; j < i; j++) k += nexg_grouped_code(out, count, j) == 0u;
    return first + k;
}

/* FrameSlice::try_from_buf (frame.rs:84-287) per frame, out_kind
 * NEXG_OUT_SLICE, 16 bytes: layer boundaries only, no checksums. FrameSlice
 * has no ParseMode (NEXG_PARSE_STRICT is ignored) and reports every inner
 * failure as an error; its walk differs from Frame's (AH is walked, ICMP
 * needs 4 B, UDP length is not checked). Ranges are frame-relative:
 *   datalink  = [0, 14)                          if NEXG_S_DATALINK
 *   network   = [l3_off, l3_off + l3_len)        if NEXG_S_NETWORK
 *   transport = [l3_off + l3_len, + l4_len)      if NEXG_S_TRANSPORT
 *   payload   = [payload_off, payload_off + payload_len)  (on success)
 * ethertype = EtherType::value(), ip_protocol (bits 8..15) =
 * IpNextProtocol::value() (143..252 -> 255). Status bits 24..26 as for
 * Frame: BufferTooShort / InvalidLength / Malformed / Truncated / BAD_EXTENT. */
#define NEXG_S_DATALINK (1u << 0)
#define NEXG_S_NETWORK (1u << 1)
#define NEXG_S_TRANSPORT (1u << 2)
#define NEXG_S_ETHERTYPE (1u << 3)
#define NEXG_S_IP_PROTOCOL (1u << 4)
#define NEXG_S_PROTO_SHIFT 8
typedef struct nexg_slice {
    uint32_t flags;
    uint16_t l3_off, l3_len, l4_len;
    uint16_t payload_off, payload_len;
    uint16_t ethertype;
} nexg_slice;

/* ---- frame batch layout ------------------------------------------------
 * Frame i occupies data[off(i), off(i)+len(i)):
 *   offsets == NULL : off(i) = i*stride
 *   offsets != NULL : off(i) = offsets[i]
 *   lengths != NULL : len(i) = lengths[i]
 *   lengths == NULL : len(i) = stride (offsets == NULL)
 *                     or offsets[i+1]-offsets[i] (offsets has count+1 entries)
 * Every len(i) must be <= 65535 (frames are at most one IPv4 datagram; the
 * reference's default read buffer is 4096, nex-datalink/src/lib.rs:229).
 * data_bytes bounds every frame extent: a frame reaching past data+data_bytes
 * gets NEXG_ERR_BAD_EXTENT. Device loads are whole 16-B aligned blocks: the
 * kernels read only inside the 16-B aligned blocks that overlap
 * [data, data + data_bytes) (bytes of those blocks outside the range may be
 * read and are ignored; such a block cannot cross a page, so this never
 * faults). All pointers are device pointers.
 *
 * hints: NEXG_FRAMES_MONOTONE (offsets + lengths layouts) promises that
 * offsets are nondecreasing and frames do not overlap, with small gaps
 * between consecutive frames (e.g. the 16-B record headers a capture file
 * keeps in place, nexg_pcap_read_raw). Such batches are streamed as
 * contiguous spans (gap bytes are read and ignored) instead of by the
 * two-pass explicit-length kernels. The kernels verify the promise per
 * 256-frame group and fall back to per-frame reads where it fails, so a
 * wrong hint costs speed, never correctness. */
#define NEXG_FRAMES_MONOTONE 0x1u
/* NEXG_FRAMES_OFFSETS32: `offsets` points to uint32_t entries (4 bytes per
 * frame instead of 8; any 4-B aligned address). offsets32[i] is offset(i)
 * modulo 2^32. When data_bytes > 0xFFFFFFFF the table is followed, at the
 * first 8-B aligned address past its count + 1 entries, by one uint64_t per
 * 256 frames, base[k] = offset(256 k) in full (nexg_offsets32_bases), and
 * offset(i) = base[i / 256] + (uint32_t)(offsets32[i] - (uint32_t)base[i / 256]):
 * every frame (and, packed, the end of its group) lies within 4 GiB after
 * its group's first frame, which packed and monotone batches satisfy by
 * construction. nexg_offsets32_bytes gives the whole table's size. */
#define NEXG_FRAMES_OFFSETS32 0x2u
typedef struct nexg_frames {
    const uint8_t* data;
    uint64_t data_bytes;
    const uint64_t* offsets;
    const uint32_t* lengths;
    uint32_t stride;
    uint32_t hints; /* NEXG_FRAMES_* */
    uint64_t count;
} nexg_frames;

/* NEXG_FRAMES_OFFSETS32 table of `count` frames: count + 1 uint32 entries,
 * then (for batches over 4 GiB) ceil((count + 1) / 256) uint64 group bases
 * at the next 8-B boundary. */
static inline const uint64_t* nexg_offsets32_bases(const void* table, uint64_t count) {
    const uintptr_t end = (uintptr_t)table + 4u * (uintptr_t)(count + 1u);
    return (const uint64_t*)((end + 7u) & ~(uintptr_t)7u);
}
static inline uint64_t nexg_offsets32_bytes(uint64_t count, int with_bases) {
    const uint64_t b = (4u * (count + 1u) + 7u) & ~(uint64_t)7u;
    return with_bases ? b + 8u * ((count + 1u + 255u) / 256u) : 4u * (count + 1u);
}

/* ---- context ----------------------------------------------------------- */
typedef struct nexg_ctx nexg_ctx;

int nexg_abi_version(void);
const char* nexg_strerror(int status);
/* Binds `device` (HIP ordinal); fails with NEXG_EDEVICE unless it is gfx950. */
int nexg_ctx_create(int device, nexg_ctx** out);
int nexg_ctx_destroy(nexg_ctx* ctx);
/* Message of the last failing call on ctx ("" if none). */
const char* nexg_ctx_last_error(const nexg_ctx* ctx);
/* Number of compute units of the bound device (for grid sizing by callers). */
int nexg_ctx_cu_count(const nexg_ctx* ctx);

/* ---- hot path ----------------------------------------------------------
 * Frame::try_from_buf_with_mode on every frame + checksum verification.
 * out_kind NEXG_OUT_DESC   -> out is nexg_desc[count]
 * out_kind NEXG_OUT_RECORD -> out is nexg_record[count]
 * out_kind NEXG_OUT_SLICE  -> out is nexg_slice[count] (FrameSlice, above) */
int nexg_parse_batch(nexg_ctx* ctx, const nexg_frames* frames,
                     const nexg_parse_option* option, int out_kind, void* out,
                     void* stream);

/* util::checksum(buf_i, skipword) for every buffer (util.rs:65-78). */
int nexg_checksum_batch(nexg_ctx* ctx, const nexg_frames* bufs,
                        uint32_t skipword, uint16_t* out, void* stream);

/* nexg_desc[count] from a NEXG_OUT_SPARSE result of the same batch and parse
 * option (codes + exceptions, layout above). Stream-ordered, device pointers. */
int nexg_sparse_expand(nexg_ctx* ctx, const nexg_frames* frames, const nexg_parse_option* option,
                       const void* sparse, nexg_desc* out, void* stream);
/* The same from a NEXG_OUT_GROUPED result. */
int nexg_grouped_expand(nexg_ctx* ctx, const nexg_frames* frames, const nexg_parse_option* option,
                        const void* grouped, nexg_desc* out, void* stream);

/* ---- in-place checksum fix-up (mutable views) -------------
 * Rewrites checksum fields inside the frames, with the raw-buffer semantics
 * of the reference's mutable views, composed the way
 * examples/mutable_chaining.rs:19-63 chains them (payload_mut of each layer
 * is the buffer of the next):
 *   MutableEthernetPacket (>= 14 B; payload = bytes after 14)
 *   EtherType 0x0800 -> MutableIpv4Packet::new (ipv4.rs:540-566: >= 20 B,
 *     IHL >= 5, IHL*4 <= len, total 0 or >= IHL*4); recompute_checksum
 *     (ipv4.rs:669-679: util::checksum(raw[..header_len], 5) into bytes
 *     10..11); payload_mut = [hl, hl + total_len - hl) with total_len = 0 ->
 *     len, else min(total, len) (ipv4.rs:591-596, 697-704)
 *   EtherType 0x86DD -> MutableIpv6Packet::new (>= 40 B); payload_mut =
 *     every byte after 40 (ipv6.rs:423-426; extension headers not walked)
 *   protocol / next header (raw byte) 17 -> MutableUdpPacket::new (udp.rs:
 *     101-121) + recompute_checksum with the enclosing IP addresses as
 *     context (udp.rs:338-369: pseudo-header sum over the WHOLE payload_mut
 *     slice, skipword 3, into bytes 6..7); 6 -> MutableTcpPacket (tcp.rs:
 *     857-876, 1009-1040, skipword 8, bytes 16..17); 1 (IPv4 only) ->
 *     MutableIcmpPacket (icmp.rs:267-273 via IcmpPacket::from_buf, >= 8 B;
 *     icmp.rs:372-377 util::checksum(raw, 1), bytes 2..3); 58 (IPv6 only) ->
 *     MutableIcmpv6Packet (icmpv6.rs:316-322, 450-470).
 * A view whose constructor returns None is skipped. `which` selects
 * NEXG_FIX_IP and/or NEXG_FIX_L4. With parse flag NEXG_PARSE_FROM_IP the IP
 * header starts at ip_offset and the version nibble picks the family.
 * The bytes of frames->data are rewritten in place (the batch's data must be
 * writable device memory; frames must not overlap). out (optional, may be
 * NULL): nexg_fixup[count]. */
#define NEXG_FIX_IP 0x1u
#define NEXG_FIX_L4 0x2u
typedef struct nexg_fixup {
    uint8_t done;   /* NEXG_FIX_* bits of the fields written                 */
    uint8_t proto;  /* L4 protocol number whose view was built (0 if none)  */
    uint16_t ip_csum; /* value written at IPv4 bytes 10..11 (if NEXG_FIX_IP) */
    uint16_t l4_csum; /* value written into the L4 header (if NEXG_FIX_L4)   */
    uint16_t l4_off;  /* frame offset of the L4 header                       */
} nexg_fixup;
int nexg_recompute_checksums_batch(nexg_ctx* ctx, const nexg_frames* frames,
                                   const nexg_parse_option* option, uint32_t which,
                                   nexg_fixup* out, void* stream);

/* ---- option lists ---------------------------------------
 * The Vec fields of Frame's headers, decoded on the device into fixed-capacity
 * arrays: Ipv4Header.options (ipv4.rs:442-508: EOL is kept and ends the list,
 * NOP is kept, an option without room for its length / with length < 2 / past
 * the header ends the walk) and TcpHeader.options (tcp.rs:767-818). Option k
 * starts at frame byte ip_opt_off + ip_pos[k] (tcp_opt_off + tcp_pos[k]); its
 * type/kind is that byte; EOL and NOP (IPv4: number = byte & 0x1f in {0, 1};
 * TCP: kind in {0, 1}) are one byte long, every other option's length is the
 * next byte and its data the length - 2 bytes after that. Counts are 0 for an
 * absent header (nexg_record flags); they equal the record's ip_nopt /
 * l4_nopt. An options area is at most 40 bytes, so 40 entries always suffice. */
typedef struct nexg_options {
    uint8_t n_ip;          /* Ipv4Header.options.len()                       */
    uint8_t n_tcp;         /* TcpHeader.options.len()                        */
    uint16_t ip_opt_off;   /* frame offset of the IPv4 options (l3_off + 20) */
    uint16_t tcp_opt_off;  /* frame offset of the TCP options (l4_off + 20)  */
    uint16_t reserved;
    uint8_t ip_pos[40];
    uint8_t tcp_pos[40];
    uint8_t pad[8];
} nexg_options;

/* Option lists for a batch already parsed with NEXG_OUT_RECORD (any parse
 * mode): records[i] must be frame i's record. Device pointers, stream-ordered. */
int nexg_decode_options(nexg_ctx* ctx, const nexg_frames* frames, const nexg_record* records,
                        nexg_options* out, void* stream);

/* ---- calibration (not a reference entry point) ---------------------------
 * The HBM stream ceilings the parse kernels are measured against, on the
 * caller's own buffer and box: `bytes` (a multiple of 16384) read with the
 * parse kernels' load shape (16-B non-temporal loads, 16-KiB tile per
 * 256-lane workgroup). out_per_64 = 8: for every 64 B read, 8 B written
 * (the nexg_desc stream shape): out[i] = {x, i} with x the XOR of the four
 * 16-B chunks lane i % 256 of tile i / 256 loaded (chunks i%256 + 256k).
 * out_per_64 = 9: the same stream capped at the fixed-stride parse kernel's
 * occupancy (6 workgroups per CU, by dynamic LDS; 8 runs 8 per CU).
 * out_per_64 = 0: read only; out[tile] = XOR of the tile's dwords (4 B per
 * 16 KiB). bench.py reports the headline kernel against both.
 * out_per_64 = 64: write only (the builders' copy-out shape: 16-B
 * non-temporal stores, 16 KiB per workgroup); `data` is not read (may be
 * NULL), `out` (16-B aligned) receives `bytes` bytes: dwords {tile, chunk, 0, 0}
 * per 16-B chunk. bench.py reports the serialize path against it. */
int nexg_probe_stream(nexg_ctx* ctx, const void* data, uint64_t bytes, uint32_t out_per_64,
                      void* out, void* stream);

/* Calibration (not a reference entry point): the clock a parse of this batch
 * runs at. Runs the span kernel that nexg_parse_batch runs for the batch
 * (packed layouts and monotone capture records; NEXG_EINVAL for any other
 * layout) with NEXG_OUT_GROUPED into `out` (NEXG_GROUPED_BYTES(count),
 * 16-B aligned: the same bytes nexg_parse_batch writes), in an
 * instance that also stores 8 u64 per 256-frame workgroup into `stamps`
 * (device, ceil(count / 256) * 8 entries, 8-B aligned): s_memtime (shader
 * clock ticks of the workgroup's XCD) at [0] entry, [1] after the span check,
 * [2] after the sub-tile loop, [3] after the fast path, [4] after the generic
 * section, [5] exit; s_memrealtime (100 MHz) at [6] entry and [7] exit. A
 * workgroup's clock is ([5] - [0]) / ([7] - [6]) x 100 MHz. The product
 * kernels contain no stamp. */
int nexg_probe_span_clock(nexg_ctx* ctx, const nexg_frames* frames, const nexg_parse_option* option,
                          void* out, uint64_t* stamps, void* stream);

/* Calibration (not a reference entry point): dependent HBM load latency.
 * Writes a ring into `buf` (device, `bytes` >= 4 MiB, 16-B aligned; 64-B
 * line i holds the index of line (i + 16411) mod (bytes / 64)) and has one lane
 * chase it for `steps` (1..2^20) dependent loads from line `start`, alone
 * (loaded = 0) or while 4 workgroups per CU stream-read the buffer (loaded =
 * 1: the conditions of a parse kernel's dependent loads). out (device, 4 u64,
 * 8-B aligned): [0] shader-clock ticks and [1] 100-MHz ticks over the chain;
 * per step = [1] / steps x 10 ns. The App. C mix's generic section waits on
 * such loads. */
int nexg_probe_latency(nexg_ctx* ctx, void* buf, uint64_t bytes, uint32_t steps, uint32_t start, uint32_t loaded,
                       uint64_t* out, void* stream);

/* ---- serialize path (udp_ping.rs:68-109 shape) -------------------------- */
typedef struct nexg_udp4_build {
    const uint32_t* src_ip;   /* per frame, IPv4 address as BE u32 value, or
                                 NULL -> def_src_ip (udp_ping: one source)   */
    const uint32_t* dst_ip;   /* per frame                                    */
    const uint16_t* src_port; /* per frame, or NULL -> def_src_port           */
    const uint16_t* dst_port; /* per frame, or NULL -> def_dst_port           */
    const uint16_t* ip_id;    /* per frame, or NULL -> def_ip_id              */
    const uint8_t* src_mac;   /* 6 bytes per frame, or NULL -> def_src_mac    */
    const uint8_t* dst_mac;   /* 6 bytes per frame, or NULL -> def_dst_mac    */
    const uint8_t* payload;   /* UDP payload shared by all frames (may be NULL) */
    uint32_t payload_len;
    uint16_t def_src_port, def_dst_port, def_ip_id;
    uint8_t def_src_mac[6], def_dst_mac[6];
    uint8_t ttl;      /* Ipv4PacketBuilder default 64 (builder/ipv4.rs:37)   */
    uint8_t ip_flags; /* 3-bit flags; udp_ping uses DontFragment = 0b010     */
    uint8_t dscp_ecn; /* dscp<<2|ecn, builder default 0                      */
    uint8_t reserved;
    uint32_t def_src_ip; /* source when src_ip is NULL (BE u32 value); sits in
                            what was padding, so the struct is unchanged in size */
    uint64_t count;
} nexg_udp4_build;

/* Writes frame i (42 + payload_len bytes) at out + i*out_stride.
 * NEXG_ERANGE if 28 + payload_len > 65535 (builder/udp.rs:83, ipv4.rs:153). */
int nexg_build_udp4_batch(nexg_ctx* ctx, const nexg_udp4_build* params,
                          uint8_t* out, uint32_t out_stride, void* stream);

/* The same build with each frame's tuple as one 16-B record (array of
 * structs, 16-B aligned): one 16-B load per frame instead of five arrays.
 * Ports and id are u16 values, addresses BE u32 values as above. */
typedef struct nexg_udp4_tuple {
    uint32_t src_ip, dst_ip;
    uint16_t src_port, dst_port;
    uint16_t ip_id, reserved;
} nexg_udp4_tuple;

/* nexg_build_udp4_batch with frame i's src_ip / dst_ip / src_port / dst_port /
 * ip_id from tuples[i] (params->count tuples); MACs, ttl, flags, dscp_ecn and
 * payload from params, whose per-frame arrays must all be NULL (NEXG_EINVAL
 * otherwise, or when tuples is NULL or not 16-B aligned). Same bytes as
 * nexg_build_udp4_batch on the same values. */
int nexg_build_udp4_tuples(nexg_ctx* ctx, const nexg_udp4_build* params, const nexg_udp4_tuple* tuples,
                           uint8_t* out, uint32_t out_stride, void* stream);

/* ---- udp_ping IPv6 branch (examples/udp_ping.rs:83-89) ---------------------
 * UdpPacketBuilder::build over IPv6 (builder/udp.rs:67-95; checksum =
 * udp::ipv6_checksum, udp.rs:480-505) -> Ipv6PacketBuilder::to_bytes
 * (builder/ipv6.rs:89-152; Ipv6Packet::to_bytes ipv6.rs:50-75) ->
 * EthernetPacketBuilder (EtherType 0x86DD). Frame = 62 + payload_len bytes. */
typedef struct nexg_udp6_build {
    const uint8_t* src_ip;    /* 16 bytes per frame, network order            */
    const uint8_t* dst_ip;    /* 16 bytes per frame                           */
    const uint16_t* src_port; /* per frame, or NULL -> def_src_port           */
    const uint16_t* dst_port; /* per frame, or NULL -> def_dst_port           */
    const uint8_t* src_mac;   /* 6 bytes per frame, or NULL -> def_src_mac    */
    const uint8_t* dst_mac;   /* 6 bytes per frame, or NULL -> def_dst_mac    */
    const uint8_t* payload;   /* UDP payload shared by all frames (may be NULL) */
    uint32_t payload_len;
    uint32_t flow_label;      /* low 20 bits (Ipv6PacketBuilder::flow_label masks) */
    uint16_t def_src_port, def_dst_port;
    uint8_t def_src_mac[6], def_dst_mac[6];
    uint8_t hop_limit;        /* Ipv6PacketBuilder default 64 (builder/ipv6.rs:33) */
    uint8_t traffic_class;    /* builder default 0                            */
    uint8_t src_shared;       /* 1: src_ip holds ONE address, the source of every
                                 frame (udp_ping's probe batch: one interface
                                 address, a destination per frame)            */
    uint8_t reserved;
    uint64_t count;
} nexg_udp6_build;

/* Writes frame i (62 + payload_len bytes) at out + i*out_stride.
 * NEXG_ERANGE if 8 + payload_len > 65535 (builder/udp.rs:83, builder/ipv6.rs:137).
 * With src_shared and every other per-frame array NULL (the probe batch) the
 * kernel reads 16 B per frame (dst_ip) and nothing else. */
int nexg_build_udp6_batch(nexg_ctx* ctx, const nexg_udp6_build* params,
                          uint8_t* out, uint32_t out_stride, void* stream);

/* ---- tcp_ping / icmp_ping ---------------------------------
 * IP + Ethernet layer shared by these builders: Ipv4PacketBuilder (IHL 5,
 * builder/ipv4.rs:94-170) or Ipv6PacketBuilder (builder/ipv6.rs:89-152), then
 * EthernetPacketBuilder (builder/ethernet.rs:63-70). */
typedef struct nexg_ip_build {
    const uint8_t* src_ip;    /* per frame: 4 B (family 4) or 16 B (family 6), network order, 4-B aligned */
    const uint8_t* dst_ip;
    const uint16_t* ip_id;    /* family 4: per frame, or NULL -> def_ip_id */
    const uint8_t* src_mac;   /* 6 B per frame, or NULL -> def_src_mac */
    const uint8_t* dst_mac;
    uint32_t family;          /* 4 or 6 */
    uint32_t flow_label;      /* family 6, low 20 bits */
    uint16_t def_ip_id;
    uint8_t def_src_mac[6], def_dst_mac[6];
    uint8_t ttl;              /* IPv4 TTL / IPv6 hop limit (builders default 64) */
    uint8_t ip_flags;         /* IPv4 3-bit flags (tcp_ping/icmp_ping: DontFragment 0b010) */
    uint8_t tos;              /* IPv4 dscp<<2|ecn / IPv6 traffic class */
    uint8_t src_shared;       /* 1: src_ip holds ONE address (4 or 16 B), the source of
                                 every frame: the probe batches of tcp_ping / icmp_ping
                                 (tcp_ping.rs:108-163, icmp_ping.rs:67-120: one interface
                                 address, a destination per target) */
    uint8_t reserved[2];
} nexg_ip_build;

/* TcpPacketBuilder::build (builder/tcp.rs:93-158; tcp.rs:521-575 to_bytes:
 * options zero-padded to 4 B, data offset = (20 + padded) / 4; checksum
 * tcp::checksum, tcp.rs:1207-1269), composed as examples/tcp_ping.rs:111-163.
 * Frame = 14 + (20|40) + 20 + padded options + payload_len bytes. */
typedef struct nexg_tcp_build {
    nexg_ip_build ip;
    const uint16_t* src_port; /* per frame, or NULL -> def_src_port */
    const uint16_t* dst_port;
    const uint32_t* seq;      /* per frame, or NULL -> def_seq */
    const uint32_t* ack;
    const uint8_t* payload;   /* shared by all frames (may be NULL) */
    uint32_t payload_len;
    uint32_t def_seq, def_ack;
    uint16_t def_src_port, def_dst_port;
    uint16_t window, urgent_ptr;
    uint8_t flags;
    uint8_t options_len;      /* encoded TcpOptionPacket bytes in options[] */
    uint8_t options[40];
    uint8_t reserved[2];
    uint64_t count;
} nexg_tcp_build;

/* IcmpPacketBuilder / Icmpv6PacketBuilder with echo_fields (builder/icmp.rs:
 * 14-86, builder/icmpv6.rs:14-90; checksums icmp.rs:429-432 / icmpv6.rs:
 * 589-599), composed as examples/icmp_ping.rs:67-102. Frame = 14 + (20|40)
 * + 8 + payload_len bytes. */
typedef struct nexg_icmp_echo_build {
    nexg_ip_build ip;
    const uint16_t* identifier; /* per frame, or NULL -> def_identifier */
    const uint16_t* sequence;   /* per frame, or NULL -> def_sequence */
    const uint8_t* payload;
    uint32_t payload_len;
    uint16_t def_identifier, def_sequence;
    uint8_t icmp_type, icmp_code; /* EchoRequest: 8/0 (IPv4), 128/0 (IPv6) */
    uint8_t reserved[2];
    uint64_t count;
} nexg_icmp_echo_build;

/* NEXG_ERANGE on BuildError::LengthOverflow (padded options > 40; segment >
 * 65515 (IPv4) / 65535 (IPv6); ICMP > 65515 / 65535). Probe batches: with
 * ip.src_shared set and every other per-frame array NULL (ports, seq / ack,
 * identifier / sequence, ip_id, MACs) the kernels read only dst_ip per frame
 * (4 / 16 B), as the tcp_ping / icmp_ping probes of one host vary only the
 * target. */
int nexg_build_tcp_batch(nexg_ctx* ctx, const nexg_tcp_build* params, uint8_t* out,
                         uint32_t out_stride, void* stream);
int nexg_build_icmp_echo_batch(nexg_ctx* ctx, const nexg_icmp_echo_build* params,
                               uint8_t* out, uint32_t out_stride, void* stream);

/* ---- arp / ndp probes (the callers examples/arp.rs, examples/ndp.rs) -------
 * ArpPacketBuilder::new(sender_mac, sender_ip, target_ip) (builder/arp.rs:
 * 18-37; build() rejects hw_addr_len != 6 / proto_addr_len != 4 with
 * InvalidFieldLength, :101-118 -> NEXG_EINVAL) serialised by ArpPacket::
 * to_bytes (arp.rs:385-399) behind EthernetPacketBuilder (EtherType 0x0806),
 * as examples/arp.rs:59-67 composes it. Frame = 14 + 28 = 42 bytes. */
typedef struct nexg_arp_build {
    const uint8_t* sender_ip;  /* 4 B per frame (network order), or NULL -> def_sender_ip */
    const uint8_t* target_ip;  /* 4 B per frame */
    const uint8_t* sender_mac; /* 6 B per frame, or NULL -> def_sender_mac (also the Ethernet source) */
    const uint8_t* target_mac; /* 6 B per frame, or NULL -> def_target_mac (builder: zero) */
    const uint8_t* eth_dst;    /* 6 B per frame, or NULL -> def_eth_dst (arp.rs: broadcast) */
    uint8_t def_sender_ip[4];
    uint8_t def_sender_mac[6], def_target_mac[6], def_eth_dst[6];
    uint16_t hardware_type;    /* ArpHardwareType::Ethernet = 1 */
    uint16_t protocol_type;    /* EtherType::Ipv4 = 0x0800 */
    uint16_t operation;        /* ArpOperation::Request = 1 */
    uint8_t hw_addr_len;       /* must be 6 */
    uint8_t proto_addr_len;    /* must be 4 */
    uint64_t count;
} nexg_arp_build;
int nexg_build_arp_batch(nexg_ctx* ctx, const nexg_arp_build* params, uint8_t* out,
                         uint32_t out_stride, void* stream);

/* NdpPacketBuilder::new(src_mac, src_ip, dst_ip).build() (builder/ndp.rs:
 * 30-84): a NeighborSolicit (type 135, code 0, reserved 0, target = dst_ip,
 * one SourceLLAddr option of length 1 carrying src_mac; icmpv6.rs:1385-1400)
 * with icmpv6::checksum over src_ip -> dst_ip (icmpv6.rs:589-599), inside
 * Ipv6PacketBuilder (next header 58) and EthernetPacketBuilder (0x86DD), as
 * examples/ndp.rs:82-108 composes it (hop limit 255; Ethernet destination
 * 33:33 + the target's last four bytes, ipv6_multicast_mac, ndp.rs:25-35).
 * ip.family must be 6; ip.dst_ip is the target; the option's MAC is the
 * Ethernet source. Frame = 14 + 40 + 32 = 86 bytes. */
typedef struct nexg_ndp_ns_build {
    nexg_ip_build ip;
    uint32_t eth_dst_multicast; /* 1: Ethernet destination from the target (ndp.rs); 0: ip.dst_mac / def */
    uint32_t reserved;
    uint64_t count;
} nexg_ndp_ns_build;
int nexg_build_ndp_ns_batch(nexg_ctx* ctx, const nexg_ndp_ns_build* params, uint8_t* out,
                            uint32_t out_stride, void* stream);

/* ---- capture-file batch ingest ---------------------------
 * Replaces nex-datalink's pcap::from_file channel (nex-datalink/src/pcap.rs:
 * 95-109) read one frame per RawReceiver::next (pcap.rs:178-190): each call
 * copies the next records' captured bytes back to back into a host buffer
 * (pinned for the H2D pipeline) and writes the packed offset table, ready for
 * nexg_parse_batch (offsets without lengths). Classic pcap (µs/ns, either
 * byte order) and pcapng (SHB, IDB, EPB, SPB, OPB). Host-side only. */
typedef struct nexg_pcap nexg_pcap;
int nexg_pcap_open(const char* path, nexg_pcap** out);
/* LINKTYPE of the file (first interface for pcapng): 1 = Ethernet; 101 =
 * raw IP (parse with NEXG_PARSE_FROM_IP, ip_offset 0). */
int nexg_pcap_linktype(const nexg_pcap* p);
const char* nexg_pcap_last_error(const nexg_pcap* p);
/* Up to max_frames records: frame k at data + offsets[k], offsets[n] = end
 * (offsets holds max_frames + 1 entries); ts_ns (optional) receives
 * timestamps in ns. *n_frames = 0 at end of file. A record that does not fit
 * data_cap waits for the next call (NEXG_ERANGE if not even one fits).
 * NEXG_EINVAL on a malformed or truncated file, after the complete records
 * before the damage were delivered. */
int nexg_pcap_read_batch(nexg_pcap* p, uint8_t* data, uint64_t data_cap, uint64_t* offsets,
                         uint64_t max_frames, uint64_t* ts_ns, uint64_t* n_frames);
/* In-place shape: the next file bytes are read straight into buf (up to cap,
 * one copy from the page cache) and the records found there are described by
 * offsets[k] / lengths[k] into buf (record headers stay in place; parse with
 * this offsets + lengths layout). Bytes of a record cut at the end of buf are
 * carried to the next call. *bytes_used = bytes of buf holding complete
 * records; *n_frames == 0 and *bytes_used == 0 means end of file. */
int nexg_pcap_read_raw(nexg_pcap* p, uint8_t* buf, uint64_t cap, uint64_t* offsets,
                       uint32_t* lengths, uint64_t max_frames, uint64_t* ts_ns,
                       uint64_t* n_frames, uint64_t* bytes_used);
/* Zero-copy shape: no read at all. nexg_pcap_map maps the file read-only
 * (the page cache itself; *data, *size = file bytes, *first = offset of the
 * first record or block). nexg_pcap_walk_mapped describes the records in the
 * window [from, from + max_bytes) of the mapping: offsets[k] (relative to
 * `from`) / lengths[k], *next = the offset after the last complete record
 * (the next call's `from`). The caller registers the mapping for DMA
 * (hipHostRegister) and copies [from, *next) to the GPU as is: the same
 * in-place layout as read_raw (record headers between frames, monotone), at
 * PCIe rate with no host copy. End of file when *next == size. Classic pcap
 * uses nexg_pcap_set_read_threads for the parallel walk. Use one shape per
 * reader: the mapped walk does not move the file position. */
int nexg_pcap_map(nexg_pcap* p, const uint8_t** data, uint64_t* size, uint64_t* first);
int nexg_pcap_walk_mapped(nexg_pcap* p, uint64_t from, uint64_t max_bytes, uint64_t* offsets,
                          uint32_t* lengths, uint64_t max_frames, uint64_t* ts_ns, uint64_t* n_frames,
                          uint64_t* next);
/* read_raw's file reads split over up to `threads` (1..64) parallel preads
 * of >= 4-MiB pieces (default 1), and for classic pcap the record walk of a
 * read (or mapped window) of >= 8 MiB split over as many threads, eight
 * interleaved chunks each (speculative chunk starts, stitched; a
 * disagreement re-walks that chunk). Results are identical for any count.
 * (read_batch stays single-threaded: parallel record copies into pinned
 * staging measured 2.5-4x slower on the GPU boxes, profiles/r01_ingest/threads.) */
int nexg_pcap_set_read_threads(nexg_pcap* p, uint32_t threads);
int nexg_pcap_close(nexg_pcap* p);

/* ---- live datalink batch rx / tx ---------------------------
 * The reference's Linux channel (nex-datalink/src/linux.rs:102-218) hands one
 * frame per RawReceiver::next (poll + recvfrom into a 4096-B buffer,
 * linux.rs:356-397) and sends one per RawSender::send (poll + sendto,
 * linux.rs:302-346); its scale-out is PACKET_FANOUT (lib.rs:70-131,
 * linux.rs:154-193). Here an AF_PACKET socket with the same Config knobs
 * (read_buffer_size, promiscuous, linux_fanout, read timeout) fills whole
 * batches: the TPACKET_V3 mmap ring (blocks of frames retired by the kernel)
 * or recvmmsg, copied into the caller's (pinned) buffer in the packed layout
 * nexg_pcap_read_batch produces (offsets only, parse with SpanTile). Each
 * frame is its first min(len, read_buffer_size) bytes, as recvfrom into the
 * reference's read buffer truncates it. One rx per GPU in one fanout group
 * is the multi-GPU ingest. Host-side only; needs
 * CAP_NET_RAW (open fails with NEXG_EPERM without it). */
#define NEXG_RX_RING 0u  /* TPACKET_V3 mmap ring (default)                   */
#define NEXG_RX_MMSG 1u  /* recvmmsg into read_buffer_size slots             */
/* FanoutType (nex-datalink/src/lib.rs:70-90) = PACKET_FANOUT_* */
#define NEXG_FANOUT_HASH 0u
#define NEXG_FANOUT_LB 1u
#define NEXG_FANOUT_CPU 2u
#define NEXG_FANOUT_ROLLOVER 3u
#define NEXG_FANOUT_RND 4u
#define NEXG_FANOUT_QM 5u
#define NEXG_FANOUT_FLAG_ROLLOVER 0x1000u /* FanoutOption.rollover */
#define NEXG_FANOUT_FLAG_DEFRAG 0x8000u   /* FanoutOption.defrag   */
/* rx flags: drop the loopback echo of frames this host sends (sll_pkttype
 * PACKET_OUTGOING); the reference keeps them (recvfrom discards sockaddr_ll,
 * linux.rs:358), so the default is to keep them too. */
#define NEXG_RX_SKIP_OUTGOING 0x1u
typedef struct nexg_rx_config {
    uint32_t read_buffer_size; /* Config.read_buffer_size (default 4096, lib.rs:229) */
    int32_t read_timeout_ms;   /* Config.read_timeout; -1 = wait (default)          */
    uint32_t promiscuous;      /* Config.promiscuous (default 1)                    */
    uint32_t fanout;           /* 1: join linux_fanout group below                  */
    uint32_t fanout_type;      /* NEXG_FANOUT_* | NEXG_FANOUT_FLAG_*               */
    uint32_t fanout_group;     /* FanoutOption.group_id                             */
    uint32_t mode;             /* NEXG_RX_RING / NEXG_RX_MMSG                       */
    uint32_t ring_block_size;  /* TPACKET_V3 block bytes (default 1 MiB)            */
    uint32_t ring_blocks;      /* blocks in the ring (default 64)                   */
    uint32_t ring_block_tov_ms;/* block retire timeout (default 2 ms)               */
    uint32_t flags;            /* NEXG_RX_*                                         */
    uint32_t reserved;
} nexg_rx_config;
typedef struct nexg_rx nexg_rx;
typedef struct nexg_tx nexg_tx;
void nexg_rx_config_default(nexg_rx_config* cfg);
int nexg_rx_open(const char* ifname, const nexg_rx_config* cfg, nexg_rx** out);
/* Up to max_frames frames (bytes packed: frame k at data + offsets[k],
 * offsets[n] = end; offsets holds max_frames + 1 entries); waits up to the
 * read timeout for the first frame (*n_frames = 0 on timeout), then takes
 * whatever the ring / socket already holds. ts_ns optional. NEXG_ERANGE
 * (nothing taken) when data_cap cannot hold the next frame (ring mode) or one
 * read_buffer_size slot (recvmmsg mode): a retry with a larger buffer
 * resumes at that frame. */
int nexg_rx_next_batch(nexg_rx* rx, uint8_t* data, uint64_t data_cap, uint64_t* offsets,
                       uint64_t max_frames, uint64_t* ts_ns, uint64_t* n_frames);
/* PACKET_STATISTICS since the last call: frames seen, frames dropped. */
int nexg_rx_stats(nexg_rx* rx, uint64_t* packets, uint64_t* drops);
int nexg_rx_close(nexg_rx* rx);
/* The ring walker on one retired TPACKET_V3 block (struct tpacket_block_desc
 * + tpacket3_hdr chain, linux/if_packet.h), from packet `first` on: frames
 * appended to the packed batch at data[*pos...] with offsets[*n...] until
 * max_frames / data_cap; *next_pkt = the first packet not taken (== the
 * block's num_pkts when done). What nexg_rx_next_batch runs on each block;
 * exported so the walk is tested on synthetic blocks without a socket. */
int nexg_tpacket3_walk(const uint8_t* block, uint64_t block_bytes, uint32_t first, uint32_t snap,
                       uint32_t flags, uint8_t* data, uint64_t data_cap, uint64_t* pos,
                       uint64_t* offsets, uint64_t max_frames, uint64_t* ts_ns, uint64_t* n,
                       uint32_t* next_pkt);
int nexg_tx_open(const char* ifname, nexg_tx** out);
/* Sends frames (host memory, the nexg_frames layout: offsets NULL -> stride)
 * with sendmmsg, up to 1024 per system call, waiting for POLLOUT as
 * RawSender::send does; *n_sent = frames the kernel accepted. */
int nexg_tx_send_batch(nexg_tx* tx, const uint8_t* data, const uint64_t* offsets, const uint32_t* lengths,
                       uint32_t stride, uint64_t count, uint64_t* n_sent);
int nexg_tx_close(nexg_tx* tx);

/* ---- synthetic workloads --------------------------
 * Frame i of a workload depends only on (seed, first_index + i), so shards
 * regenerate identically on any GPU count. */
#define NEXG_WL_UDP64 1 /* 64-B Eth/IPv4/UDP, 1/16 with a flipped checksum bit */
#define NEXG_WL_IMIX 2  /* 64/576/1500 at 7:4:1 over {v4,v6}x{TCP,UDP,ICMP}   */

/* Frame length of each frame of the workload (device lengths[count]). */
int nexg_gen_lengths(nexg_ctx* ctx, int workload, uint64_t seed,
                     uint64_t first_index, uint64_t count, uint32_t* lengths,
                     void* stream);
/* Writes frame i at data + offsets[i] (offsets NULL -> i*stride). */
int nexg_gen_frames(nexg_ctx* ctx, int workload, uint64_t seed,
                    uint64_t first_index, uint64_t count, uint8_t* data,
                    const uint64_t* offsets, uint32_t stride, void* stream);
/* SER parameter tuples: src_ip, dst_ip, src_port, dst_port, ip_id. */
int nexg_gen_udp4_params(nexg_ctx* ctx, uint64_t seed, uint64_t first_index,
                         uint64_t count, uint32_t* src_ip, uint32_t* dst_ip,
                         uint16_t* src_port, uint16_t* dst_port,
                         uint16_t* ip_id, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* NEXG_H */
