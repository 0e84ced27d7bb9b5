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
 *     is stream-ordered: the call returns before the kernels finish.
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
    NEXG_ERANGE = -5   /* BuildError::LengthOverflow (builder/error.rs:8)  */
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
 * arp.rs:340-371). Fields of absent layers are 0. */
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
 * data_bytes bounds every device load: no byte at or past data+data_bytes is
 * read. All pointers are device pointers. */
typedef struct nexg_frames {
    const uint8_t* data;
    uint64_t data_bytes;
    const uint64_t* offsets;
    const uint32_t* lengths;
    uint32_t stride;
    uint32_t reserved;
    uint64_t count;
} nexg_frames;

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
 * out_per_64 = 0: read only; out[tile] = XOR of the tile's dwords (4 B per
 * 16 KiB). bench.py reports the headline kernel against both. */
int nexg_probe_stream(nexg_ctx* ctx, const void* data, uint64_t bytes, uint32_t out_per_64,
                      void* out, void* stream);

/* ---- serialize path (udp_ping.rs:68-109 shape) -------------------------- */
typedef struct nexg_udp4_build {
    const uint32_t* src_ip;   /* per frame, IPv4 address as BE u32 value     */
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
    uint64_t count;
} nexg_udp4_build;

/* Writes frame i (42 + payload_len bytes) at out + i*out_stride.
 * NEXG_ERANGE if 28 + payload_len > 65535 (builder/udp.rs:83, ipv4.rs:153). */
int nexg_build_udp4_batch(nexg_ctx* ctx, const nexg_udp4_build* params,
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
    uint8_t reserved[2];
    uint64_t count;
} nexg_udp6_build;

/* Writes frame i (62 + payload_len bytes) at out + i*out_stride.
 * NEXG_ERANGE if 8 + payload_len > 65535 (builder/udp.rs:83, builder/ipv6.rs:137). */
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
    uint8_t reserved[3];
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
 * 65515 (IPv4) / 65535 (IPv6); ICMP > 65515 / 65535). */
int nexg_build_tcp_batch(nexg_ctx* ctx, const nexg_tcp_build* params, uint8_t* out,
                         uint32_t out_stride, void* stream);
int nexg_build_icmp_echo_batch(nexg_ctx* ctx, const nexg_icmp_echo_build* params,
                               uint8_t* out, uint32_t out_stride, void* stream);

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
/* read_raw's file reads split over up to `threads` (1..64) parallel preads
 * of >= 4-MiB pieces (default 1). Results are identical for any count.
 * (read_batch stays single-threaded: parallel record copies into pinned
 * staging measured 2.5-4x slower on the GPU boxes, profiles/r01_ingest/threads.) */
int nexg_pcap_set_read_threads(nexg_pcap* p, uint32_t threads);
int nexg_pcap_close(nexg_pcap* p);

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
