/*
 * nex_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of shellrow/nex nex-packet's per-frame path, used as the
 * parity checker for the HIP engine (nex_amd). Only tests/, __graft_entry__
 * smoke() and bench.py's cpu_baseline leg may load it; the product never does.
 *
 * Parity pinning: the reference is Rust with no Cargo.lock and no vendored
 * crates, and cargo/rustc are absent from this image, so the reference cannot
 * be built or run here. This restatement is pinned by the
 * reference's own known-answer tests and fixtures, committed as data under
 * tests/golden/ (util.rs:190-261, icmpv6.rs:606-631, frame.rs:665-784,
 * ipv4.rs:944-1204, ipv6.rs:706-802, tcp.rs:1276-1314, udp.rs:511-527,
 * icmp.rs:708-725, the fuzz seed corpus and the bench frames).
 *
 * Every function follows the reference literally — including re-serialising
 * packets before checksumming them (to_bytes), as the Rust does — so that it is
 * an independent algorithm from the GPU kernels, which fold the same
 * arithmetic into closed-form word sums.
 */
#ifndef NEX_ORACLE_H
#define NEX_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/nexg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* util.rs:65 checksum(data, skipword) */
uint16_t nexo_checksum(const uint8_t* data, size_t len, size_t skipword);
/* util.rs:141 sum_be_words (private in the reference; exposed for its KATs) */
uint32_t nexo_sum_be_words(const uint8_t* data, size_t len, size_t skipword);
/* util.rs:169 sum_be_words_joined */
uint32_t nexo_sum_be_words_joined(const uint8_t* data, size_t len,
                                  size_t skipword, const uint8_t* extra,
                                  size_t extra_len);
/* util.rs:81 ipv4_checksum */
uint16_t nexo_ipv4_checksum(const uint8_t* data, size_t len, size_t skipword,
                            const uint8_t* extra, size_t extra_len,
                            const uint8_t src[4], const uint8_t dst[4],
                            uint8_t proto);
/* util.rs:111 ipv6_checksum */
uint16_t nexo_ipv6_checksum(const uint8_t* data, size_t len, size_t skipword,
                            const uint8_t* extra, size_t extra_len,
                            const uint8_t src[16], const uint8_t dst[16],
                            uint8_t proto);

/* frame.rs:309 Frame::try_from_buf_with_mode + verification checksums for one
 * frame, written as a nexg_record (and its nexg_desc projection). */
void nexo_parse_frame(const uint8_t* frame, size_t len, uint32_t flags,
                      uint32_t ip_offset, nexg_record* rec);
void nexo_record_to_desc(const nexg_record* rec, nexg_desc* desc);
/* Ipv4Header.options / TcpHeader.options of the same Frame as positions
 * (include/nexg.h nexg_options; ipv4.rs:442-508, tcp.rs:767-818). */
void nexo_decode_options(const uint8_t* frame, size_t len, uint32_t flags,
                         uint32_t ip_offset, nexg_options* out);

/* Batch form over a host-memory nexg_frames layout (pointers are HOST). */
int nexo_parse_batch(const nexg_frames* frames, uint32_t flags,
                     uint32_t ip_offset, nexg_record* recs, nexg_desc* descs,
                     int nthreads);

/* Builders: udp_ping.rs:68-109 composition for one tuple. Returns bytes
 * written (42 + payload_len) or -1 on BuildError. */
/* FrameSlice::try_from_buf (frame.rs:84-287) */
void nexo_slice_frame(const uint8_t* packet, size_t len, uint32_t flags, uint32_t ip_offset,
                      nexg_slice* out);
void nexo_slice_batch(const nexg_frames* fr, uint32_t flags, uint32_t ip_offset, nexg_slice* out);

/* IP/Ethernet layer parameters of the tcp_ping / icmp_ping builders. v4
 * addresses use the first 4 bytes of src/dst. */
typedef struct nexo_ip_spec {
    int family; /* 4 or 6 */
    uint8_t src[16], dst[16];
    uint8_t src_mac[6], dst_mac[6];
    uint16_t ip_id;
    uint8_t ttl, ip_flags, dscp_ecn; /* v6: ttl = hop limit, dscp_ecn = traffic class */
    uint32_t flow_label;
} nexo_ip_spec;
int nexo_build_tcp(const nexo_ip_spec* ip, uint16_t sport, uint16_t dport, uint32_t seq,
                   uint32_t ack, uint8_t flags, uint16_t window, uint16_t urg,
                   const uint8_t* opts, uint32_t opt_len, const uint8_t* payload,
                   uint32_t payload_len, uint8_t* out);
int nexo_build_icmp_echo(const nexo_ip_spec* ip, uint8_t type, uint8_t code, uint16_t ident,
                         uint16_t seqno, const uint8_t* payload, uint32_t payload_len,
                         uint8_t* out);
/* examples/arp.rs:59-67: ArpPacketBuilder (builder/arp.rs:18-118) behind
 * Ethernet; -1 on InvalidFieldLength (hw_len != 6 / proto_len != 4). */
int nexo_build_arp(const uint8_t eth_dst[6], const uint8_t sender_mac[6], const uint8_t sender_ip[4],
                   const uint8_t target_mac[6], const uint8_t target_ip[4], uint16_t hardware_type,
                   uint16_t protocol_type, uint16_t operation, uint8_t hw_len, uint8_t proto_len,
                   uint8_t* out);
/* examples/ndp.rs:82-108: NdpPacketBuilder (builder/ndp.rs:30-84) inside
 * Ipv6PacketBuilder + EthernetPacketBuilder; ip->dst is the target; the
 * Ethernet destination is ip->dst_mac (the caller applies ndp.rs's
 * ipv6_multicast_mac when it wants it). 86 bytes. */
int nexo_build_ndp_ns(const nexo_ip_spec* ip, uint8_t* out);

int nexo_build_udp4(const uint8_t src_mac[6], const uint8_t dst_mac[6],
                    uint32_t src_ip, uint32_t dst_ip, uint16_t sport,
                    uint16_t dport, uint16_t ip_id, uint8_t ttl,
                    uint8_t ip_flags, uint8_t dscp_ecn, const uint8_t* payload,
                    uint32_t payload_len, uint8_t* out);
/* a batch of udp_ping IPv4 builds with empty payloads, 42 B per tuple at
 * out + 42 i (the serialize bench's CPU baseline) */
typedef struct {
    const uint8_t* src_mac;
    const uint8_t* dst_mac;
    const uint32_t* src_ip;
    const uint32_t* dst_ip;
    const uint16_t* src_port;
    const uint16_t* dst_port;
    const uint16_t* ip_id;
    uint64_t count;
    uint8_t ttl, ip_flags;
} nexo_udp4_tuples;
int nexo_build_udp4_batch(const nexo_udp4_tuples* p, uint8_t* out, int nthreads);
int nexo_build_udp6(const uint8_t src_mac[6], const uint8_t dst_mac[6],
                    const uint8_t src_ip[16], const uint8_t dst_ip[16], uint16_t sport,
                    uint16_t dport, uint8_t hop_limit, uint8_t traffic_class,
                    uint32_t flow_label, const uint8_t* payload, uint32_t payload_len,
                    uint8_t* out);

/* A probe batch of one of the udp_ping / tcp_ping / icmp_ping compositions:
 * every field from `ip` and the L4 fields below, except the destination, which
 * is dst[i] (4 B for family 4, 16 B for 6); frame i (flen bytes, the return
 * value of one single build) at out + flen i. kind: 0 tcp (nexo_build_tcp),
 * 1 icmp echo (nexo_build_icmp_echo), 2 udp over IPv6 (nexo_build_udp6).
 * Static index-range split over nthreads (the probe builders' CPU baseline).
 * Returns flen, or -1 (length overflow). */
typedef struct {
    int kind;
    nexo_ip_spec ip;
    const uint8_t* dst;
    uint64_t count;
    uint16_t sport, dport, window, urg;   /* tcp; udp6: sport / dport */
    uint32_t seq, ack;
    uint8_t tcp_flags, icmp_type, icmp_code, pad0;
    uint16_t ident, seqno;                 /* icmp echo */
    const uint8_t* opts; uint32_t opt_len;
    const uint8_t* payload; uint32_t payload_len;
} nexo_probe_batch;
int nexo_build_probe_batch(const nexo_probe_batch* p, uint8_t* out, int nthreads);

/* nexg_recompute_checksums_batch's semantics for one frame, in place: the
 * mutable views' recompute_checksum chained as mutable_chaining.rs:19-63. */
void nexo_recompute_frame(uint8_t* frame, size_t len, uint32_t flags, uint32_t ip_offset, uint32_t which,
                          nexg_fixup* out);

/* Synthetic workloads, independent CPU implementation
 * of the generator the engine ships (nexg_gen_*). */
uint32_t nexo_gen_length(int workload, uint64_t seed, uint64_t index);
void nexo_gen_frame(int workload, uint64_t seed, uint64_t index, uint8_t* out);
void nexo_gen_udp4_params(uint64_t seed, uint64_t index, uint32_t* src_ip,
                          uint32_t* dst_ip, uint16_t* sport, uint16_t* dport,
                          uint16_t* ip_id);

#ifdef __cplusplus
}
#endif
#endif
