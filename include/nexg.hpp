/*
 * nexg.hpp — C++17 host API above the C ABI (include/nexg.h), mirroring
 * nex-packet's frame API for code that called the reference from a compiled
 * language (the reference is Rust; cargo is absent here, so this is the host
 * side a C++ caller links against, INTEGRATION.md gives the Rust binding).
 *
 * Names, field meanings and error behaviour follow the reference:
 *   ParseMode / ParseOption / ParseError   parse.rs:34-97, frame.rs:47-50
 *   Frame, DatalinkLayer, IpLayer, TransportLayer   frame.rs:21-60
 *   EthernetHeader ethernet.rs:152-160, ArpHeader arp.rs:300-311,
 *   Ipv4Header ipv4.rs:187-202 (+ Ipv4OptionPacket ipv4.rs:39-182),
 *   Ipv6Header ipv6.rs:14-23, IcmpHeader icmp.rs:172-176,
 *   Icmpv6Header icmpv6.rs:229-234, TcpHeader tcp.rs:482-494
 *   (+ TcpOptionPacket tcp.rs:33-476), UdpHeader udp.rs:22-27
 *   Engine::try_from_bufs   Frame::try_from_buf_with_mode (frame.rs:309) on a
 *                           batch: one Result<Frame, ParseError> per frame
 *   Engine::frame_slices    FrameSlice::try_from_buf (frame.rs:86) on a batch
 *   Engine::build_udp_ping  UdpPacketBuilder -> Ipv4PacketBuilder ->
 *                           EthernetPacketBuilder (udp_ping.rs:68-109) per
 *                           tuple, Result<frames, BuildError>
 *   Engine::build_tcp_ping / build_icmp_ping   tcp_ping.rs:111-163 /
 *                           icmp_ping.rs:67-102 (IPv4 or IPv6 per batch)
 * The device does the parse and the checksums (nexg_parse_batch,
 * NEXG_OUT_RECORD) and the option lists (nexg_decode_options); this header
 * only reads header fields out of the frame bytes at the offsets the device
 * reported. API misuse and HIP failures throw nexg::Error; per-frame parse
 * failures are data (Result), as in the reference. Header-only; link
 * libnexg.so and amdhip64.
 */
#ifndef NEXG_HPP
#define NEXG_HPP

#include <hip/hip_runtime.h>

#include <array>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <optional>
#include <stdexcept>
#include <string>
#include <utility>
#include <variant>
#include <vector>

#include "nexg.h"

namespace nexg {

/* ---- parse knobs and errors ------------------------------------------- */

enum class ParseMode { Lenient, Strict };  // parse.rs:34-46

struct ParseOption {  // frame.rs:47-50 (+ the NEXG_PARSE_VLAN extension, off by default)
    bool from_ip_packet = false;
    size_t offset = 0;
    bool unwrap_vlan = false;
    uint32_t flags(ParseMode mode) const {
        return (from_ip_packet ? NEXG_PARSE_FROM_IP : 0u) | (unwrap_vlan ? NEXG_PARSE_VLAN : 0u) |
               (mode == ParseMode::Strict ? NEXG_PARSE_STRICT : 0u);
    }
};

enum class ParseErrorKind : uint8_t {  // parse.rs:51-97
    BufferTooShort = NEXG_ERR_BUFFER_TOO_SHORT,
    InvalidLength = NEXG_ERR_INVALID_LENGTH,
    Malformed = NEXG_ERR_MALFORMED,
    Truncated = NEXG_ERR_TRUNCATED,
    BadExtent = NEXG_ERR_BAD_EXTENT,  // caller error: frame longer than 65535 bytes
};

// The reference's ParseError with its payload (parse.rs:53-81), carried in
// the failed frame's record (include/nexg.h NEXG_CTX_*): `context` is the
// reference's context string; minimum / actual (BufferTooShort), value
// (InvalidLength), expected / actual (Truncated).
struct ParseError {
    ParseErrorKind kind;
    const char* context = nullptr;
    size_t minimum = 0, actual = 0, value = 0, expected = 0;
    const char* name() const {
        switch (kind) {
            case ParseErrorKind::BufferTooShort: return "BufferTooShort";
            case ParseErrorKind::InvalidLength: return "InvalidLength";
            case ParseErrorKind::Malformed: return "Malformed";
            case ParseErrorKind::Truncated: return "Truncated";
            default: return "BadExtent";
        }
    }
    static const char* context_of(uint32_t ctx) {
        static const char* const k[] = {nullptr, "Ethernet packet", "Frame dummy Ethernet classification",
                                        "IPv4 packet", "IPv4 packet version", "IPv4 header length", "IPv4 header",
                                        "IPv4 total length", "IPv4 options", "IPv4 option length", "IPv6 packet",
                                        "IPv6 packet version", "IPv6 payload", "IPv6 extension header",
                                        "IPv6 routing header", "IPv6 fragment header"};
        return ctx < sizeof(k) / sizeof(k[0]) ? k[ctx] : nullptr;
    }
    // the error of a failed frame's NEXG_OUT_RECORD record
    static ParseError from_record(const nexg_record& r) {
        ParseError e{(ParseErrorKind)NEXG_STATUS(r.flags)};
        if (e.kind == ParseErrorKind::BadExtent) return e;
        e.context = context_of(r.l4_type);
        if (e.kind == ParseErrorKind::BufferTooShort) { e.minimum = r.ip_src; e.actual = r.ip_dst; }
        if (e.kind == ParseErrorKind::InvalidLength) e.value = r.ip_src;
        if (e.kind == ParseErrorKind::Truncated) { e.expected = r.ip_src; e.actual = r.ip_dst; }
        return e;
    }
};

enum class BuildError { LengthOverflow, AddressFamilyMismatch, InvalidFieldLength };  // builder/error.rs:6-53

// Result<T, E>, as the reference's parse (ParseError) and build (BuildError)
// functions return
template <class T, class E = ParseError>
class Result {
   public:
    Result(T v) : v_(std::move(v)) {}
    Result(E e) : v_(e) {}
    bool is_ok() const { return v_.index() == 0; }
    bool is_err() const { return v_.index() == 1; }
    const T& value() const { return std::get<0>(v_); }
    T& value() { return std::get<0>(v_); }
    const E& error() const { return std::get<1>(v_); }

   private:
    std::variant<T, E> v_;
};

struct Error : std::runtime_error {
    using std::runtime_error::runtime_error;
};

/* ---- addresses and headers -------------------------------------------- */

using MacAddr = std::array<uint8_t, 6>;

struct Ipv4Addr {
    std::array<uint8_t, 4> octets{};
    std::string to_string() const {
        char b[16];
        snprintf(b, sizeof(b), "%u.%u.%u.%u", octets[0], octets[1], octets[2], octets[3]);
        return b;
    }
    bool operator==(const Ipv4Addr& o) const { return octets == o.octets; }
};

struct Ipv6Addr {
    std::array<uint8_t, 16> octets{};
    bool operator==(const Ipv6Addr& o) const { return octets == o.octets; }
};

struct EthernetHeader {  // ethernet.rs:152-160
    MacAddr destination{}, source{};
    uint16_t ethertype = 0;  // EtherType::value()
};

struct ArpHeader {  // arp.rs:300-311
    uint16_t hardware_type = 0, protocol_type = 0;
    uint8_t hw_addr_len = 0, proto_addr_len = 0;
    uint16_t operation = 0;
    MacAddr sender_hw_addr{};
    Ipv4Addr sender_proto_addr;
    MacAddr target_hw_addr{};
    Ipv4Addr target_proto_addr;
};

struct Ipv4OptionHeader {  // ipv4.rs:39-182
    uint8_t copied = 0, class_ = 0, number = 0;  // number = Ipv4OptionType::value()
    std::optional<uint8_t> length;
};
struct Ipv4OptionPacket {
    Ipv4OptionHeader header;
    std::vector<uint8_t> data;
};

struct Ipv4Header {  // ipv4.rs:187-202
    uint8_t version = 4, header_length = 0, dscp = 0, ecn = 0;
    uint16_t total_length = 0, identification = 0;
    uint8_t flags = 0;
    uint16_t fragment_offset = 0;
    uint8_t ttl = 0;
    uint8_t next_level_protocol = 0;  // IpNextProtocol::value() (143..=252 -> 255, Q8)
    uint16_t checksum = 0;
    Ipv4Addr source, destination;
    std::vector<Ipv4OptionPacket> options;
};

struct Ipv6Header {  // ipv6.rs:14-23
    uint8_t version = 6, traffic_class = 0;
    uint32_t flow_label = 0;
    uint16_t payload_length = 0;
    uint8_t next_header = 0;  // raw byte 6 (Q10)
    uint8_t hop_limit = 0;
    Ipv6Addr source, destination;
};

struct IcmpHeader {  // icmp.rs:172-176
    uint8_t icmp_type = 0, icmp_code = 0;
    uint16_t checksum = 0;
};
struct Icmpv6Header {  // icmpv6.rs:229-234
    uint8_t icmpv6_type = 0, icmpv6_code = 0;
    uint16_t checksum = 0;
};

struct TcpOptionPacket {  // tcp.rs:33-476
    uint8_t kind = 0;
    std::optional<uint8_t> length;
    std::vector<uint8_t> data;
};

struct TcpHeader {  // tcp.rs:482-494
    uint16_t source = 0, destination = 0;
    uint32_t sequence = 0, acknowledgement = 0;
    uint8_t data_offset = 0, reserved = 0, flags = 0;
    uint16_t window = 0, checksum = 0, urgent_ptr = 0;
    std::vector<TcpOptionPacket> options;
};

struct UdpHeader {  // udp.rs:22-27
    uint16_t source = 0, destination = 0, length = 0, checksum = 0;
};

struct DatalinkLayer {
    std::optional<EthernetHeader> ethernet;
    std::optional<ArpHeader> arp;
};
struct IpLayer {
    std::optional<Ipv4Header> ipv4;
    std::optional<Ipv6Header> ipv6;
    std::optional<IcmpHeader> icmp;
    std::optional<Icmpv6Header> icmpv6;
};
struct TransportLayer {
    std::optional<TcpHeader> tcp;
    std::optional<UdpHeader> udp;
};

// What the engine adds to the Frame path: the packet-API verification
// checksums (DESIGN.md §1 "Verify semantics")
struct Checksums {
    bool ip_checked = false, ip_ok = false, ip_panic = false, l4_checked = false, l4_ok = false;
    uint16_t ip_computed = 0, l4_computed = 0;
};

struct Frame {  // frame.rs:54-60
    std::optional<DatalinkLayer> datalink;
    std::optional<IpLayer> ip;
    std::optional<TransportLayer> transport;
    std::vector<uint8_t> payload;
    size_t packet_len = 0;
    Checksums checksums;
};

// FrameSlice (frame.rs:62-83): layer boundaries borrowed from the input frame
struct Bytes {
    const uint8_t* data = nullptr;
    size_t len = 0;
    std::vector<uint8_t> to_vec() const { return std::vector<uint8_t>(data, data + len); }
};
struct FrameSlice {
    Bytes packet;
    std::optional<Bytes> datalink, network, transport;
    Bytes payload;
    std::optional<uint16_t> ethertype;
    std::optional<uint8_t> ip_protocol;
};

inline Result<FrameSlice> frame_slice_from(const nexg_slice& s, const uint8_t* b, size_t len) {
    if (NEXG_STATUS(s.flags)) return ParseError{(ParseErrorKind)NEXG_STATUS(s.flags)};
    FrameSlice fs;
    fs.packet = Bytes{b, len};
    if (s.flags & NEXG_S_DATALINK) fs.datalink = Bytes{b, 14};
    if (s.flags & NEXG_S_NETWORK) fs.network = Bytes{b + s.l3_off, s.l3_len};
    if (s.flags & NEXG_S_TRANSPORT) fs.transport = Bytes{b + s.l3_off + s.l3_len, s.l4_len};
    fs.payload = Bytes{b + s.payload_off, s.payload_len};
    if (s.flags & NEXG_S_ETHERTYPE) fs.ethertype = s.ethertype;
    if (s.flags & NEXG_S_IP_PROTOCOL) fs.ip_protocol = (uint8_t)(s.flags >> NEXG_S_PROTO_SHIFT);
    return fs;
}

// The udp_ping frame shape (examples/udp_ping.rs:68-109): UdpPacketBuilder ->
// Ipv4PacketBuilder -> EthernetPacketBuilder, one frame per tuple
struct UdpPingTuple {
    Ipv4Addr source, destination;
    uint16_t src_port = 0, dst_port = 0, ip_id = 0;
};
struct UdpPingShape {
    MacAddr src_mac{}, dst_mac{};
    uint8_t ttl = 64;       // Ipv4PacketBuilder default (builder/ipv4.rs:37)
    uint8_t ip_flags = 2;   // udp_ping sets DontFragment
    std::vector<uint8_t> payload;
};

// An IPv4 or IPv6 address for the builders (std::net::IpAddr)
struct IpAddr {
    uint8_t family = 4;                // 4 or 6
    std::array<uint8_t, 16> octets{};  // IPv4 in the first 4 bytes
    static IpAddr from(const Ipv4Addr& a) {
        IpAddr r;
        memcpy(r.octets.data(), a.octets.data(), 4);
        return r;
    }
    static IpAddr from(const Ipv6Addr& a) {
        IpAddr r;
        r.family = 6;
        r.octets = a.octets;
        return r;
    }
};

// tcp_ping's frame (examples/tcp_ping.rs:111-163): TcpPacketBuilder ->
// Ipv4/Ipv6PacketBuilder -> EthernetPacketBuilder
struct TcpPingTuple {
    IpAddr source, destination;
    uint16_t src_port = 0, dst_port = 0, ip_id = 0;
    uint32_t sequence = 0, acknowledgement = 0;
};
struct TcpPingShape {
    MacAddr src_mac{}, dst_mac{};
    uint8_t ttl = 64, ip_flags = 2, tos = 0;
    uint32_t flow_label = 0;
    uint8_t flags = 0x02;  // SYN
    uint16_t window = 0xffff, urgent_ptr = 0;
    std::vector<uint8_t> options;  // encoded TcpOptionPacket bytes (padded to 4 B on the wire)
    std::vector<uint8_t> payload;
};

// icmp_ping's frame (examples/icmp_ping.rs:67-102): an echo request
// (IcmpPacketBuilder / Icmpv6PacketBuilder with echo_fields)
struct IcmpPingTuple {
    IpAddr source, destination;
    uint16_t identifier = 0, sequence = 0, ip_id = 0;
};
struct IcmpPingShape {
    MacAddr src_mac{}, dst_mac{};
    uint8_t ttl = 64, ip_flags = 2, tos = 0;
    uint32_t flow_label = 0;
    std::vector<uint8_t> payload;
};

// arp.rs's request (examples/arp.rs:59-67): ArpPacketBuilder::new(sender_mac,
// sender_ip, target) behind a broadcast EthernetPacketBuilder
struct ArpProbeShape {
    MacAddr sender_mac{};
    Ipv4Addr sender_ip{};
    MacAddr eth_dst{{0xff, 0xff, 0xff, 0xff, 0xff, 0xff}};
    uint16_t operation = 1;  // ArpOperation::Request
    uint8_t hw_addr_len = 6, proto_addr_len = 4;  // build() accepts only 6 / 4
};
// ndp.rs's solicitation (examples/ndp.rs:82-108): NdpPacketBuilder::new(src_mac,
// src_ip, target) inside Ipv6PacketBuilder (hop limit 255) and Ethernet to
// 33:33 + the target's last four bytes
struct NdpProbeShape {
    MacAddr src_mac{};
    Ipv6Addr src_ip{};
    uint8_t hop_limit = 255;
};

/* ---- materialisation from a device record ------------------------------ */

namespace detail {
inline uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
inline Ipv4Addr v4(uint32_t be_value) {
    return Ipv4Addr{{(uint8_t)(be_value >> 24), (uint8_t)(be_value >> 16), (uint8_t)(be_value >> 8),
                     (uint8_t)be_value}};
}
inline MacAddr mac(const uint8_t* p) {
    MacAddr m;
    memcpy(m.data(), p, 6);
    return m;
}
inline Ipv4OptionPacket ipv4_option_at(const uint8_t* p) {
    Ipv4OptionPacket o;
    o.header.copied = (p[0] >> 7) & 1;
    o.header.class_ = (p[0] >> 5) & 3;
    o.header.number = p[0] & 0x1F;
    if (o.header.number > 1) {
        o.header.length = p[1];
        o.data.assign(p + 2, p + p[1]);
    }
    return o;
}
inline TcpOptionPacket tcp_option_at(const uint8_t* p) {
    TcpOptionPacket o;
    o.kind = p[0];
    if (o.kind > 1) {
        o.length = p[1];
        o.data.assign(p + 2, p + p[1]);
    }
    return o;
}
}  // namespace detail

// Frame from one NEXG_OUT_RECORD record, the frame bytes and (for the option
// lists) the frame's nexg_options. Mirrors nex_amd/frame.py::frame_from_record.
inline Result<Frame> frame_from_record(const nexg_record& r, const uint8_t* b, size_t len,
                                       const nexg_options& opts) {
    using namespace detail;
    const uint32_t f = r.flags;
    if (NEXG_STATUS(f)) return ParseError::from_record(r);
    if (r.payload_off + (size_t)r.payload_len > len || r.l3_off > len) throw Error("record does not fit its frame");
    Frame fr;
    const uint32_t l3 = r.l3_off;
    if (f & NEXG_L_ETHERNET) {
        DatalinkLayer dl;
        EthernetHeader eth;
        eth.ethertype = r.ethertype;
        // a real Ethernet header unless from_ip_packet fabricated one (frame.rs:396-400)
        if ((f & NEXG_L_VLAN) || (l3 == 14 && be16(b + 12) == r.ethertype)) {
            eth.destination = mac(b);
            eth.source = mac(b + 6);
        }
        dl.ethernet = eth;
        if (f & NEXG_L_ARP) {
            ArpHeader a;
            const uint8_t* p = b + l3;
            a.hardware_type = be16(p);
            a.protocol_type = be16(p + 2);
            a.hw_addr_len = p[4];
            a.proto_addr_len = p[5];
            a.operation = be16(p + 6);
            a.sender_hw_addr = mac(p + 8);
            memcpy(a.sender_proto_addr.octets.data(), p + 14, 4);
            a.target_hw_addr = mac(p + 18);
            memcpy(a.target_proto_addr.octets.data(), p + 24, 4);
            dl.arp = a;
        }
        fr.datalink = dl;
    }
    if (f & NEXG_L_IP) {
        IpLayer ip;
        if (f & NEXG_L_IPV4) {
            Ipv4Header h;
            h.header_length = r.ip_ver_ihl & 15;
            h.dscp = r.ip_tos >> 2;
            h.ecn = r.ip_tos & 3;
            h.total_length = r.ip_length;
            h.identification = (uint16_t)(r.ip_word >> 16);
            h.flags = (r.ip_word >> 13) & 7;
            h.fragment_offset = r.ip_word & 0x1FFF;
            h.ttl = r.ip_ttl;
            h.next_level_protocol = r.ip_proto;
            h.checksum = r.ip_csum;
            h.source = v4(r.ip_src);
            h.destination = v4(r.ip_dst);
            for (int k = 0; k < opts.n_ip; k++) h.options.push_back(ipv4_option_at(b + opts.ip_opt_off + opts.ip_pos[k]));
            ip.ipv4 = std::move(h);
        }
        if (f & NEXG_L_IPV6) {
            Ipv6Header h;
            h.traffic_class = r.ip_tos;
            h.flow_label = r.ip_word;
            h.payload_length = r.ip_length;
            h.next_header = r.ip_proto;
            h.hop_limit = r.ip_ttl;
            memcpy(h.source.octets.data(), b + l3 + 8, 16);
            memcpy(h.destination.octets.data(), b + l3 + 24, 16);
            ip.ipv6 = h;
        }
        if (f & NEXG_L_ICMP) ip.icmp = IcmpHeader{r.l4_type, r.l4_code, r.l4_csum};
        if (f & NEXG_L_ICMPV6) ip.icmpv6 = Icmpv6Header{r.l4_type, r.l4_code, r.l4_csum};
        fr.ip = std::move(ip);
    }
    if (f & NEXG_L_TRANSPORT) {
        TransportLayer tp;
        if (f & NEXG_L_TCP) {
            TcpHeader h;
            h.source = r.src_port;
            h.destination = r.dst_port;
            h.sequence = r.tcp_seq;
            h.acknowledgement = r.tcp_ack;
            h.data_offset = r.l4_code >> 4;
            h.reserved = r.l4_code & 15;
            h.flags = r.l4_type;
            h.window = r.tcp_window;
            h.checksum = r.l4_csum;
            h.urgent_ptr = r.tcp_urg;
            for (int k = 0; k < opts.n_tcp; k++) h.options.push_back(tcp_option_at(b + opts.tcp_opt_off + opts.tcp_pos[k]));
            tp.tcp = std::move(h);
        }
        if (f & NEXG_L_UDP) tp.udp = UdpHeader{r.src_port, r.dst_port, r.l4_length, r.l4_csum};
        fr.transport = std::move(tp);
    }
    fr.payload.assign(b + r.payload_off, b + r.payload_off + r.payload_len);
    fr.packet_len = r.packet_len;
    fr.checksums = Checksums{(f & NEXG_C_IP_CHECKED) != 0, (f & NEXG_C_IP_OK) != 0, (f & NEXG_C_IP_PANIC) != 0,
                             (f & NEXG_C_L4_CHECKED) != 0, (f & NEXG_C_L4_OK) != 0, r.ip_csum_calc,
                             r.l4_csum_calc};
    return fr;
}

/* ---- ICMP sub-message views (icmp.rs:434-700, icmpv6.rs echo) ---------------
 * What examples/dump.rs:226-350 downcasts an IcmpPacket / Icmpv6Packet to.
 * The packet comes from a Frame (Frame.ip.icmp + Frame.payload, which for
 * ICMP is every byte after the 4-B header, Q15); each conversion applies the
 * reference's type check and minimum payload and fails with its message. */
struct IcmpPacket {  // icmp.rs:178-183
    IcmpHeader header;
    std::vector<uint8_t> payload;
    size_t total_len() const { return 4 + payload.size(); }  // icmp.rs:241-243
};
struct Icmpv6Packet {  // icmpv6.rs:236-241
    Icmpv6Header header;
    std::vector<uint8_t> payload;
    size_t total_len() const { return 4 + payload.size(); }
};
inline std::optional<IcmpPacket> icmp_packet(const Frame& f) {
    if (!f.ip || !f.ip->icmp) return std::nullopt;
    return IcmpPacket{*f.ip->icmp, f.payload};
}
inline std::optional<Icmpv6Packet> icmpv6_packet(const Frame& f) {
    if (!f.ip || !f.ip->icmpv6) return std::nullopt;
    return Icmpv6Packet{*f.ip->icmpv6, f.payload};
}
namespace icmp {
template <uint8_t TYPE>
struct EchoPacket {  // echo_request (icmp.rs:478-504) / echo_reply (icmp.rs:547-573)
    IcmpHeader header;
    uint16_t identifier = 0, sequence_number = 0;
    std::vector<uint8_t> payload;
    static Result<EchoPacket, const char*> try_from(const IcmpPacket& p) {
        if (p.header.icmp_type != TYPE) return TYPE == 8 ? "Not an Echo Request" : "Not an Echo Reply";
        if (p.payload.size() < 4) return TYPE == 8 ? "Payload too short for Echo Request" : "Payload too short for Echo Reply";
        return EchoPacket{p.header, detail::be16(p.payload.data()), detail::be16(p.payload.data() + 2),
                          std::vector<uint8_t>(p.payload.begin() + 4, p.payload.end())};
    }
};
using EchoRequestPacket = EchoPacket<8>;
using EchoReplyPacket = EchoPacket<0>;
struct DestinationUnreachablePacket {  // icmp.rs:618-647
    IcmpHeader header;
    uint16_t unused = 0, next_hop_mtu = 0;
    std::vector<uint8_t> payload;
    static Result<DestinationUnreachablePacket, const char*> try_from(const IcmpPacket& p) {
        if (p.header.icmp_type != 3) return "Not a Destination Unreachable";
        if (p.payload.size() < 4) return "Payload too short for Destination Unreachable";
        return DestinationUnreachablePacket{p.header, detail::be16(p.payload.data()), detail::be16(p.payload.data() + 2),
                                            std::vector<uint8_t>(p.payload.begin() + 4, p.payload.end())};
    }
};
struct TimeExceededPacket {  // icmp.rs:664-699
    IcmpHeader header;
    uint32_t unused = 0;
    std::vector<uint8_t> payload;
    static Result<TimeExceededPacket, const char*> try_from(const IcmpPacket& p) {
        if (p.header.icmp_type != 11) return "Not a Time Exceeded";
        if (p.payload.size() < 4) return "Payload too short for Time Exceeded";
        const uint32_t u = ((uint32_t)detail::be16(p.payload.data()) << 16) | detail::be16(p.payload.data() + 2);
        return TimeExceededPacket{p.header, u, std::vector<uint8_t>(p.payload.begin() + 4, p.payload.end())};
    }
};
}  // namespace icmp
namespace icmpv6 {
template <uint8_t TYPE>
struct EchoPacket {  // echo_request (icmpv6.rs:2268-2294) / echo_reply (2427-2453): 8-B minimum
    Icmpv6Header header;
    uint16_t identifier = 0, sequence_number = 0;
    std::vector<uint8_t> payload;
    static Result<EchoPacket, const char*> try_from(const Icmpv6Packet& p) {
        if (p.header.icmpv6_type != TYPE)
            return TYPE == 128 ? "Not an Echo Request packet" : "Not an Echo Reply packet";
        if (p.payload.size() < 8) return TYPE == 128 ? "Payload too short for Echo Request" : "Payload too short for Echo Reply";
        return EchoPacket{p.header, detail::be16(p.payload.data()), detail::be16(p.payload.data() + 2),
                          std::vector<uint8_t>(p.payload.begin() + 4, p.payload.end())};
    }
    size_t total_len() const { return 8 + payload.size(); }
};
using EchoRequestPacket = EchoPacket<128>;
using EchoReplyPacket = EchoPacket<129>;

/* Neighbor Discovery messages (icmpv6.rs ndp, 640-1901), both ways the
 * reference builds them: try_from(Icmpv6Packet) is the TryFrom conversion
 * dump.rs uses (fixed part read from the packet payload, options in 8-B
 * chunks), from_bytes(message) is Packet::try_from_buf over the whole ICMPv6
 * message (type byte first; options walked by their length field, the rest
 * kept as payload) as the reference's ndp_tests call it. Quirks kept: RS / RA
 * from_bytes need 24 B and panic in the reference on a length-0 option (an
 * error here), NS / NA / Redirect stop there; TryFrom for NS asks a 24-B and
 * for Redirect a 40-B payload although their fixed parts are 20 / 36 B. */
namespace ndp {
struct NdpOptionPacket {  // icmpv6.rs:776-857
    uint8_t option_type = 0;
    uint8_t length = 0;  // unit: 8 bytes
    std::vector<uint8_t> payload;
    static Result<NdpOptionPacket, const char*> from_bytes(const uint8_t* b, size_t n) {  // icmpv6.rs:784-810
        if (n < 2) return "Malformed";
        const size_t total = (size_t)b[1] * 8;
        if (n < total) return "Malformed";
        if (total < 2) return "NDP option of length 0 (the reference underflows)";
        return NdpOptionPacket{b[0], b[1], std::vector<uint8_t>(b + 2, b + total)};
    }
    void append_to(std::vector<uint8_t>& out) const {  // icmpv6.rs:817-823
        out.push_back(option_type);
        out.push_back(length);
        out.insert(out.end(), payload.begin(), payload.end());
    }
};
namespace detail_ndp {
inline Result<std::vector<NdpOptionPacket>, const char*> chunks(const std::vector<uint8_t>& p, size_t from) {
    std::vector<NdpOptionPacket> out;  // TryFrom: 8-B chunks, type = chunk[0], length = chunk[1]
    for (size_t k = from; k < p.size(); k += 8) {
        const size_t e = k + 8 < p.size() ? k + 8 : p.size();
        if (e - k < 2) return "NDP option chunk of 1 byte (the reference panics)";
        out.push_back(NdpOptionPacket{p[k], p[k + 1], std::vector<uint8_t>(p.begin() + k + 2, p.begin() + e)});
    }
    return out;
}
// try_from_buf option walk from byte i; the rest becomes `rest`
inline const char* walk(const uint8_t* b, size_t n, size_t i, bool stop_short, std::vector<NdpOptionPacket>& out,
                        std::vector<uint8_t>& rest) {
    while (i + 2 <= n) {
        const size_t ol = (size_t)b[i + 1] * 8;
        if (stop_short && ol < 2) break;
        if (i + ol > n) break;
        if (ol < 2) return "NDP option of length 0 (the reference panics)";
        out.push_back(NdpOptionPacket{b[i], b[i + 1], std::vector<uint8_t>(b + i + 2, b + i + ol)});
        i += ol;
    }
    rest.assign(b + i, b + n);
    return nullptr;
}
inline uint32_t be32(const uint8_t* p) { return ((uint32_t)detail::be16(p) << 16) | detail::be16(p + 2); }
inline Ipv6Addr v6(const uint8_t* p) {
    Ipv6Addr a;
    memcpy(a.octets.data(), p, 16);
    return a;
}
inline void head(std::vector<uint8_t>& o, const Icmpv6Header& h) {
    o.push_back(h.icmpv6_type);
    o.push_back(h.icmpv6_code);
    o.push_back((uint8_t)(h.checksum >> 8));
    o.push_back((uint8_t)h.checksum);
}
inline void put32(std::vector<uint8_t>& o, uint32_t v) {
    for (int k = 3; k >= 0; k--) o.push_back((uint8_t)(v >> (8 * k)));
}
inline Icmpv6Header hdr(const uint8_t* b) { return Icmpv6Header{b[0], b[1], detail::be16(b + 2)}; }
}  // namespace detail_ndp

struct RouterSolicitPacket {  // icmpv6.rs:872-1023
    Icmpv6Header header;
    uint32_t reserved = 0;
    std::vector<NdpOptionPacket> options;
    std::vector<uint8_t> payload;
    static Result<RouterSolicitPacket, const char*> try_from(const Icmpv6Packet& p) {
        if (p.header.icmpv6_type != 133) return "Not a Router Solicitation packet";
        if (p.payload.size() < 8) return "Payload too short for Router Solicitation";
        auto o = detail_ndp::chunks(p.payload, 4);
        if (o.is_err()) return o.error();
        return RouterSolicitPacket{p.header, detail_ndp::be32(p.payload.data()), o.value(), {}};
    }
    static Result<RouterSolicitPacket, const char*> from_bytes(const uint8_t* b, size_t n) {
        if (n < 24) return "Malformed";  // NDP_SOL_PACKET_LEN
        RouterSolicitPacket m{detail_ndp::hdr(b), detail_ndp::be32(b + 4), {}, {}};
        if (const char* e = detail_ndp::walk(b, n, 8, false, m.options, m.payload)) return e;
        return m;
    }
    std::vector<uint8_t> to_bytes() const {
        std::vector<uint8_t> o;
        detail_ndp::head(o, header);
        detail_ndp::put32(o, reserved);
        for (const auto& x : options) x.append_to(o);
        return o;
    }
    size_t total_len() const { return 8 + 4 + payload.size(); }
};

struct RouterAdvertPacket {  // icmpv6.rs:1055-1234
    Icmpv6Header header;
    uint8_t hop_limit = 0, flags = 0;
    uint16_t lifetime = 0;
    uint32_t reachable_time = 0, retrans_time = 0;
    std::vector<NdpOptionPacket> options;
    std::vector<uint8_t> payload;
    static Result<RouterAdvertPacket, const char*> try_from(const Icmpv6Packet& p) {
        if (p.header.icmpv6_type != 134) return "Not a Router Advertisement packet";
        if (p.payload.size() < 16) return "Payload too short for Router Advertisement";
        auto o = detail_ndp::chunks(p.payload, 12);
        if (o.is_err()) return o.error();
        const uint8_t* q = p.payload.data();
        return RouterAdvertPacket{p.header, q[0], q[1], detail::be16(q + 2), detail_ndp::be32(q + 4),
                                  detail_ndp::be32(q + 8), o.value(), {}};
    }
    static Result<RouterAdvertPacket, const char*> from_bytes(const uint8_t* b, size_t n) {
        if (n < 24) return "Malformed";  // NDP_ADV_PACKET_LEN
        RouterAdvertPacket m{detail_ndp::hdr(b), b[4], b[5], detail::be16(b + 6), detail_ndp::be32(b + 8),
                             detail_ndp::be32(b + 12), {}, {}};
        if (const char* e = detail_ndp::walk(b, n, 16, false, m.options, m.payload)) return e;
        return m;
    }
    std::vector<uint8_t> to_bytes() const {
        std::vector<uint8_t> o;
        detail_ndp::head(o, header);
        o.push_back(hop_limit);
        o.push_back(flags);
        o.push_back((uint8_t)(lifetime >> 8));
        o.push_back((uint8_t)lifetime);
        detail_ndp::put32(o, reachable_time);
        detail_ndp::put32(o, retrans_time);
        for (const auto& x : options) x.append_to(o);
        return o;
    }
    size_t total_len() const { return 8 + 16 + payload.size(); }
};

struct NeighborSolicitPacket {  // icmpv6.rs:1258-1434
    Icmpv6Header header;
    uint32_t reserved = 0;
    Ipv6Addr target_addr;
    std::vector<NdpOptionPacket> options;
    std::vector<uint8_t> payload;
    static Result<NeighborSolicitPacket, const char*> try_from(const Icmpv6Packet& p) {
        if (p.header.icmpv6_type != 135) return "Not a Neighbor Solicitation packet";
        if (p.payload.size() < 24) return "Payload too short for Neighbor Solicitation";
        auto o = detail_ndp::chunks(p.payload, 20);
        if (o.is_err()) return o.error();
        return NeighborSolicitPacket{p.header, detail_ndp::be32(p.payload.data()), detail_ndp::v6(p.payload.data() + 4),
                                     o.value(), {}};
    }
    static Result<NeighborSolicitPacket, const char*> from_bytes(const uint8_t* b, size_t n) {
        if (n < 24) return "Malformed";
        NeighborSolicitPacket m{detail_ndp::hdr(b), detail_ndp::be32(b + 4), detail_ndp::v6(b + 8), {}, {}};
        if (const char* e = detail_ndp::walk(b, n, 24, true, m.options, m.payload)) return e;
        return m;
    }
    std::vector<uint8_t> to_bytes() const {
        std::vector<uint8_t> o;
        detail_ndp::head(o, header);
        detail_ndp::put32(o, reserved);
        o.insert(o.end(), target_addr.octets.begin(), target_addr.octets.end());
        for (const auto& x : options) x.append_to(o);
        return o;
    }
    size_t total_len() const { return 8 + 24 + payload.size(); }
};

struct NeighborAdvertPacket {  // icmpv6.rs:1472-1664
    Icmpv6Header header;
    uint8_t flags = 0;
    uint32_t reserved = 0;  // u24be
    Ipv6Addr target_addr;
    std::vector<NdpOptionPacket> options;
    std::vector<uint8_t> payload;
    static Result<NeighborAdvertPacket, const char*> try_from(const Icmpv6Packet& p) {
        if (p.header.icmpv6_type != 136) return "Not a Neighbor Advert packet";
        if (p.payload.size() < 20) return "Payload too short for Neighbor Advert";
        auto o = detail_ndp::chunks(p.payload, 20);
        if (o.is_err()) return o.error();
        const uint8_t* q = p.payload.data();
        return NeighborAdvertPacket{p.header, q[0], detail_ndp::be32(q) & 0xFFFFFFu, detail_ndp::v6(q + 4), o.value(), {}};
    }
    static Result<NeighborAdvertPacket, const char*> from_bytes(const uint8_t* b, size_t n) {
        if (n < 24) return "Malformed";
        NeighborAdvertPacket m{detail_ndp::hdr(b), b[4], detail_ndp::be32(b + 4) & 0xFFFFFFu, detail_ndp::v6(b + 8), {}, {}};
        if (const char* e = detail_ndp::walk(b, n, 24, true, m.options, m.payload)) return e;
        return m;
    }
    std::vector<uint8_t> to_bytes() const {
        std::vector<uint8_t> o;
        detail_ndp::head(o, header);
        detail_ndp::put32(o, (uint32_t)flags << 24 | (reserved & 0xFFFFFFu));
        o.insert(o.end(), target_addr.octets.begin(), target_addr.octets.end());
        for (const auto& x : options) x.append_to(o);
        return o;
    }
    size_t total_len() const { return 8 + 24 + payload.size(); }
};

struct RedirectPacket {  // icmpv6.rs:1696-1901
    Icmpv6Header header;
    uint32_t reserved = 0;
    Ipv6Addr target_addr, dest_addr;
    std::vector<NdpOptionPacket> options;
    std::vector<uint8_t> payload;
    static Result<RedirectPacket, const char*> try_from(const Icmpv6Packet& p) {
        if (p.header.icmpv6_type != 137) return "Not a Redirect packet";
        if (p.payload.size() < 40) return "Payload too short for Redirect";
        auto o = detail_ndp::chunks(p.payload, 36);
        if (o.is_err()) return o.error();
        const uint8_t* q = p.payload.data();
        return RedirectPacket{p.header, detail_ndp::be32(q), detail_ndp::v6(q + 4), detail_ndp::v6(q + 20), o.value(), {}};
    }
    static Result<RedirectPacket, const char*> from_bytes(const uint8_t* b, size_t n) {
        if (n < 40) return "Malformed";
        RedirectPacket m{detail_ndp::hdr(b), detail_ndp::be32(b + 4), detail_ndp::v6(b + 8), detail_ndp::v6(b + 24), {}, {}};
        if (const char* e = detail_ndp::walk(b, n, 40, true, m.options, m.payload)) return e;
        return m;
    }
    std::vector<uint8_t> to_bytes() const {
        std::vector<uint8_t> o;
        detail_ndp::head(o, header);
        detail_ndp::put32(o, reserved);
        o.insert(o.end(), target_addr.octets.begin(), target_addr.octets.end());
        o.insert(o.end(), dest_addr.octets.begin(), dest_addr.octets.end());
        for (const auto& x : options) x.append_to(o);
        return o;
    }
    size_t total_len() const { return 8 + 40 + payload.size(); }
};

// The whole ICMPv6 message of a Frame's Icmpv6Packet (header + payload),
// what from_bytes takes
inline std::vector<uint8_t> message_bytes(const Icmpv6Packet& p) {
    std::vector<uint8_t> o;
    detail_ndp::head(o, p.header);
    o.insert(o.end(), p.payload.begin(), p.payload.end());
    return o;
}
}  // namespace ndp
}  // namespace icmpv6

/* ---- the engine --------------------------------------------------------- */

// The calling thread's current device switched for a scope and restored after
// (Engine methods: scratch hipMalloc, copies and launches on the engine's device
// whatever device the caller has current).
struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(int d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != d) {
            const hipError_t e = hipSetDevice(d);
            if (e != hipSuccess) throw Error(std::string("hipSetDevice: ") + hipGetErrorString(e));
        }
    }
    ~DeviceScope() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
    DeviceScope(const DeviceScope&) = delete;
    DeviceScope& operator=(const DeviceScope&) = delete;
};

class Engine {  // one nexg context on one gfx950 device, one stream
   public:
    explicit Engine(int device = 0) : device_(device) {
        DeviceScope ds(device);
        check(nexg_ctx_create(device, &ctx_), "nexg_ctx_create");
        check_hip(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
    }
    ~Engine() {
        DeviceScope ds(device_);
        for (auto& b : scratch_) (void)hipFree(b.p);
        if (stream_) (void)hipStreamDestroy(stream_);
        if (ctx_) nexg_ctx_destroy(ctx_);
    }
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;

    nexg_ctx* ctx() const { return ctx_; }
    int device() const { return device_; }
    hipStream_t stream() const { return stream_; }

    // Device-resident batch (frames / out are device pointers), stream-ordered
    void parse(const nexg_frames& frames, ParseOption option, ParseMode mode, int out_kind, void* out) {
        DeviceScope ds(device_);
        const nexg_parse_option o{option.flags(mode), (uint32_t)option.offset};
        check(nexg_parse_batch(ctx_, &frames, &o, out_kind, out, stream_), "nexg_parse_batch");
    }

    // Frame::try_from_buf_with_mode (frame.rs:309) on every host frame: the
    // batch is packed, copied to the device, parsed (NEXG_OUT_RECORD), its
    // option lists decoded, and each Frame materialised from its record.
    std::vector<Result<Frame>> try_from_bufs(const std::vector<std::vector<uint8_t>>& frames,
                                             ParseOption option = {}, ParseMode mode = ParseMode::Lenient) {
        DeviceScope ds(device_);
        const uint64_t n = frames.size();
        std::vector<Result<Frame>> out;
        if (n == 0) return out;
        HostBatch hb(*this, frames);
        void* d_recs = scratch(3, n * 64);
        void* d_opts = scratch(4, n * 96);
        parse(hb.fb, option, mode, NEXG_OUT_RECORD, d_recs);
        check(nexg_decode_options(ctx_, &hb.fb, static_cast<const nexg_record*>(d_recs),
                                  static_cast<nexg_options*>(d_opts), stream_),
              "nexg_decode_options");
        std::vector<nexg_record> recs(n);
        std::vector<nexg_options> opts(n);
        check_hip(hipMemcpyAsync(recs.data(), d_recs, n * 64, hipMemcpyDeviceToHost, stream_), "D2H");
        check_hip(hipMemcpyAsync(opts.data(), d_opts, n * 96, hipMemcpyDeviceToHost, stream_), "D2H");
        check_hip(hipStreamSynchronize(stream_), "hipStreamSynchronize");
        out.reserve(n);
        for (uint64_t i = 0; i < n; i++)
            out.push_back(frame_from_record(recs[i], frames[i].data(), frames[i].size(), opts[i]));
        return out;
    }

    // FrameSlice::try_from_buf (frame.rs:86) on every host frame; the slices
    // borrow `frames`, which must outlive them
    std::vector<Result<FrameSlice>> frame_slices(const std::vector<std::vector<uint8_t>>& frames,
                                                 ParseOption option = {}) {
        DeviceScope ds(device_);
        const uint64_t n = frames.size();
        std::vector<Result<FrameSlice>> out;
        if (n == 0) return out;
        HostBatch hb(*this, frames);
        void* d_sl = scratch(3, n * 16);
        parse(hb.fb, option, ParseMode::Lenient, NEXG_OUT_SLICE, d_sl);
        std::vector<nexg_slice> sl(n);
        check_hip(hipMemcpyAsync(sl.data(), d_sl, n * 16, hipMemcpyDeviceToHost, stream_), "D2H");
        check_hip(hipStreamSynchronize(stream_), "hipStreamSynchronize");
        out.reserve(n);
        for (uint64_t i = 0; i < n; i++) out.push_back(frame_slice_from(sl[i], frames[i].data(), frames[i].size()));
        return out;
    }

    // The parse result of every host frame as nexg_desc (layers, checksum
    // verdicts, payload location: what Frame::try_from_buf reports, without
    // the header fields), through the grouped output the bench times
    // (NEXG_OUT_GROUPED: 17 B per 64 single-shape frames) decoded on the host
    std::vector<nexg_desc> descriptors(const std::vector<std::vector<uint8_t>>& frames, ParseOption option = {},
                                       ParseMode mode = ParseMode::Lenient) {
        DeviceScope ds(device_);
        const uint64_t n = frames.size();
        std::vector<nexg_desc> out(n);
        if (n == 0) return out;
        HostBatch hb(*this, frames);
        const uint64_t bytes = NEXG_GROUPED_BYTES(n);
        void* d_g = scratch(3, bytes);
        parse(hb.fb, option, mode, NEXG_OUT_GROUPED, d_g);
        std::vector<uint8_t> g(bytes);
        check_hip(hipMemcpyAsync(g.data(), d_g, bytes, hipMemcpyDeviceToHost, stream_), "D2H");
        check_hip(hipStreamSynchronize(stream_), "hipStreamSynchronize");
        const nexg_desc* exc = reinterpret_cast<const nexg_desc*>(g.data() + NEXG_GROUPED_EXC_OFFSET(n));
        const uint32_t fl = option.flags(mode);
        uint64_t kg = 0, kt = 0;  // exceptions so far in the frame's group / tile
        for (uint64_t i = 0; i < n; i++) {
            if ((i & 63u) == 0) kg = 0;
            if ((i & 255u) == 0) kt = 0;
            if (!nexg_sparse_decode(nexg_grouped_code(g.data(), n, i), (uint32_t)frames[i].size(), fl,
                                    (uint32_t)option.offset, &out[i])) {
                // (nexg_grouped_exc_slot, without its rescan of the run)
                const bool run = g[i >> 6] == NEXG_GROUPED_TILE_RUN;
                out[i] = exc[run ? (i & ~(uint64_t)255u) + kt : (i & ~(uint64_t)63u) + kg];
                kg++;
                kt++;
            }
        }
        return out;
    }

    // udp_ping's probe batch: one source address and port pair (udp_ping.rs:30-31,
    // 54-66) and a destination per target, identification 0 (the
    // Ipv4PacketBuilder default): the builder reads 4 B per frame
    Result<std::vector<std::vector<uint8_t>>, BuildError> build_udp_probes(const Ipv4Addr& source,
                                                                           const std::vector<Ipv4Addr>& targets,
                                                                           uint16_t src_port, uint16_t dst_port,
                                                                           const UdpPingShape& shape) {
        DeviceScope ds(device_);
        if (28ull + shape.payload.size() > 65535ull) return BuildError::LengthOverflow;
        const uint64_t n = targets.size();
        const uint32_t L = 42u + (uint32_t)shape.payload.size();
        if (n == 0) return std::vector<std::vector<uint8_t>>{};
        std::vector<uint32_t> dst(n);
        for (uint64_t i = 0; i < n; i++) {
            const auto& b = targets[i].octets;
            dst[i] = (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3];
        }
        void* d_dst = upload(6, dst.data(), n * 4);
        void* d_pl = shape.payload.empty() ? nullptr : upload(10, shape.payload.data(), shape.payload.size());
        void* d_out = scratch(11, (uint64_t)n * L);
        nexg_udp4_build p{};
        p.dst_ip = static_cast<const uint32_t*>(d_dst);
        p.def_src_ip = (uint32_t)source.octets[0] << 24 | (uint32_t)source.octets[1] << 16 |
                       (uint32_t)source.octets[2] << 8 | source.octets[3];
        p.def_src_port = src_port;
        p.def_dst_port = dst_port;
        p.payload = static_cast<const uint8_t*>(d_pl);
        p.payload_len = (uint32_t)shape.payload.size();
        memcpy(p.def_src_mac, shape.src_mac.data(), 6);
        memcpy(p.def_dst_mac, shape.dst_mac.data(), 6);
        p.ttl = shape.ttl;
        p.ip_flags = shape.ip_flags;
        p.count = n;
        check(nexg_build_udp4_batch(ctx_, &p, static_cast<uint8_t*>(d_out), L, stream_), "nexg_build_udp4_batch");
        return download_frames(d_out, n, L);
    }

    // udp_ping's build (udp_ping.rs:68-109) for every tuple: 42 + payload bytes
    // each; BuildError::LengthOverflow when the UDP / IPv4 length would pass
    // 65535 (builder/udp.rs:83, builder/ipv4.rs:153)
    Result<std::vector<std::vector<uint8_t>>, BuildError> build_udp_ping(const std::vector<UdpPingTuple>& t,
                                                                         const UdpPingShape& shape) {
        DeviceScope ds(device_);
        if (28ull + shape.payload.size() > 65535ull) return BuildError::LengthOverflow;
        const uint64_t n = t.size();
        const uint32_t L = 42u + (uint32_t)shape.payload.size();
        std::vector<std::vector<uint8_t>> frames;
        if (n == 0) return frames;
        // one 16-B record per tuple: a single H2D copy and one load per frame
        // on the device (nexg_build_udp4_tuples)
        std::vector<nexg_udp4_tuple> tup(n);
        for (uint64_t i = 0; i < n; i++) {
            const auto& a = t[i].source.octets;
            const auto& b = t[i].destination.octets;
            tup[i].src_ip = (uint32_t)a[0] << 24 | (uint32_t)a[1] << 16 | (uint32_t)a[2] << 8 | a[3];
            tup[i].dst_ip = (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3];
            tup[i].src_port = t[i].src_port;
            tup[i].dst_port = t[i].dst_port;
            tup[i].ip_id = t[i].ip_id;
            tup[i].reserved = 0;
        }
        void* d_tup = scratch(5, n * sizeof(nexg_udp4_tuple));
        void* d_pl = scratch(10, shape.payload.size());
        void* d_out = scratch(11, (uint64_t)n * L);
        check_hip(hipMemcpyAsync(d_tup, tup.data(), n * sizeof(nexg_udp4_tuple), hipMemcpyHostToDevice, stream_),
                  "H2D");
        if (!shape.payload.empty())
            check_hip(hipMemcpyAsync(d_pl, shape.payload.data(), shape.payload.size(), hipMemcpyHostToDevice,
                                     stream_), "H2D");
        nexg_udp4_build p{};
        p.payload = shape.payload.empty() ? nullptr : static_cast<const uint8_t*>(d_pl);
        p.payload_len = (uint32_t)shape.payload.size();
        memcpy(p.def_src_mac, shape.src_mac.data(), 6);
        memcpy(p.def_dst_mac, shape.dst_mac.data(), 6);
        p.ttl = shape.ttl;
        p.ip_flags = shape.ip_flags;
        p.count = n;
        check(nexg_build_udp4_tuples(ctx_, &p, static_cast<const nexg_udp4_tuple*>(d_tup),
                                     static_cast<uint8_t*>(d_out), L, stream_), "nexg_build_udp4_tuples");
        std::vector<uint8_t> host((uint64_t)n * L);
        check_hip(hipMemcpyAsync(host.data(), d_out, host.size(), hipMemcpyDeviceToHost, stream_), "D2H");
        check_hip(hipStreamSynchronize(stream_), "hipStreamSynchronize");
        frames.reserve(n);
        for (uint64_t i = 0; i < n; i++) frames.emplace_back(host.begin() + i * L, host.begin() + (i + 1) * L);
        return frames;
    }

    // tcp_ping's build for every tuple (one address family per batch:
    // BuildError::AddressFamilyMismatch otherwise, builder/error.rs)
    Result<std::vector<std::vector<uint8_t>>, BuildError> build_tcp_ping(const std::vector<TcpPingTuple>& t,
                                                                         const TcpPingShape& shape) {
        DeviceScope ds(device_);
        std::vector<std::vector<uint8_t>> frames;
        if (t.empty()) return frames;
        if (shape.options.size() > 40) return BuildError::LengthOverflow;
        const uint8_t fam = t[0].source.family;
        for (const auto& x : t)
            if (x.source.family != fam || x.destination.family != fam) return BuildError::AddressFamilyMismatch;
        const uint64_t n = t.size();
        const uint32_t L = 14u + (fam == 4 ? 20u : 40u) + 20u + (((uint32_t)shape.options.size() + 3u) & ~3u) +
                           (uint32_t)shape.payload.size();
        nexg_tcp_build p{};
        fill_ip(p.ip, t, shape.src_mac, shape.dst_mac, fam, shape.ttl, shape.ip_flags, shape.tos, shape.flow_label, 5);
        std::vector<uint16_t> sp(n), dp(n);
        std::vector<uint32_t> seq(n), ack(n);
        for (uint64_t i = 0; i < n; i++) {
            sp[i] = t[i].src_port;
            dp[i] = t[i].dst_port;
            seq[i] = t[i].sequence;
            ack[i] = t[i].acknowledgement;
        }
        p.src_port = static_cast<const uint16_t*>(upload(10, sp.data(), n * 2));
        p.dst_port = static_cast<const uint16_t*>(upload(11, dp.data(), n * 2));
        p.seq = static_cast<const uint32_t*>(upload(12, seq.data(), n * 4));
        p.ack = static_cast<const uint32_t*>(upload(13, ack.data(), n * 4));
        p.payload = shape.payload.empty() ? nullptr
                                          : static_cast<const uint8_t*>(upload(14, shape.payload.data(), shape.payload.size()));
        p.payload_len = (uint32_t)shape.payload.size();
        p.window = shape.window;
        p.urgent_ptr = shape.urgent_ptr;
        p.flags = shape.flags;
        p.options_len = (uint8_t)shape.options.size();
        if (!shape.options.empty()) memcpy(p.options, shape.options.data(), shape.options.size());
        p.count = n;
        void* d_out = scratch(15, n * L);
        const int rc = nexg_build_tcp_batch(ctx_, &p, static_cast<uint8_t*>(d_out), L, stream_);
        if (rc == NEXG_ERANGE) return BuildError::LengthOverflow;
        check(rc, "nexg_build_tcp_batch");
        return download_frames(d_out, n, L);
    }

    // icmp_ping's echo request for every tuple (EchoRequest 8 / ICMPv6 128, code 0)
    Result<std::vector<std::vector<uint8_t>>, BuildError> build_icmp_ping(const std::vector<IcmpPingTuple>& t,
                                                                          const IcmpPingShape& shape) {
        DeviceScope ds(device_);
        std::vector<std::vector<uint8_t>> frames;
        if (t.empty()) return frames;
        const uint8_t fam = t[0].source.family;
        for (const auto& x : t)
            if (x.source.family != fam || x.destination.family != fam) return BuildError::AddressFamilyMismatch;
        const uint64_t n = t.size();
        const uint32_t L = 14u + (fam == 4 ? 20u : 40u) + 8u + (uint32_t)shape.payload.size();
        nexg_icmp_echo_build p{};
        fill_ip(p.ip, t, shape.src_mac, shape.dst_mac, fam, shape.ttl, shape.ip_flags, shape.tos, shape.flow_label, 5);
        std::vector<uint16_t> id(n), sq(n);
        for (uint64_t i = 0; i < n; i++) {
            id[i] = t[i].identifier;
            sq[i] = t[i].sequence;
        }
        p.identifier = static_cast<const uint16_t*>(upload(10, id.data(), n * 2));
        p.sequence = static_cast<const uint16_t*>(upload(11, sq.data(), n * 2));
        p.payload = shape.payload.empty() ? nullptr
                                          : static_cast<const uint8_t*>(upload(14, shape.payload.data(), shape.payload.size()));
        p.payload_len = (uint32_t)shape.payload.size();
        p.icmp_type = fam == 4 ? 8 : 128;
        p.icmp_code = 0;
        p.count = n;
        void* d_out = scratch(15, n * L);
        const int rc = nexg_build_icmp_echo_batch(ctx_, &p, static_cast<uint8_t*>(d_out), L, stream_);
        if (rc == NEXG_ERANGE) return BuildError::LengthOverflow;
        check(rc, "nexg_build_icmp_echo_batch");
        return download_frames(d_out, n, L);
    }

    // an ARP request for every target (nexg_build_arp_batch)
    Result<std::vector<std::vector<uint8_t>>, BuildError> build_arp_requests(const std::vector<Ipv4Addr>& targets,
                                                                             const ArpProbeShape& shape) {
        DeviceScope ds(device_);
        std::vector<std::vector<uint8_t>> frames;
        if (shape.hw_addr_len != 6 || shape.proto_addr_len != 4) return BuildError::InvalidFieldLength;
        if (targets.empty()) return frames;
        const uint64_t n = targets.size();
        std::vector<uint8_t> tip(n * 4);
        for (uint64_t i = 0; i < n; i++) memcpy(tip.data() + 4 * i, targets[i].octets.data(), 4);
        nexg_arp_build p{};
        p.target_ip = static_cast<const uint8_t*>(upload(16, tip.data(), tip.size()));
        memcpy(p.def_sender_ip, shape.sender_ip.octets.data(), 4);
        memcpy(p.def_sender_mac, shape.sender_mac.data(), 6);
        memcpy(p.def_eth_dst, shape.eth_dst.data(), 6);
        p.hardware_type = 1;
        p.protocol_type = 0x0800;
        p.operation = shape.operation;
        p.hw_addr_len = shape.hw_addr_len;
        p.proto_addr_len = shape.proto_addr_len;
        p.count = n;
        void* d_out = scratch(15, n * 42);
        check(nexg_build_arp_batch(ctx_, &p, static_cast<uint8_t*>(d_out), 42, stream_), "nexg_build_arp_batch");
        return download_frames(d_out, n, 42);
    }

    // an NDP neighbor solicitation for every target (nexg_build_ndp_ns_batch)
    std::vector<std::vector<uint8_t>> build_ndp_solicits(const std::vector<Ipv6Addr>& targets,
                                                         const NdpProbeShape& shape) {
        DeviceScope ds(device_);
        if (targets.empty()) return {};
        const uint64_t n = targets.size();
        std::vector<uint8_t> src(n * 16), dst(n * 16);
        for (uint64_t i = 0; i < n; i++) {
            memcpy(src.data() + 16 * i, shape.src_ip.octets.data(), 16);
            memcpy(dst.data() + 16 * i, targets[i].octets.data(), 16);
        }
        nexg_ndp_ns_build p{};
        p.ip.src_ip = static_cast<const uint8_t*>(upload(16, src.data(), src.size()));
        p.ip.dst_ip = static_cast<const uint8_t*>(upload(17, dst.data(), dst.size()));
        p.ip.family = 6;
        memcpy(p.ip.def_src_mac, shape.src_mac.data(), 6);
        p.ip.ttl = shape.hop_limit;
        p.eth_dst_multicast = 1;
        p.count = n;
        void* d_out = scratch(15, n * 86);
        check(nexg_build_ndp_ns_batch(ctx_, &p, static_cast<uint8_t*>(d_out), 86, stream_), "nexg_build_ndp_ns_batch");
        return download_frames(d_out, n, 86);
    }

    // Mutable{Ipv4,Udp,Tcp,Icmp,Icmpv6}Packet::recompute_checksum over every
    // frame's raw buffer (ipv4.rs:669-679, udp.rs:338-369, tcp.rs:1009-1040,
    // icmp.rs:372-377, icmpv6.rs:450-470), chained as mutable_chaining.rs:
    // the frames are rewritten in place; one nexg_fixup per frame says which
    // fields were written (which = NEXG_FIX_IP | NEXG_FIX_L4)
    std::vector<nexg_fixup> recompute_checksums(std::vector<std::vector<uint8_t>>& frames, ParseOption option = {},
                                                uint32_t which = NEXG_FIX_IP | NEXG_FIX_L4) {
        DeviceScope ds(device_);
        const uint64_t n = frames.size();
        std::vector<nexg_fixup> fx(n);
        if (n == 0) return fx;
        HostBatch hb(*this, frames);
        void* d_fx = scratch(3, n * sizeof(nexg_fixup));
        const nexg_parse_option o{option.flags(ParseMode::Lenient), (uint32_t)option.offset};
        check(nexg_recompute_checksums_batch(ctx_, &hb.fb, &o, which, static_cast<nexg_fixup*>(d_fx), stream_),
              "nexg_recompute_checksums_batch");
        std::vector<uint8_t> data(hb.data.size());
        check_hip(hipMemcpyAsync(data.data(), const_cast<uint8_t*>(hb.fb.data), data.size(), hipMemcpyDeviceToHost,
                                 stream_), "D2H");
        check_hip(hipMemcpyAsync(fx.data(), d_fx, n * sizeof(nexg_fixup), hipMemcpyDeviceToHost, stream_), "D2H");
        check_hip(hipStreamSynchronize(stream_), "hipStreamSynchronize");
        for (uint64_t i = 0; i < n; i++)
            std::copy(data.begin() + hb.offs[i], data.begin() + hb.offs[i] + hb.lens[i], frames[i].begin());
        return fx;
    }

   private:
    void* upload(size_t slot, const void* src, size_t n) {
        void* d = scratch(slot, n);
        if (n) check_hip(hipMemcpyAsync(d, src, n, hipMemcpyHostToDevice, stream_), "H2D");
        return d;
    }
    std::vector<std::vector<uint8_t>> download_frames(const void* d_out, uint64_t n, uint32_t L) {
        std::vector<uint8_t> host(n * L);
        check_hip(hipMemcpyAsync(host.data(), d_out, host.size(), hipMemcpyDeviceToHost, stream_), "D2H");
        check_hip(hipStreamSynchronize(stream_), "hipStreamSynchronize");
        std::vector<std::vector<uint8_t>> frames;
        frames.reserve(n);
        for (uint64_t i = 0; i < n; i++) frames.emplace_back(host.begin() + i * L, host.begin() + (i + 1) * L);
        return frames;
    }
    // per-tuple addresses / ids into nexg_ip_build (scratch slots first .. first+2)
    template <class Tuple>
    void fill_ip(nexg_ip_build& ip, const std::vector<Tuple>& t, const MacAddr& smac, const MacAddr& dmac,
                 uint8_t fam, uint8_t ttl, uint8_t ip_flags, uint8_t tos, uint32_t flow_label, size_t first) {
        const size_t w = fam == 4 ? 4 : 16;
        std::vector<uint8_t> src(t.size() * w), dst(t.size() * w);
        std::vector<uint16_t> id(t.size());
        for (size_t i = 0; i < t.size(); i++) {
            memcpy(src.data() + i * w, t[i].source.octets.data(), w);
            memcpy(dst.data() + i * w, t[i].destination.octets.data(), w);
            id[i] = t[i].ip_id;
        }
        ip.src_ip = static_cast<const uint8_t*>(upload(first, src.data(), src.size()));
        ip.dst_ip = static_cast<const uint8_t*>(upload(first + 1, dst.data(), dst.size()));
        ip.ip_id = fam == 4 ? static_cast<const uint16_t*>(upload(first + 2, id.data(), id.size() * 2)) : nullptr;
        ip.family = fam;
        ip.flow_label = flow_label;
        memcpy(ip.def_src_mac, smac.data(), 6);
        memcpy(ip.def_dst_mac, dmac.data(), 6);
        ip.ttl = ttl;
        ip.ip_flags = ip_flags;
        ip.tos = tos;
    }
    // grow-only device scratch, one buffer per slot: every call ends with a
    // stream sync, so the next call may reuse them (no hipMalloc per batch)
    struct Scratch {
        void* p = nullptr;
        size_t size = 0;
    };
    std::vector<Scratch> scratch_;
    int device_ = 0;
    void* scratch(size_t slot, size_t n) {
        if (slot >= scratch_.size()) scratch_.resize(slot + 1);
        Scratch& b = scratch_[slot];
        if (b.size < n || !b.p) {
            if (b.p) (void)hipFree(b.p);
            b.p = nullptr;
            b.size = 0;
            check_hip(hipMalloc(&b.p, n ? n : 16), "hipMalloc");
            b.size = n ? n : 16;
        }
        return b.p;
    }
    // host frames packed (4-B aligned starts) with offsets + lengths, on the device
    struct HostBatch {
        std::vector<uint8_t> data;
        std::vector<uint64_t> offs;
        std::vector<uint32_t> lens;
        nexg_frames fb{};
        HostBatch(Engine& e, const std::vector<std::vector<uint8_t>>& frames)
            : offs(frames.size()), lens(frames.size()) {
            uint64_t pos = 0;
            for (size_t i = 0; i < frames.size(); i++) {
                offs[i] = pos;
                lens[i] = (uint32_t)frames[i].size();
                pos += (frames[i].size() + 3) & ~(uint64_t)3;
            }
            data.assign(pos ? pos : 16, 0);
            for (size_t i = 0; i < frames.size(); i++)
                if (!frames[i].empty()) memcpy(data.data() + offs[i], frames[i].data(), frames[i].size());
            void* d_data = e.scratch(0, data.size());
            void* d_offs = e.scratch(1, offs.size() * 8);
            void* d_lens = e.scratch(2, lens.size() * 4);
            check_hip(hipMemcpyAsync(d_data, data.data(), data.size(), hipMemcpyHostToDevice, e.stream_), "H2D");
            check_hip(hipMemcpyAsync(d_offs, offs.data(), offs.size() * 8, hipMemcpyHostToDevice, e.stream_), "H2D");
            check_hip(hipMemcpyAsync(d_lens, lens.data(), lens.size() * 4, hipMemcpyHostToDevice, e.stream_), "H2D");
            fb.data = static_cast<const uint8_t*>(d_data);
            fb.data_bytes = data.size();
            fb.offsets = static_cast<const uint64_t*>(d_offs);
            fb.lengths = static_cast<const uint32_t*>(d_lens);
            fb.count = frames.size();
        }
    };

   public:
    Result<Frame> try_from_buf(const std::vector<uint8_t>& frame, ParseOption option = {},
                               ParseMode mode = ParseMode::Lenient) {
        return std::move(try_from_bufs({frame}, option, mode)[0]);
    }

   private:
    void check(int rc, const char* what) {
        if (rc != NEXG_OK)
            throw Error(std::string(what) + " failed: " + (ctx_ ? nexg_ctx_last_error(ctx_) : "no context"));
    }
    static void check_hip(hipError_t e, const char* what) {
        if (e != hipSuccess) throw Error(std::string(what) + ": " + hipGetErrorString(e));
    }
    nexg_ctx* ctx_ = nullptr;
    hipStream_t stream_ = nullptr;
};

/* ---- capture-file source (nexg_pcap_*; pcap::from_file, pcap.rs:95-109) -- */

class PcapReader {  // classic pcap / pcapng, a batch of records per call
   public:
    explicit PcapReader(const std::string& path) {
        if (nexg_pcap_open(path.c_str(), &p_) != NEXG_OK) throw Error("cannot open " + path + " as pcap/pcapng");
    }
    ~PcapReader() {
        if (p_) nexg_pcap_close(p_);
    }
    PcapReader(const PcapReader&) = delete;
    PcapReader& operator=(const PcapReader&) = delete;

    int linktype() const { return nexg_pcap_linktype(p_); }  // 1 Ethernet, 101 raw IP
    // ParseOption a capture of this link type needs (raw IP: from_ip_packet, offset 0)
    ParseOption parse_option() const {
        ParseOption o;
        o.from_ip_packet = linktype() == 101;
        return o;
    }
    // up to max_frames records (fewer at the end of the file, none after it);
    // throws on a malformed file after the complete records before the damage
    std::vector<std::vector<uint8_t>> next_batch(uint64_t max_frames, uint64_t data_cap = 64u << 20) {
        buf_.resize(data_cap);
        offs_.resize(max_frames + 1);
        uint64_t n = 0;
        if (nexg_pcap_read_batch(p_, buf_.data(), buf_.size(), offs_.data(), max_frames, nullptr, &n) != NEXG_OK)
            throw Error(std::string("capture read failed: ") + nexg_pcap_last_error(p_));
        std::vector<std::vector<uint8_t>> frames(n);
        for (uint64_t i = 0; i < n; i++) frames[i].assign(buf_.begin() + offs_[i], buf_.begin() + offs_[i + 1]);
        return frames;
    }

    // Zero-copy shape (nexg_pcap_map / nexg_pcap_walk_mapped): the file's
    // page-cache mapping (valid while the reader lives) and the records of
    // one window of it, described in place; register the mapping for DMA
    // (hipHostRegister) and copy [from, next) to the device as is.
    struct MappedWindow {
        uint64_t from = 0, next = 0;     // file range of the complete records
        std::vector<uint64_t> offsets;  // relative to from
        std::vector<uint32_t> lengths;
    };
    const uint8_t* map(uint64_t* size, uint64_t* first) {
        const uint8_t* d = nullptr;
        if (nexg_pcap_map(p_, &d, size, first) != NEXG_OK)
            throw Error(std::string("capture map failed: ") + nexg_pcap_last_error(p_));
        return d;
    }
    // records of [pos, pos + max_bytes); pos advances past them (end of file: pos == size)
    MappedWindow walk_mapped(uint64_t& pos, uint64_t max_bytes, uint64_t max_frames) {
        MappedWindow w;
        w.from = pos;
        w.offsets.resize(max_frames);
        w.lengths.resize(max_frames);
        uint64_t n = 0;
        if (nexg_pcap_walk_mapped(p_, pos, max_bytes, w.offsets.data(), w.lengths.data(), max_frames, nullptr, &n,
                                  &w.next) != NEXG_OK)
            throw Error(std::string("capture walk failed: ") + nexg_pcap_last_error(p_));
        w.offsets.resize(n);
        w.lengths.resize(n);
        pos = w.next;
        return w;
    }

   private:
    nexg_pcap* p_ = nullptr;
    std::vector<uint8_t> buf_;
    std::vector<uint64_t> offs_;
};

/* ---- live datalink (nexg_rx_* / nexg_tx_*; nex-datalink's Linux channel) -- */

namespace datalink {

enum class FanoutType : uint32_t {  // lib.rs:70-90
    HASH = NEXG_FANOUT_HASH, LB = NEXG_FANOUT_LB, CPU = NEXG_FANOUT_CPU,
    ROLLOVER = NEXG_FANOUT_ROLLOVER, RND = NEXG_FANOUT_RND, QM = NEXG_FANOUT_QM
};
struct FanoutOption {  // lib.rs:92-131
    uint16_t group_id = 0;
    FanoutType fanout_type = FanoutType::HASH;
    bool defrag = false, rollover = false;
};
struct Config {  // lib.rs:229-240 (the Linux knobs) + the batch ring
    uint32_t read_buffer_size = 4096;
    int32_t read_timeout_ms = -1;  // read_timeout: None
    bool promiscuous = true;
    bool has_fanout = false;
    FanoutOption linux_fanout{};
    uint32_t mode = NEXG_RX_RING;  // or NEXG_RX_MMSG
    uint32_t ring_block_size = 1u << 20, ring_blocks = 64, ring_block_tov_ms = 2;
    bool skip_outgoing = false;
};

// RawReceiver::next (linux.rs:356-397), a batch of frames per call
class RawReceiver {
   public:
    RawReceiver(const std::string& ifname, const Config& c = {}) {
        nexg_rx_config k;
        nexg_rx_config_default(&k);
        k.read_buffer_size = c.read_buffer_size;
        k.read_timeout_ms = c.read_timeout_ms;
        k.promiscuous = c.promiscuous;
        k.fanout = c.has_fanout;
        k.fanout_type = (uint32_t)c.linux_fanout.fanout_type | (c.linux_fanout.defrag ? NEXG_FANOUT_FLAG_DEFRAG : 0u) |
                        (c.linux_fanout.rollover ? NEXG_FANOUT_FLAG_ROLLOVER : 0u);
        k.fanout_group = c.linux_fanout.group_id;
        k.mode = c.mode;
        k.ring_block_size = c.ring_block_size;
        k.ring_blocks = c.ring_blocks;
        k.ring_block_tov_ms = c.ring_block_tov_ms;
        k.flags = c.skip_outgoing ? NEXG_RX_SKIP_OUTGOING : 0u;
        const int rc = nexg_rx_open(ifname.c_str(), &k, &rx_);
        if (rc != NEXG_OK) throw Error("nexg_rx_open(" + ifname + "): " + nexg_strerror(rc));
    }
    ~RawReceiver() {
        if (rx_) nexg_rx_close(rx_);
    }
    RawReceiver(const RawReceiver&) = delete;
    RawReceiver& operator=(const RawReceiver&) = delete;
    // frames already received (waits up to the read timeout for the first)
    std::vector<std::vector<uint8_t>> next_batch(uint64_t max_frames = 4096, uint64_t data_cap = 16u << 20) {
        buf_.resize(data_cap);
        offs_.resize(max_frames + 1);
        uint64_t n = 0;
        const int rc = nexg_rx_next_batch(rx_, buf_.data(), buf_.size(), offs_.data(), max_frames, nullptr, &n);
        if (rc != NEXG_OK) throw Error(std::string("nexg_rx_next_batch: ") + nexg_strerror(rc));
        std::vector<std::vector<uint8_t>> frames(n);
        for (uint64_t i = 0; i < n; i++) frames[i].assign(buf_.begin() + offs_[i], buf_.begin() + offs_[i + 1]);
        return frames;
    }
    nexg_rx* handle() const { return rx_; }

   private:
    nexg_rx* rx_ = nullptr;
    std::vector<uint8_t> buf_;
    std::vector<uint64_t> offs_;
};

// RawSender::send (linux.rs:302-346), a batch per call (sendmmsg)
class RawSender {
   public:
    explicit RawSender(const std::string& ifname) {
        const int rc = nexg_tx_open(ifname.c_str(), &tx_);
        if (rc != NEXG_OK) throw Error("nexg_tx_open(" + ifname + "): " + nexg_strerror(rc));
    }
    ~RawSender() {
        if (tx_) nexg_tx_close(tx_);
    }
    RawSender(const RawSender&) = delete;
    RawSender& operator=(const RawSender&) = delete;
    // frames the kernel accepted
    uint64_t send_batch(const std::vector<std::vector<uint8_t>>& frames) {
        std::vector<uint8_t> data;
        std::vector<uint64_t> offs(frames.size() + 1, 0);
        for (size_t i = 0; i < frames.size(); i++) {
            data.insert(data.end(), frames[i].begin(), frames[i].end());
            offs[i + 1] = data.size();
        }
        uint64_t sent = 0;
        const int rc = nexg_tx_send_batch(tx_, data.data(), offs.data(), nullptr, 0, frames.size(), &sent);
        if (rc != NEXG_OK) throw Error(std::string("nexg_tx_send_batch: ") + nexg_strerror(rc));
        return sent;
    }

   private:
    nexg_tx* tx_ = nullptr;
};

}  // namespace datalink

}  // namespace nexg

#endif  // NEXG_HPP
