// TEST INFRASTRUCTURE: the C++ host API (include/nexg.hpp) checked with the
// reference's own unit-test assertions, written as the reference writes them
// (frame.rs:665-784, ipv4.rs:944-1204, ipv6.rs:706-741, tcp.rs:1276-1314,
// udp.rs:511-527, icmp.rs:708-725, icmpv6.rs:606-631). Frames come from
// tests/golden/reference_vectors.json via a text fixture (name flags
// ip_offset hex per line) the pytest writes.
//   --gpu <fixture>: Frames from nexg::Engine::try_from_bufs (the device path)
//   --cpu <fixture>: Frames materialised by nexg::frame_from_record from the
//                    oracle's records (checks the C++ materialisation without
//                    a GPU; the oracle is test infrastructure)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <unistd.h>

#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/nexg.hpp"
#include "../../oracle/nex_oracle.h"

using namespace nexg;

static int failures = 0, checks = 0;
#define CHECK(c)                                                                  \
    do {                                                                          \
        checks++;                                                                 \
        if (!(c)) { failures++; fprintf(stderr, "%s:%d: CHECK(%s) failed\n", __FILE__, __LINE__, #c); } \
    } while (0)

struct Fixture {
    uint32_t flags = 0, ip_offset = 0;
    std::vector<uint8_t> bytes;
};

static std::vector<uint8_t> hex(const std::string& s) {
    std::vector<uint8_t> b;
    for (size_t i = 0; i + 1 < s.size(); i += 2) b.push_back((uint8_t)strtoul(s.substr(i, 2).c_str(), nullptr, 16));
    return b;
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const bool gpu = std::string(argv[1]) == "--gpu";
    std::map<std::string, Fixture> fx;
    std::ifstream in(argv[2]);
    std::string line;
    while (std::getline(in, line)) {
        std::istringstream ss(line);
        std::string name, h;
        Fixture f;
        ss >> name >> f.flags >> f.ip_offset >> h;
        f.bytes = hex(h);
        fx[name] = f;
    }
    std::vector<std::string> names;
    std::vector<std::vector<uint8_t>> frames;
    for (auto& kv : fx) {
        names.push_back(kv.first);
        frames.push_back(kv.second.bytes);
    }
    // Frame::try_from_buf_with_mode per fixture, in its own ParseOption/ParseMode
    std::map<std::string, Result<Frame>> got;
    std::unique_ptr<Engine> eng;
    if (gpu) eng.reset(new Engine(0));
    for (size_t i = 0; i < names.size(); i++) {
        const Fixture& f = fx[names[i]];
        ParseOption opt;
        opt.from_ip_packet = (f.flags & NEXG_PARSE_FROM_IP) != 0;
        opt.offset = f.ip_offset;
        const ParseMode mode = (f.flags & NEXG_PARSE_STRICT) ? ParseMode::Strict : ParseMode::Lenient;
        if (gpu) {
            got.emplace(names[i], eng->try_from_buf(f.bytes, opt, mode));
        } else {
            nexg_record r;
            nexg_options o;
            nexo_parse_frame(f.bytes.data(), f.bytes.size(), f.flags, f.ip_offset, &r);
            nexo_decode_options(f.bytes.data(), f.bytes.size(), f.flags, f.ip_offset, &o);
            got.emplace(names[i], frame_from_record(r, f.bytes.data(), f.bytes.size(), o));
        }
    }
    auto frame = [&](const char* n) -> const Frame& {
        const auto& r = got.at(n);
        if (r.is_err()) { fprintf(stderr, "%s: unexpected %s\n", n, r.error().name()); exit(1); }
        return r.value();
    };
    auto bytes = [](const char* s) { return std::vector<uint8_t>(s, s + strlen(s)); };

    {  // ethernet.rs:458-476, 510-539
        const Frame& f = frame("ethernet_parse_basic");
        CHECK(f.datalink->ethernet->destination == (MacAddr{0xaa, 0xbb, 0xcc, 0xdd, 0xee, 0xff}));
        CHECK(f.datalink->ethernet->source == (MacAddr{0x11, 0x22, 0x33, 0x44, 0x55, 0x66}));
        CHECK(f.datalink->ethernet->ethertype == 0x0800);
        const auto& s = got.at("ethernet_too_short");
        CHECK(s.is_err() && s.error().kind == ParseErrorKind::BufferTooShort);
        // ethernet.rs:513-520: BufferTooShort { "Ethernet packet", minimum 14, actual 4 }
        CHECK(s.error().context && std::string(s.error().context) == "Ethernet packet");
        CHECK(s.error().minimum == 14 && s.error().actual == 4);
        const Frame& u = frame("ethernet_unknown_ethertype_dead");
        CHECK(u.datalink->ethernet->ethertype == 0xdead && !u.ip);
    }
    {  // ipv6.rs:672-704 header fields; icmpv6.rs:2531-2549 echo request
        const Frame& f = frame("ipv6_basic_header_fields");
        const auto& h = *f.ip->ipv6;
        CHECK(h.version == 6 && h.traffic_class == 0xaa && h.flow_label == 0x12345);
        CHECK(h.payload_length == 0 && h.next_header == 17 && h.hop_limit == 64);
        CHECK(h.source.octets[15] == 1 && h.destination == Ipv6Addr{});
        const Frame& e = frame("icmpv6_echo_request_parse");
        CHECK(e.ip->icmpv6 && e.ip->icmpv6->icmpv6_type == 128 && e.ip->icmpv6->icmpv6_code == 0);
        CHECK(e.ip->icmpv6->checksum == 0xbeef);
        CHECK(e.payload.size() == 9 && e.payload[0] == 0x12 && e.payload[1] == 0x34 && e.payload[2] == 0x56 &&
              e.payload[3] == 0x78 && e.payload[4] == 'p');
        // icmpv6.rs:2531-2549: EchoRequestPacket id 0x1234, seq 0x5678, payload "ping!"
        const auto er = icmpv6::EchoRequestPacket::try_from(*icmpv6_packet(e));
        CHECK(er.is_ok() && er.value().identifier == 0x1234 && er.value().sequence_number == 0x5678);
        CHECK(er.is_ok() && er.value().payload == bytes("ping!"));
        CHECK(icmpv6::EchoReplyPacket::try_from(*icmpv6_packet(e)).is_err());
    }
    {  // icmp.rs:708-815: the sub-message views dump.rs downcasts to
        const auto rq = icmp::EchoRequestPacket::try_from(*icmp_packet(frame("icmp_echo_request")));
        CHECK(rq.is_ok() && rq.value().identifier == 1234 && rq.value().sequence_number == 42);
        CHECK(rq.is_ok() && rq.value().payload == bytes("ping") && rq.value().header.checksum == 0x3abc);
        const auto rp = icmp::EchoReplyPacket::try_from(*icmp_packet(frame("icmp_echo_reply_roundtrip")));
        CHECK(rp.is_ok() && rp.value().identifier == 5678 && rp.value().sequence_number == 99);
        CHECK(rp.is_ok() && rp.value().payload == bytes("pong"));
        const auto du = icmp::DestinationUnreachablePacket::try_from(*icmp_packet(frame("icmp_destination_unreachable")));
        CHECK(du.is_ok() && du.value().next_hop_mtu == 1500 && du.value().payload == bytes("bad ip"));
        const auto te = icmp::TimeExceededPacket::try_from(*icmp_packet(frame("icmp_time_exceeded")));
        CHECK(te.is_ok() && te.value().unused == 0xdeadbeefu && te.value().payload == bytes("timeout"));
        CHECK(icmp::TimeExceededPacket::try_from(*icmp_packet(frame("icmp_echo_request"))).is_err());
        CHECK(std::string(icmp::EchoReplyPacket::try_from(*icmp_packet(frame("icmp_echo_request"))).error()) ==
              "Not an Echo Reply");
    }
    {  // icmpv6.rs ndp_tests (1922-2171): the messages decoded from the Frame's ICMPv6 packet
        using namespace icmpv6::ndp;
        const Ipv6Addr ff02_1{{0xff, 0x02, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1}};
        auto msg = [&](const char* n) { return message_bytes(*icmpv6_packet(frame(n))); };
        {  // basic_rs_parse
            const auto m = msg("icmpv6_ndp_router_solicit");
            const auto rs = RouterSolicitPacket::from_bytes(m.data(), m.size());
            CHECK(rs.is_ok() && rs.value().header.icmpv6_type == 133 && rs.value().header.icmpv6_code == 0);
            CHECK(rs.is_ok() && rs.value().header.checksum == 0 && rs.value().reserved == 0);
            CHECK(rs.is_ok() && rs.value().options.size() == 2);
            CHECK(rs.is_ok() && rs.value().options[0].option_type == 2 && rs.value().options[0].length == 1);
            CHECK(rs.is_ok() && rs.value().options[0].payload == std::vector<uint8_t>(6, 0));
            CHECK(rs.is_ok() && rs.value().options[1].option_type == 1 && rs.value().options[1].length == 1);
            CHECK(rs.is_ok() && rs.value().to_bytes() == m);
            const auto tf = RouterSolicitPacket::try_from(*icmpv6_packet(frame("icmpv6_ndp_router_solicit")));
            CHECK(tf.is_ok() && tf.value().options.size() == 2 && tf.value().total_len() == 12);
        }
        {  // basic_ra_parse
            const auto m = msg("icmpv6_ndp_router_advert");
            const auto ra = RouterAdvertPacket::from_bytes(m.data(), m.size());
            CHECK(ra.is_ok() && ra.value().header.icmpv6_type == 134 && ra.value().hop_limit == 0xff);
            CHECK(ra.is_ok() && ra.value().flags == 0x80 && ra.value().lifetime == 0x900);
            CHECK(ra.is_ok() && ra.value().reachable_time == 0x12345678 && ra.value().retrans_time == 0x87654321u);
            CHECK(ra.is_ok() && ra.value().options.size() == 2 && ra.value().options[0].option_type == 1);
            CHECK(ra.is_ok() && ra.value().options[1].option_type == 5 && ra.value().options[1].length == 1);
            CHECK(ra.is_ok() && ra.value().options[1].payload == (std::vector<uint8_t>{0, 0, 0x57, 0x68, 0x61, 0x74}));
            CHECK(ra.is_ok() && ra.value().to_bytes() == m);
        }
        {  // basic_ns_parse (TryFrom asks 24 B of payload: this 24-B message fails it)
            const auto m = msg("icmpv6_ndp_neighbor_solicit");
            const auto ns = NeighborSolicitPacket::from_bytes(m.data(), m.size());
            CHECK(ns.is_ok() && ns.value().header.icmpv6_type == 135 && ns.value().reserved == 0);
            CHECK(ns.is_ok() && ns.value().target_addr == ff02_1 && ns.value().options.empty());
            const auto tf = NeighborSolicitPacket::try_from(*icmpv6_packet(frame("icmpv6_ndp_neighbor_solicit")));
            CHECK(tf.is_err() && std::string(tf.error()) == "Payload too short for Neighbor Solicitation");
        }
        {  // basic_na_parse
            const auto m = msg("icmpv6_ndp_neighbor_advert");
            const auto na = NeighborAdvertPacket::from_bytes(m.data(), m.size());
            CHECK(na.is_ok() && na.value().header.icmpv6_type == 136 && na.value().flags == 0x80);
            CHECK(na.is_ok() && na.value().reserved == 0 && na.value().target_addr == ff02_1);
            const auto tf = NeighborAdvertPacket::try_from(*icmpv6_packet(frame("icmpv6_ndp_neighbor_advert")));
            CHECK(tf.is_ok() && tf.value().flags == 0x80 && tf.value().target_addr == ff02_1);
            CHECK(tf.is_ok() && tf.value().total_len() == 32);
        }
        {  // basic_redirect_parse (TryFrom asks 40 B of payload: this 40-B message fails it)
            const auto m = msg("icmpv6_ndp_redirect");
            const auto rd = RedirectPacket::from_bytes(m.data(), m.size());
            CHECK(rd.is_ok() && rd.value().header.icmpv6_type == 137 && rd.value().reserved == 0);
            CHECK(rd.is_ok() && rd.value().target_addr == ff02_1 && rd.value().dest_addr == Ipv6Addr{});
            CHECK(rd.is_ok() && rd.value().to_bytes() == m);
            const auto tf = RedirectPacket::try_from(*icmpv6_packet(frame("icmpv6_ndp_redirect")));
            CHECK(tf.is_err() && std::string(tf.error()) == "Payload too short for Redirect");
        }
        {  // basic_option_parsing (icmpv6.rs:1908-1920) and basic_na_create (2128-2155)
            const uint8_t ob[] = {0x02, 0x01, 0x06, 0x05, 0x04, 0x03, 0x02, 0x01, 0x00, 0x00, 0x00};
            const auto o = NdpOptionPacket::from_bytes(ob, sizeof(ob));
            CHECK(o.is_ok() && o.value().option_type == 2 && o.value().length == 1);
            CHECK(o.is_ok() && o.value().payload == (std::vector<uint8_t>{6, 5, 4, 3, 2, 1}));
            NeighborAdvertPacket na{Icmpv6Header{136, 0, 0}, 0x80, 0, ff02_1, {}, {}};
            const std::vector<uint8_t> want{0x88, 0, 0, 0, 0x80, 0, 0, 0, 0xff, 0x02, 0, 0, 0, 0, 0, 0,
                                            0, 0, 0, 0, 0, 0, 0, 0x01};
            CHECK(na.to_bytes() == want);
        }
    }
    {  // frame.rs:665-680 unknown EtherType keeps the payload
        const Frame& f = frame("unknown_ethertype_keeps_payload");
        CHECK(f.datalink && f.datalink->ethernet && f.datalink->ethernet->ethertype == 0x88b5);
        CHECK(!f.ip && !f.transport);
        CHECK(f.payload == (std::vector<uint8_t>{0xde, 0xad, 0xbe, 0xef}));
    }
    {  // frame.rs:681-712 IPv4/UDP frame
        const Frame& f = frame("ipv4_udp_frame");
        CHECK(f.ip && f.ip->ipv4 && f.ip->ipv4->version == 4);
        CHECK(f.transport && f.transport->udp && f.transport->udp->destination == 53);
        CHECK(f.payload == (std::vector<uint8_t>{1, 2, 3, 4}));
    }
    {  // frame.rs:713-734 from_ip_packet: dummy Ethernet header
        const Frame& f = frame("dummy_ethernet_ipv4");
        CHECK(f.datalink && f.datalink->ethernet && f.datalink->ethernet->ethertype == 0x0800);
        CHECK(f.datalink->ethernet->source == (MacAddr{}) && f.datalink->ethernet->destination == (MacAddr{}));
    }
    {  // ipv4.rs:944-1020 options: NOP, RecordRoute(len 4, data 12 34), EOL
        const Frame& f = frame("ipv4_with_options");
        const auto& h = *f.ip->ipv4;
        CHECK(h.header_length == 7 && h.total_length == 32);
        CHECK(h.options.size() == 3);
        CHECK(h.options[0].header.number == 1 && !h.options[0].header.length);
        CHECK(h.options[1].header.number == 7 && h.options[1].header.length == 4);
        CHECK(h.options[1].data == (std::vector<uint8_t>{0x12, 0x34}));
        CHECK(h.options[2].header.number == 0);
        CHECK(f.payload == (std::vector<uint8_t>{0xde, 0xad, 0xbe, 0xef}));
    }
    {  // ipv4.rs:944-970 round trip fields
        const Frame& f = frame("ipv4_round_trip");
        const auto& h = *f.ip->ipv4;
        CHECK(h.source.to_string() == "192.168.0.1" && h.destination.to_string() == "192.168.0.199");
        CHECK(h.checksum == 0xb1e6 && h.total_length == 28);
        CHECK(f.checksums.ip_checked && !f.checksums.ip_ok);  // the fixture's field does not verify
    }
    {  // ipv4.rs:1176-1204 strict truncation is an error, lenient is not; zero total length
        const auto& s = got.at("ipv4_strict_truncation");
        CHECK(s.is_err() && s.error().kind == ParseErrorKind::Truncated);
        CHECK(std::string(s.error().context) == "IPv4 packet" && s.error().expected == 40 && s.error().actual == 24);
        CHECK(frame("ipv4_lenient_truncation").ip->ipv4->total_length == 24);
        const Frame& z = frame("ipv4_zero_total_length");
        CHECK(z.ip->ipv4->total_length == 24);
        CHECK(z.payload == (std::vector<uint8_t>{0xde, 0xad, 0xbe, 0xef}));
    }
    {  // ipv6.rs:706-741 traffic class, flow label, payload
        const Frame& f = frame("ipv6_from_bytes");
        CHECK(f.ip->ipv6 && f.ip->ipv6->traffic_class == 0x0A && f.ip->ipv6->flow_label == 0x12345);
        CHECK(f.payload == bytes("Hello!!\n"));
    }
    {  // tcp.rs:1276-1314 options NOP, NOP, Timestamp; header 32; payload "test"
        const Frame& f = frame("tcp_basic_parse");
        const auto& t = *f.transport->tcp;
        CHECK(t.source == 49511 && t.destination == 9000);
        CHECK(t.sequence == 2419577528u && t.acknowledgement == 2487988854u);
        CHECK(t.data_offset == 8 && t.window == 4015 && t.checksum == 0xc031);
        CHECK(t.options.size() == 3 && t.options[0].kind == 1 && t.options[1].kind == 1);
        CHECK(t.options[2].kind == 8 && t.options[2].length == 10);
        CHECK(t.options[2].data == (std::vector<uint8_t>{0x2c, 0x57, 0xcd, 0xa5, 0x02, 0xa0, 0x41, 0x92}));
        CHECK(f.payload == bytes("test"));
    }
    {  // udp.rs:511-527
        const Frame& f = frame("udp_basic_parse");
        const auto& u = *f.transport->udp;
        CHECK(u.source == 0x1234 && u.destination == 0xabcd && u.length == 12 && u.checksum == 0x55aa);
        CHECK(f.payload == bytes("data"));
    }
    {  // icmp.rs:708-725 echo request, id 1234, seq 42
        const Frame& f = frame("icmp_echo_request");
        CHECK(f.ip->icmp && f.ip->icmp->icmp_type == 8 && f.ip->icmp->checksum == 0x3abc);
        CHECK(!f.transport);
        CHECK(f.payload.size() >= 4 && f.payload[0] == 0x04 && f.payload[1] == 0xd2 && f.payload[3] == 42);
    }
    {  // icmp.rs:728-815 echo reply / destination unreachable / time exceeded
        const Frame& r = frame("icmp_echo_reply_roundtrip");
        CHECK(r.ip->icmp && r.ip->icmp->icmp_type == 0 && r.payload.size() == 8);
        CHECK(detail::be16(r.payload.data()) == 5678 && detail::be16(r.payload.data() + 2) == 99);
        const Frame& u = frame("icmp_destination_unreachable");
        CHECK(u.ip->icmp->icmp_type == 3 && u.ip->icmp->icmp_code == 3);
        CHECK(detail::be16(u.payload.data() + 2) == 1500);  // next_hop_mtu
        const Frame& x = frame("icmp_time_exceeded");
        CHECK(x.ip->icmp->icmp_type == 11 && x.payload.size() == 11 && x.payload[0] == 0xde);
    }
    {  // icmpv6.rs:606-631 checksum KAT
        const Frame& f = frame("icmpv6_echo_request_lo");
        CHECK(f.ip->icmpv6 && f.ip->icmpv6->icmpv6_type == 128);
        CHECK(f.checksums.l4_checked && f.checksums.l4_computed == 0x1d2e);
    }
    {  // frame.rs:760-784 IPv6 + hop-by-hop: Frame dispatches on the raw next header (Q10)
        const Frame& f = frame("frame_slice_ipv6_hbh_udp");
        CHECK(f.ip->ipv6 && f.ip->ipv6->next_header == 0 && !f.transport);
        CHECK(f.payload == (std::vector<uint8_t>{0x04, 0xd2, 0x00, 0x35, 0x00, 0x0b, 0x00, 0x00, 'd', 'n', 's'}));
    }
    {  // frame.rs:747-784 FrameSlice boundaries (IPv4/TCP; IPv6 + hop-by-hop + UDP)
        std::vector<std::vector<uint8_t>> sf = {fx["frame_slice_ipv4_tcp"].bytes, fx["frame_slice_ipv6_hbh_udp"].bytes};
        std::vector<Result<FrameSlice>> sl;
        if (gpu) {
            sl = eng->frame_slices(sf);
        } else {
            for (auto& b : sf) {
                nexg_slice s;
                nexo_slice_frame(b.data(), b.size(), 0, 0, &s);
                sl.push_back(frame_slice_from(s, b.data(), b.size()));
            }
        }
        CHECK(sl[0].is_ok() && sl[1].is_ok());
        const FrameSlice& a = sl[0].value();
        CHECK(a.datalink && a.datalink->data == sf[0].data() && a.datalink->len == 14);
        CHECK(a.network && a.network->data == sf[0].data() + 14 && a.network->len == 20);
        CHECK(a.transport && a.transport->data == sf[0].data() + 34 && a.transport->len == 20);
        CHECK(a.payload.to_vec() == bytes("data"));
        const FrameSlice& b6 = sl[1].value();
        CHECK(b6.network && b6.network->len == 48 && b6.transport && b6.transport->len == 8);
        CHECK(b6.payload.to_vec() == bytes("dns"));
    }
    if (gpu) {  // examples/udp_ping.rs:68-109 (192.168.1.100 -> 1.1.1.1, 53443 -> 33435, DF, TTL 64)
        UdpPingTuple t;
        t.source = Ipv4Addr{{192, 168, 1, 100}};
        t.destination = Ipv4Addr{{1, 1, 1, 1}};
        t.src_port = 53443;
        t.dst_port = 33435;
        UdpPingShape shape;
        shape.src_mac = MacAddr{2, 0, 0, 0, 0, 1};
        shape.dst_mac = MacAddr{2, 0, 0, 0, 0, 2};
        auto built = eng->build_udp_ping({t, t}, shape);
        CHECK(built.is_ok() && built.value().size() == 2 && built.value()[0].size() == 42);
        std::vector<uint8_t> want(42);
        nexo_build_udp4(shape.src_mac.data(), shape.dst_mac.data(), 0xC0A80164u, 0x01010101u, 53443, 33435, 0, 64, 2, 0,
                        nullptr, 0, want.data());
        CHECK(built.value()[0] == want);
        auto parsed = eng->try_from_bufs(built.value());  // builder.rs -> Frame round trip
        CHECK(parsed[0].is_ok() && parsed[0].value().checksums.ip_ok && parsed[0].value().checksums.l4_ok);
        CHECK(parsed[0].value().ip->ipv4->total_length == 28 && parsed[0].value().transport->udp->length == 8);
        CHECK(parsed[0].value().ip->ipv4->flags == 2 && parsed[0].value().ip->ipv4->ttl == 64);
        UdpPingShape big = shape;  // builder/udp.rs:83 LengthOverflow
        big.payload.assign(65535 - 28 + 1, 0);
        auto over = eng->build_udp_ping({t}, big);
        CHECK(over.is_err() && over.error() == BuildError::LengthOverflow);
        // udp_ping's probe batch (one source and port pair, a destination per
        // target): the tuple builder's bytes for the same tuples, 300 targets
        std::vector<Ipv4Addr> targets;
        std::vector<UdpPingTuple> tuples;
        for (uint32_t k = 0; k < 300; k++) {
            targets.push_back(Ipv4Addr{{10, (uint8_t)(k >> 8), (uint8_t)k, 7}});
            UdpPingTuple u = t;
            u.destination = targets.back();
            tuples.push_back(u);
        }
        auto probes = eng->build_udp_probes(t.source, targets, 53443, 33435, shape);
        auto same = eng->build_udp_ping(tuples, shape);
        CHECK(probes.is_ok() && same.is_ok() && probes.value() == same.value());
        // descriptors through the grouped output == the records' descriptors,
        // single-shape groups (the probes) and mixed groups (the golden frames)
        std::vector<std::vector<uint8_t>> mix = probes.value();
        for (int k = 0; k < 3; k++)
            for (const auto& kv : fx)
                if (kv.second.flags == 0) mix.push_back(kv.second.bytes);  // the golden frames parsed by default
        const auto desc = eng->descriptors(mix);
        std::vector<nexg_record> rec(mix.size());
        for (size_t i = 0; i < mix.size(); i++) nexo_parse_frame(mix[i].data(), (uint32_t)mix[i].size(), 0, 0, &rec[i]);
        bool eq = desc.size() == mix.size();
        for (size_t i = 0; eq && i < mix.size(); i++)
            eq = desc[i].flags == rec[i].flags && desc[i].payload_off == rec[i].payload_off &&
                 desc[i].payload_len == rec[i].payload_len;
        CHECK(eq);
    }
    if (gpu) {  // examples/arp.rs / examples/ndp.rs probes, bytes == the oracle's restatement
        ArpProbeShape as;
        as.sender_mac = MacAddr{0x02, 0x42, 0xac, 0x11, 0x00, 0x02};
        as.sender_ip = Ipv4Addr{{192, 168, 1, 10}};
        const auto arp = eng->build_arp_requests({Ipv4Addr{{192, 168, 1, 1}}, Ipv4Addr{{10, 0, 0, 7}}}, as);
        CHECK(arp.is_ok() && arp.value().size() == 2 && arp.value()[1].size() == 42);
        uint8_t want[128];
        const uint8_t bc[6] = {0xff, 0xff, 0xff, 0xff, 0xff, 0xff}, zero6[6] = {0, 0, 0, 0, 0, 0};
        const uint8_t tip[4] = {10, 0, 0, 7};
        CHECK(nexo_build_arp(bc, as.sender_mac.data(), as.sender_ip.octets.data(), zero6, tip, 1, 0x0800, 1, 6, 4,
                             want) == 42);
        CHECK(arp.is_ok() && memcmp(arp.value()[1].data(), want, 42) == 0);
        ArpProbeShape bad = as;
        bad.hw_addr_len = 5;  // builder/arp.rs:101-108
        const auto e = eng->build_arp_requests({Ipv4Addr{{1, 2, 3, 4}}}, bad);
        CHECK(e.is_err() && e.error() == BuildError::InvalidFieldLength);
        NdpProbeShape ns;
        ns.src_mac = MacAddr{0x02, 0, 0, 0, 0, 0x99};
        ns.src_ip.octets[0] = 0xfe; ns.src_ip.octets[1] = 0x80; ns.src_ip.octets[15] = 0x01;
        Ipv6Addr tgt;
        tgt.octets[0] = 0xfe; tgt.octets[1] = 0x80; tgt.octets[13] = 0xab; tgt.octets[14] = 0xcd; tgt.octets[15] = 0xef;
        const auto sol = eng->build_ndp_solicits({tgt}, ns);
        nexo_ip_spec sp{};
        sp.family = 6;
        memcpy(sp.src, ns.src_ip.octets.data(), 16);
        memcpy(sp.dst, tgt.octets.data(), 16);
        memcpy(sp.src_mac, ns.src_mac.data(), 6);
        const uint8_t mc[6] = {0x33, 0x33, 0x00, 0xab, 0xcd, 0xef};  // ndp.rs:25-35
        memcpy(sp.dst_mac, mc, 6);
        sp.ttl = 255;
        CHECK(nexo_build_ndp_ns(&sp, want) == 86);
        CHECK(sol.size() == 1 && sol[0].size() == 86 && memcmp(sol[0].data(), want, 86) == 0);
        const auto back = eng->try_from_buf(sol[0], ParseOption{}, ParseMode::Lenient);  // it parses and verifies
        CHECK(back.is_ok() && back.value().ip && back.value().ip->icmpv6 && back.value().ip->icmpv6->icmpv6_type == 135);
        CHECK(back.is_ok() && back.value().checksums.l4_ok);
    }
    if (gpu) {  // tcp_ping / icmp_ping builds (builder/tcp.rs:175-228, examples/tcp_ping.rs:111-123,
                // examples/icmp_ping.rs:67-80) against the oracle's builders, IPv4 and IPv6
        for (int fam : {4, 6}) {
            TcpPingTuple t;
            if (fam == 4) {
                t.source = IpAddr::from(Ipv4Addr{{192, 168, 1, 100}});
                t.destination = IpAddr::from(Ipv4Addr{{192, 168, 1, 1}});
            } else {
                Ipv6Addr a, b;
                a.octets[15] = 1;
                b.octets[15] = 2;
                t.source = IpAddr::from(a);
                t.destination = IpAddr::from(b);
            }
            t.src_port = 1234;
            t.dst_port = 80;
            t.sequence = 1;
            t.acknowledgement = 2;
            TcpPingShape sh;
            sh.window = 1024;
            sh.options = {0x02, 0x04, 0x05, 0xb4, 0x04, 0x02, 0x01, 0x01, 0x03, 0x03, 0x07};  // mss, sack_perm, nop, nop, wscale
            sh.payload = {'a', 'b', 'c'};
            auto b = eng->build_tcp_ping({t, t}, sh);
            CHECK(b.is_ok() && b.value().size() == 2);
            nexo_ip_spec spec{};
            spec.family = fam;
            memcpy(spec.src, t.source.octets.data(), 16);
            memcpy(spec.dst, t.destination.octets.data(), 16);
            spec.ttl = 64;
            spec.ip_flags = 2;
            std::vector<uint8_t> want(14 + (fam == 4 ? 20 : 40) + 20 + 12 + 3);
            nexo_build_tcp(&spec, 1234, 80, 1, 2, 0x02, 1024, 0, sh.options.data(), (uint32_t)sh.options.size(),
                           sh.payload.data(), 3, want.data());
            CHECK(b.value()[0] == want);
            auto f = eng->try_from_bufs(b.value());
            // 11 option bytes + 1 zero pad: the walk reads the pad as EOL (tcp.rs:767-818)
            CHECK(f[0].is_ok() && f[0].value().checksums.l4_ok && f[0].value().transport->tcp->options.size() == 6);
            CHECK(f[0].value().transport->tcp->options[5].kind == 0 && f[0].value().transport->tcp->data_offset == 8);
            IcmpPingTuple it;
            it.source = t.source;
            it.destination = t.destination;
            it.identifier = 0x1234;
            it.sequence = 1;
            IcmpPingShape ish;
            ish.payload = {'h', 'e', 'l', 'l', 'o'};
            auto e = eng->build_icmp_ping({it}, ish);
            std::vector<uint8_t> wante(14 + (fam == 4 ? 20 : 40) + 8 + 5);
            nexo_build_icmp_echo(&spec, fam == 4 ? 8 : 128, 0, 0x1234, 1, ish.payload.data(), 5, wante.data());
            CHECK(e.is_ok() && e.value()[0] == wante);
            auto fe = eng->try_from_bufs(e.value());
            CHECK(fe[0].is_ok() && fe[0].value().checksums.l4_ok);
            // examples/mutable_chaining.rs: clear the checksum fields, recompute
            // them over the raw buffers (Mutable*Packet::recompute_checksum)
            // -> the builders' bytes again
            std::vector<std::vector<uint8_t>> fix = {b.value()[0], e.value()[0]};
            const size_t ip = 14, l4 = 14 + (fam == 4 ? 20 : 40);
            for (auto& x : fix) {
                if (fam == 4) x[ip + 10] = x[ip + 11] = 0;
            }
            fix[0][l4 + 16] = fix[0][l4 + 17] = 0xEE;  // TCP checksum
            fix[1][l4 + 2] = fix[1][l4 + 3] = 0x11;    // ICMP / ICMPv6 checksum
            auto fx = eng->recompute_checksums(fix);
            CHECK(fix[0] == b.value()[0] && fix[1] == e.value()[0]);
            CHECK((fx[0].done & NEXG_FIX_L4) && fx[0].proto == 6 && fx[0].l4_off == l4);
            CHECK((fx[1].done & NEXG_FIX_L4) && fx[1].proto == (fam == 4 ? 1 : 58));
            CHECK(((fx[0].done & NEXG_FIX_IP) != 0) == (fam == 4));
        }
        TcpPingTuple a, b6;
        a.source = a.destination = IpAddr::from(Ipv4Addr{{10, 0, 0, 1}});
        b6.source = b6.destination = IpAddr::from(Ipv6Addr{});
        auto mix = eng->build_tcp_ping({a, b6}, TcpPingShape{});
        CHECK(mix.is_err() && mix.error() == BuildError::AddressFamilyMismatch);
        TcpPingShape big;
        big.options.assign(50, 0x01);  // builder/tcp.rs:211-228: options past 40 B
        auto over = eng->build_tcp_ping({a}, big);
        CHECK(over.is_err() && over.error() == BuildError::LengthOverflow);
    }
    if (!gpu) {  // datalink::RawSender / RawReceiver over loopback where CAP_NET_RAW is held
        try {
            datalink::Config c;
            c.read_timeout_ms = 300;
            c.skip_outgoing = true;
            datalink::RawReceiver rx("lo", c);
            datalink::RawSender tx("lo");
            std::vector<std::vector<uint8_t>> out;
            for (int i = 0; i < 32; i++) {
                std::vector<uint8_t> f(64 + 8 * i, 0);
                for (int k = 0; k < 6; k++) f[k] = 0xFF;
                const uint8_t src[6] = {0x02, 0x6E, 0x65, 0x78, 0x43, (uint8_t)i};
                memcpy(f.data() + 6, src, 6);
                f[12] = 0x88;
                f[13] = 0xB5;  // local experimental EtherType
                f[20] = (uint8_t)i;
                out.push_back(f);
            }
            CHECK(tx.send_batch(out) == out.size());
            std::vector<std::vector<uint8_t>> in;
            for (int tries = 0; tries < 10 && in.size() < out.size(); tries++)
                for (auto& f : rx.next_batch())
                    if (f.size() >= 12 && f[6] == 0x02 && f[7] == 0x6E && f[10] == 0x43) in.push_back(f);
            CHECK(in == out);
        } catch (const Error& e) {
            printf("datalink checks skipped: %s\n", e.what());
        }
    }
    // PcapReader: the fixtures as a classic pcap file, read back packed and
    // walked in place through the mapping (the zero-copy shape): same frames
    {
        char path[] = "/tmp/nexg_cpp_pcap_XXXXXX";
        const int fd = mkstemp(path);
        FILE* f = fdopen(fd, "wb");
        const uint32_t gh[6] = {0xA1B2C3D4u, 0x00040002u, 0, 0, 65535, 1};
        fwrite(gh, 4, 6, f);
        for (size_t i = 0; i < frames.size(); i++) {
            const uint32_t rh[4] = {(uint32_t)i, 0, (uint32_t)frames[i].size(), (uint32_t)frames[i].size()};
            fwrite(rh, 4, 4, f);
            fwrite(frames[i].data(), 1, frames[i].size(), f);
        }
        fclose(f);
        std::vector<std::vector<uint8_t>> packed, mapped;
        {
            PcapReader r(path);
            for (auto b = r.next_batch(7); !b.empty(); b = r.next_batch(7)) packed.insert(packed.end(), b.begin(), b.end());
        }
        {
            PcapReader r(path);
            uint64_t size = 0, pos = 0;
            const uint8_t* m = r.map(&size, &pos);
            while (pos < size) {
                const auto w = r.walk_mapped(pos, 4096, 5);
                for (size_t k = 0; k < w.offsets.size(); k++)
                    mapped.emplace_back(m + w.from + w.offsets[k], m + w.from + w.offsets[k] + w.lengths[k]);
            }
        }
        unlink(path);
        CHECK(packed == frames);
        CHECK(mapped == frames);
    }
    // every fixture: Frame fields == the record the oracle writes (device == oracle in --gpu)
    for (const auto& n : names) {
        const Fixture& fxt = fx[n];
        nexg_record r;
        nexo_parse_frame(fxt.bytes.data(), fxt.bytes.size(), fxt.flags, fxt.ip_offset, &r);
        const auto& g = got.at(n);
        CHECK(g.is_err() == (NEXG_STATUS(r.flags) != 0));
        if (g.is_ok()) {
            CHECK(g.value().packet_len == r.packet_len);
            CHECK(g.value().payload.size() == r.payload_len);
            CHECK(g.value().checksums.l4_computed == r.l4_csum_calc && g.value().checksums.ip_computed == r.ip_csum_calc);
        }
    }
    printf("%s: %d checks, %d failures, %zu fixtures\n", gpu ? "gpu" : "cpu", checks, failures, names.size());
    return failures ? 1 : 0;
}
