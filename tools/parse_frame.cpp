// parse_frame — the C++ counterpart of the reference's examples/parse_frame.rs
// over a capture file: records are read a batch at a time (nexg_pcap_*,
// nex-datalink's pcap::from_file channel, pcap.rs:95-109), parsed on the GPU
// through the C++ host API (nexg::Engine::try_from_bufs = Frame::try_from_buf
// per frame, parse_frame.rs:43-73) and printed in display_frame's layout
// (parse_frame.rs:76-131), line for line as `python -m nex_amd.parse_frame`.
//   build: make -C tools parse_frame      run: tools/parse_frame capture.pcap [batch]
#include <stdio.h>
#include <stdlib.h>

#include <map>
#include <string>
#include <vector>

#include "../include/nexg.hpp"

namespace {

std::string mac(const nexg::MacAddr& m) {
    char b[18];
    snprintf(b, sizeof(b), "%02x:%02x:%02x:%02x:%02x:%02x", m[0], m[1], m[2], m[3], m[4], m[5]);
    return b;
}

// std::net::Ipv6Addr's Display: IPv4-mapped addresses as ::ffff:a.b.c.d,
// otherwise RFC 5952 (longest run of >= 2 zero groups as ::, the first on ties)
std::string ipv6(const nexg::Ipv6Addr& a) {
    uint16_t g[8];
    for (int i = 0; i < 8; i++) g[i] = (uint16_t)(a.octets[2 * i] << 8 | a.octets[2 * i + 1]);
    if (!g[0] && !g[1] && !g[2] && !g[3] && !g[4] && g[5] == 0xffff) {
        char b[32];
        snprintf(b, sizeof(b), "::ffff:%u.%u.%u.%u", a.octets[12], a.octets[13], a.octets[14], a.octets[15]);
        return b;
    }
    int best = -1, blen = 0;
    for (int i = 0; i < 8;) {
        if (g[i] != 0) { i++; continue; }
        int j = i;
        while (j < 8 && g[j] == 0) j++;
        if (j - i > blen && j - i >= 2) { best = i; blen = j - i; }
        i = j;
    }
    std::string s;
    char b[8];
    for (int i = 0; i < 8; i++) {
        if (i == best) { s += "::"; i += blen - 1; continue; }
        if (!s.empty() && s.back() != ':') s += ":";
        snprintf(b, sizeof(b), "%x", g[i]);
        s += b;
    }
    return s;
}

const std::map<uint16_t, const char*> kEtherTypes = {
    {0x0800, "Ipv4"}, {0x0806, "Arp"}, {0x0842, "WakeOnLan"}, {0x22F3, "Trill"}, {0x6003, "DECnet"},
    {0x8035, "Rarp"}, {0x809B, "AppleTalk"}, {0x80F3, "Aarp"}, {0x8137, "Ipx"}, {0x8204, "Qnx"},
    {0x86DD, "Ipv6"}, {0x8808, "FlowControl"}, {0x8819, "CobraNet"}, {0x8847, "Mpls"}, {0x8848, "MplsMcast"},
    {0x8863, "PppoeDiscovery"}, {0x8864, "PppoeSession"}, {0x8100, "Vlan"}, {0x88A8, "PBridge"},
    {0x88CC, "Lldp"}, {0x88F7, "Ptp"}, {0x8902, "Cfm"}, {0x9100, "QinQ"}, {0x8899, "Rldp"}};
const std::map<uint8_t, const char*> kProtocols = {
    {0, "Hopopt"}, {1, "Icmp"}, {2, "Igmp"}, {4, "Ipv4"}, {6, "Tcp"}, {17, "Udp"}, {41, "Ipv6"},
    {43, "Ipv6Route"}, {44, "Ipv6Frag"}, {47, "Gre"}, {50, "Esp"}, {51, "Ah"}, {58, "Icmpv6"},
    {59, "Ipv6NoNxt"}, {60, "Ipv6Opts"}, {132, "Sctp"}, {255, "Reserved"}};

std::string ethertype(uint16_t v) {
    auto it = kEtherTypes.find(v);
    if (it != kEtherTypes.end()) return it->second;
    return "Unknown(" + std::to_string(v) + ")";  // EtherType's derived Debug
}
std::string protocol(uint8_t v) {
    auto it = kProtocols.find(v);
    if (it != kProtocols.end()) return it->second;
    return "IpNextProtocol(" + std::to_string(v) + ")";
}

void display_frame(const nexg::Frame& f) {  // parse_frame.rs:76-131
    printf("Packet Frame (%zu bytes)\n", f.packet_len);
    if (f.datalink) {
        if (f.datalink->ethernet) {
            const auto& e = *f.datalink->ethernet;
            printf("  Ethernet: %s > %s (%s)\n", mac(e.source).c_str(), mac(e.destination).c_str(),
                   ethertype(e.ethertype).c_str());
        }
        if (f.datalink->arp) {
            const auto& a = *f.datalink->arp;
            const char* op = a.operation == 1 ? "Request" : a.operation == 2 ? "Reply" : nullptr;
            std::string ops = op ? op : "Unknown(" + std::to_string(a.operation) + ")";
            printf("  ARP: %s(%s) > %s(%s); operation: %s\n", mac(a.sender_hw_addr).c_str(),
                   a.sender_proto_addr.to_string().c_str(), mac(a.target_hw_addr).c_str(),
                   a.target_proto_addr.to_string().c_str(), ops.c_str());
        }
    }
    if (f.ip) {
        if (f.ip->ipv4)
            printf("  IPv4: %s -> %s (protocol: %s)\n", f.ip->ipv4->source.to_string().c_str(),
                   f.ip->ipv4->destination.to_string().c_str(), protocol(f.ip->ipv4->next_level_protocol).c_str());
        if (f.ip->ipv6)
            printf("  IPv6: %s -> %s (next header: %s)\n", ipv6(f.ip->ipv6->source).c_str(),
                   ipv6(f.ip->ipv6->destination).c_str(), protocol(f.ip->ipv6->next_header).c_str());
        if (f.ip->icmp) printf("  ICMP: present\n");
        if (f.ip->icmpv6) printf("  ICMPv6: present\n");
    }
    if (f.transport) {
        if (f.transport->tcp) printf("  TCP: %u -> %u\n", f.transport->tcp->source, f.transport->tcp->destination);
        if (f.transport->udp) printf("  UDP: %u -> %u\n", f.transport->udp->source, f.transport->udp->destination);
    }
    if (!f.payload.empty()) printf("  Payload: %zu bytes\n", f.payload.size());
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s capture.pcap [batch_frames]\n", argv[0]);
        return 2;
    }
    const uint64_t batch = argc > 2 ? strtoull(argv[2], nullptr, 0) : 65536;
    try {
        nexg::PcapReader cap(argv[1]);
        const nexg::ParseOption opt = cap.parse_option();
        nexg::Engine eng(0);
        uint64_t no = 1;
        for (;;) {
            const auto frames = cap.next_batch(batch, batch * 2048);
            if (frames.empty()) break;
            const auto res = eng.try_from_bufs(frames, opt);
            for (size_t i = 0; i < frames.size(); i++, no++) {
                printf("---- Interface: %s, No.: %llu, Total Length: %zu bytes ----\n", argv[1],
                       (unsigned long long)no, frames[i].size());
                if (res[i].is_err()) printf("Failed to parse packet as Frame\n");
                else display_frame(res[i].value());
            }
        }
    } catch (const nexg::Error& e) {
        fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
