// nexg_fixup.hip — nexg_recompute_checksums_batch: in-place checksum fix-up
// with the raw-buffer semantics of nex-packet's mutable views, chained as
// examples/mutable_chaining.rs:19-63 chains them (include/nexg.h):
//   MutableIpv4Packet::recompute_checksum  ipv4.rs:669-679  (header, skipword 5)
//   MutableUdpPacket::recompute_checksum   udp.rs:338-369   (pseudo, skipword 3)
//   MutableTcpPacket::recompute_checksum   tcp.rs:1009-1040 (pseudo, skipword 8)
//   MutableIcmpPacket::recompute_checksum  icmp.rs:372-377  (skipword 1)
//   MutableIcmpv6Packet::recompute_checksum icmpv6.rs:450-470 (pseudo, skipword 1)
// The checksums are util.rs:65-137 over each view's whole buffer (for the L4
// views: the enclosing IP view's payload_mut slice), in the same congruent
// closed form as the parse path (frame_core.hpp header): no re-serialisation.
//
// Not a streaming hot path (one lane per frame, 16-B loads through the frame,
// two 2-B byte-pair stores); the egress half of the checksum story.
#include "parse_kernels.hpp"

namespace nexg {

__device__ __forceinline__ void put_be16(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}

__global__ __launch_bounds__(256) void k_recompute(ParseArgs a, uint32_t which, nexg_fixup* out) {
    const uint64_t idx = (uint64_t)blockIdx.x * kTile + threadIdx.x;
    if (idx >= a.count) return;
    nexg_fixup fx{0, 0, 0, 0, 0};
    uint64_t off;
    uint32_t len;
    if (!frame_extent(a, idx, off, len)) {
        if (out) out[idx] = fx;
        return;
    }
    uint8_t* f = const_cast<uint8_t*>(a.data) + off;
    const GlobalFrame gf{f};
    const FrameOps<GlobalFrame> o{gf, (uint32_t)(reinterpret_cast<uint64_t>(f) & 1u)};
    // Ethernet view (ethernet.rs:355-361) or the raw IP packet at ip_offset
    uint32_t L = 14, family = 0;
    if (a.opt_flags & NEXG_PARSE_FROM_IP) {
        L = a.ip_offset;
        const uint32_t v = L < len ? (uint32_t)f[L] >> 4 : 0u;
        family = v == 4u ? 4u : (v == 6u ? 6u : 0u);
    } else if (len >= 14u) {
        const uint32_t et = o.be16(12);
        family = et == 0x0800u ? 4u : (et == 0x86DDu ? 6u : 0u);
    }
    const uint32_t n = family && L < len ? len - L : 0u;
    uint32_t P = 0, m = 0, proto = 0;
    uint64_t pseudo = 0;
    bool l4 = false;
    if (family == 4u && n >= 20u) {
        // MutableIpv4Packet::new (ipv4.rs:540-566)
        const uint32_t hl = ((uint32_t)f[L] & 15u) * 4u, total = o.be16(L + 2);
        if (hl >= 20u && hl <= n && (total == 0u || total >= hl)) {
            if (which & NEXG_FIX_IP) {  // util::checksum(raw[..header_len], 5)
                const uint32_t c = fold_complement(o.wsum(L, L + 10) + o.wsum(L + 12, L + hl));
                put_be16(f + L + 10, c);
                fx.done |= NEXG_FIX_IP;
                fx.ip_csum = (uint16_t)c;
            }
            const uint32_t eff = total == 0u ? n : (total < n ? total : n);  // total_len, ipv4.rs:697-704
            P = L + hl;
            m = eff - hl;
            proto = f[L + 9];
            pseudo = (uint64_t)o.be16(L + 12) + o.be16(L + 14) + o.be16(L + 16) + o.be16(L + 18);
            l4 = proto == 17u || proto == 6u || proto == 1u;
        }
    } else if (family == 6u && n >= 40u) {  // MutableIpv6Packet::new: >= 40 B, payload = rest
        P = L + 40;
        m = n - 40u;
        proto = f[L + 6];
#pragma unroll
        for (uint32_t k = 0; k < 32; k += 2) pseudo += o.be16(L + 8 + k);
        l4 = proto == 17u || proto == 6u || proto == 58u;
    }
    if (l4 && (which & NEXG_FIX_L4)) {
        uint32_t sk = 0;  // byte offset of the checksum word (skipword * 2)
        bool view = false;
        if (proto == 17u) {  // MutableUdpPacket::new (udp.rs:101-121)
            const uint32_t ul = m >= 8u ? o.be16(P + 4) : 0u;
            view = m >= 8u && (ul == 0u || (ul >= 8u && ul <= m));
            sk = 6;
        } else if (proto == 6u) {  // MutableTcpPacket::new (tcp.rs:857-876)
            const uint32_t hl = m >= 20u ? ((uint32_t)f[P + 12] >> 4) * 4u : 0u;
            view = m >= 20u && hl >= 20u && hl <= m;
            sk = 16;
        } else {  // ICMP / ICMPv6: IcmpPacket::from_buf needs the 8-B header (icmp.rs:188-191)
            view = m >= 8u;
            sk = 2;
        }
        if (view) {
            uint64_t t = o.wsum(P, P + sk) + o.wsum(P + sk + 2u, P + m);
            if (proto != 1u) t += pseudo + proto + m;  // util.rs:89-97 / 119-127 (len as one u32)
            const uint32_t c = fold_complement(t);
            put_be16(f + P + sk, c);
            fx.done |= NEXG_FIX_L4;
            fx.proto = (uint8_t)proto;
            fx.l4_csum = (uint16_t)c;
            fx.l4_off = (uint16_t)P;
        }
    }
    if (out) out[idx] = fx;
}

hipError_t launch_recompute(const ParseArgs& a, uint32_t which, nexg_fixup* out, hipStream_t s) {
    if (a.count == 0) return hipSuccess;
    const uint64_t blocks = (a.count + kTile - 1) / kTile;
    hipLaunchKernelGGL(k_recompute, dim3((uint32_t)blocks), dim3(kTile), 0, s, a, which, out);
    return hipGetLastError();
}

}  // namespace nexg
