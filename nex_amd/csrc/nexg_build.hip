// nexg_build.hip — serialize path and synthetic workload synthesis.
//
// k_build_udp4: the examples/udp_ping.rs:68-109 composition
//   UdpPacketBuilder::build (builder/udp.rs:67-95: length = 8 + payload,
//   checksum via udp::checksum over to_bytes with skipword 3, computed 0 kept)
//   -> Ipv4PacketBuilder::to_bytes (builder/ipv4.rs:94-170: IHL 5, total
//   length, ipv4::checksum) -> EthernetPacketBuilder::to_bytes
//   (builder/ethernet.rs:68, ethernet.rs:211-216)
// on one lane per tuple. Frames are assembled in LDS and leave the CU as
// coalesced 16-B stores of the tile's contiguous output range.
//
// k_gen_*: SURVEY.md Appendix C workloads. splitmix64 is counter based
// (draw m of frame i is mix(seed ^ i*phi + (m+1)*phi)), so a wave fills one
// frame cooperatively: lane l produces 8-byte words l, l+64, ...
#include <stdlib.h>

#include "frame_core.hpp"
#include "nexg_internal.hpp"

namespace nexg {

constexpr uint64_t kPhi = 0x9E3779B97F4A7C15ull;

NEXG_HD uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
NEXG_HD uint64_t draw(uint64_t s0, uint64_t m) { return mix64(s0 + (m + 1) * kPhi); }

// IMIX class/protocol draw (App. C): the length class keeps 7:4:1 exactly; a
// protocol that does not fit the class (v6+TCP in 64 B) is redrawn from the
// following draws. Returns draws consumed.
NEXG_HD uint32_t imix_class(uint64_t s0, uint32_t& len, uint32_t& proto) {
    uint32_t m = 0;
    const uint64_t c0 = draw(s0, m++);
    const uint32_t cls = (uint32_t)(c0 % 12u);
    len = cls < 7u ? 64u : (cls < 11u ? 576u : 1500u);
    proto = (uint32_t)((c0 >> 32) % 6u);
    while (proto == 3u && len == 64u) proto = (uint32_t)(draw(s0, m++) % 6u);
    return m;
}

// ---------------------------------------------------------------- builder

constexpr uint32_t kBuildTile = 256;
constexpr uint32_t kBuildMaxStride = 128;

struct BuildArgs {
    nexg_udp4_build p;
    uint8_t* out;
    uint32_t out_stride;
    const nexg_udp4_tuple* tuples;  // AOS builds: one 16-B tuple per frame
    uint32_t tile_order;            // tile_index order (nexg_internal.hpp)
};

// Dynamic LDS beside k_build_udp4<64>'s 16-KiB static tile so that 5
// workgroups fit a CU's 160 KiB instead of 8 (at most 32 KiB each): fewer
// concurrent write streams per CU. 16M udp_ping frames in contiguous eighths
// (profiles/r04/occupancy/builder_occupancy_ab.log): probe batch 0.887-0.891
// of 8 TB/s written against 0.743 at 8 per CU, full tuples 0.717-0.719 against
// 0.681; 4 per CU the same, 6 and 7 in between. NEXG_BUILD_LDS_PAD overrides
// (measurement).
constexpr uint32_t kBuildCapPad = 160u * 1024u / 5u - (kBuildTile * 64u + 16u) - 256u;
uint32_t build_lds_pad() {
    static const uint32_t pad = [] {
        const char* e = getenv("NEXG_BUILD_LDS_PAD");
        if (!e) return kBuildCapPad;
        const long v = atol(e);  // clamped: a negative or oversized pad fails every build launch
        return v <= 0 ? 0u : v >= (long)kBuildCapPad ? kBuildCapPad : (uint32_t)v;
    }();
    return pad;
}

// Frame header given as NH (odd) little-endian halfwords of its bytes, written
// to LDS at an even offset d0: (NH-1)/2 dword writes + 1 halfword write, the
// dword run shifted by one halfword when d0 = 2 mod 4.
template <int NH>
__device__ __forceinline__ void lds_put_halfwords(uint8_t* smem, uint32_t d0, const uint32_t (&hw)[NH]) {
    static_assert(NH % 2 == 1, "odd halfword count");
    const bool al = (d0 & 2u) == 0;
    const uint32_t b32 = al ? d0 : d0 + 2u;
#pragma unroll
    for (int m = 0; m < NH / 2; m++) {
        const uint32_t v = al ? (hw[2 * m] | (hw[2 * m + 1] << 16)) : (hw[2 * m + 1] | (hw[2 * m + 2] << 16));
        *reinterpret_cast<uint32_t*>(smem + b32 + 4u * m) = v;
    }
    *reinterpret_cast<uint16_t*>(smem + (al ? d0 + 2u * (NH - 1) : d0)) = (uint16_t)(al ? hw[NH - 1] : hw[0]);
}

// N (even) halfwords at an even offset e: dword writes, the run shifted by a
// halfword (one 2-B write at each end) when e = 2 mod 4
template <int N>
__device__ __forceinline__ void lds_put_even_run(uint8_t* smem, uint32_t e, const uint32_t (&hw)[N]) {
    static_assert(N % 2 == 0, "even halfword count");
    if ((e & 2u) == 0) {
#pragma unroll
        for (int m = 0; m < N / 2; m++)
            *reinterpret_cast<uint32_t*>(smem + e + 4u * m) = hw[2 * m] | (hw[2 * m + 1] << 16);
    } else {
        *reinterpret_cast<uint16_t*>(smem + e) = (uint16_t)hw[0];
#pragma unroll
        for (int m = 0; m < N / 2 - 1; m++)
            *reinterpret_cast<uint32_t*>(smem + e + 2u + 4u * m) = hw[2 * m + 1] | (hw[2 * m + 2] << 16);
        *reinterpret_cast<uint16_t*>(smem + e + 2u * (N - 1)) = (uint16_t)hw[N - 1];
    }
}

// NH (odd) halfwords of frame bytes at any LDS offset d0. Even d0:
// lds_put_halfwords. Odd d0 (odd frame strides): the first byte alone, the
// next 2 NH - 2 bytes re-paired into halfwords at the even offset d0 + 1
// (dword writes), the last byte alone — instead of 2 NH byte writes.
template <int NH>
__device__ __forceinline__ void lds_put_frame_hw(uint8_t* smem, uint32_t d0, const uint32_t (&hw)[NH]) {
    if ((d0 & 1u) == 0) {
        lds_put_halfwords<NH>(smem, d0, hw);
        return;
    }
    uint32_t sh[NH - 1];
#pragma unroll
    for (int k = 0; k < NH - 1; k++) sh[k] = (hw[k] >> 8) | ((hw[k + 1] & 0xFFu) << 8);
    smem[d0] = (uint8_t)hw[0];
    lds_put_even_run<NH - 1>(smem, d0 + 1u, sh);
    smem[d0 + 2u * NH - 1u] = (uint8_t)(hw[NH - 1] >> 8);
}

__device__ __forceinline__ uint32_t bswap16(uint32_t v) { return ((v & 0xFFu) << 8) | ((v >> 8) & 0xFFu); }

// Per-frame parameter or the batch default. The array is read as a global
// (address-space 1) pointer: written as `per ? per[i] : def` with def in the
// kernel arguments, the compiler selected between the two addresses and issued
// flat loads (counted on both vmcnt and lgkmcnt) for every parameter.
template <class T>
__device__ __forceinline__ uint32_t per_or_def(const T* per, uint64_t i, uint32_t def) {
    return per ? (uint32_t)NEXG_GLOBAL(T, per)[i] : def;
}

// tile copy-out shared by the builders: nf frames of `stride` bytes staged
// contiguously in LDS leave as 16-B non-temporal stores (+ byte tail of a
// partial tile). Non-temporal: the udp_ping build of 16M frames takes 0.132
// instead of 0.165 ms with identical HBM traffic (PMC).
__device__ __forceinline__ void build_copy_out(const uint8_t* smem, uint8_t* T, uint32_t bytes) {
    const uint32_t tid = threadIdx.x;
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    for (uint32_t c = tid; c < bytes / 16u; c += kBuildTile)
        __builtin_nontemporal_store(reinterpret_cast<const v4u*>(smem)[c], reinterpret_cast<v4u*>(T) + c);
    const uint32_t tail = bytes & ~15u;
    if (tid < bytes - tail) T[tail + tid] = smem[tail + tid];
}

// BE word sum of the shared payload (it starts at an even L4 offset), once
// per workgroup: all threads call it together; 0 without a barrier when the
// payload is empty (udp_ping's case), so the empty build pays nothing
__device__ __forceinline__ uint32_t shared_payload_sum(const uint8_t* pl, uint32_t n, uint32_t* s) {
    if (n == 0) return 0u;  // kernel argument: uniform over the workgroup
    if (threadIdx.x == 0) *s = 0;
    __syncthreads();
    uint32_t ps = 0;
    for (uint32_t k = 2u * threadIdx.x; k < n; k += 2u * kBuildTile)
        ps += ((uint32_t)pl[k] << 8) | (k + 1 < n ? (uint32_t)pl[k + 1] : 0u);
    if (ps) atomicAdd(s, ps);
    __syncthreads();
    return *s;
}

// MAXS = largest stride the LDS tile holds (0: direct global writes).
// FULL: per-tuple address, port and id arrays present, MACs from the defaults —
// every parameter load is unconditional, so a lane issues all five before its
// first wait (the general form waits once per optional array).
// PROBE: the udp_ping probe batch (udp_ping.rs:30-31, 68-109 per target): only
// dst_ip is per frame; source address, ports, id and MACs are the batch's.
// AOS: the per-frame tuple as one 16-B record (nexg_udp4_tuple), read with one
// plain dwordx4 load per lane instead of five SoA loads (NEXG_AOS_NT=1 builds
// the non-temporal load for A/B: 0.150 vs 0.136 ms, profiles/r04/ab/).
template <uint32_t MAXS, bool FULL = false, bool PROBE = false, bool AOS = false>
__global__ __launch_bounds__(256) void k_build_udp4(BuildArgs a) {
    constexpr bool STAGED = MAXS != 0;
    __shared__ __attribute__((aligned(16))) uint8_t smem[STAGED ? kBuildTile * MAXS : 16];
    const nexg_udp4_build& p = a.p;
    const uint64_t first = tile_index(a.tile_order) * kBuildTile;
    const uint64_t left = p.count - first;
    const uint32_t nf = left < kBuildTile ? (uint32_t)left : kBuildTile;
    const uint32_t tid = threadIdx.x;
    const uint64_t i = first + tid;
    const uint32_t flen = 42u + p.payload_len;
    __shared__ uint32_t s_pay;
    const uint64_t pw = shared_payload_sum(p.payload, p.payload_len, &s_pay);
    if (tid < nf) {
#ifndef NEXG_AOS_NT
#define NEXG_AOS_NT 0
#endif
#if NEXG_AOS_NT
        const u32x4 tv = AOS ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.tuples) + i) : u32x4{0, 0, 0, 0};
#else
        const u32x4 tv = AOS ? reinterpret_cast<const u32x4*>(a.tuples)[i] : u32x4{0, 0, 0, 0};
#endif
        const uint32_t dst = AOS ? tv.y : p.dst_ip[i];
        const uint32_t src = AOS ? tv.x : FULL ? p.src_ip[i] : PROBE ? p.def_src_ip : (p.src_ip ? p.src_ip[i] : p.def_src_ip);
        const uint32_t sp = AOS ? tv.z & 0xFFFFu : FULL ? p.src_port[i] : PROBE ? p.def_src_port : (p.src_port ? p.src_port[i] : p.def_src_port);
        const uint32_t dp = AOS ? tv.z >> 16 : FULL ? p.dst_port[i] : PROBE ? p.def_dst_port : (p.dst_port ? p.dst_port[i] : p.def_dst_port);
        const uint32_t id = AOS ? tv.w & 0xFFFFu : FULL ? p.ip_id[i] : PROBE ? p.def_ip_id : (p.ip_id ? p.ip_id[i] : p.def_ip_id);
        const uint32_t ulen = 8u + p.payload_len, total = 20u + ulen;
        const uint64_t addr = (uint64_t)(src >> 16) + (src & 0xFFFFu) + (dst >> 16) + (dst & 0xFFFFu);
        // udp.rs:443-477 on to_bytes(): pseudo + sport + dport + length (+ payload)
        const uint32_t ucs = fold_complement(addr + 17u + ulen + sp + dp + ulen + pw);
        // ipv4.rs:932-938 on to_bytes()[..20]
        const uint32_t w0 = (0x45u << 8) | p.dscp_ecn, w3 = ((uint32_t)(p.ip_flags & 7u)) << 13;
        const uint32_t w4 = ((uint32_t)p.ttl << 8) | 17u;
        const uint32_t ics = fold_complement(addr + w0 + total + id + w3 + w4);
        uint8_t h[42];
        for (int k = 0; k < 6; k++) {
            h[k] = !FULL && !PROBE && !AOS && p.dst_mac ? p.dst_mac[i * 6 + k] : p.def_dst_mac[k];
            h[6 + k] = !FULL && !PROBE && !AOS && p.src_mac ? p.src_mac[i * 6 + k] : p.def_src_mac[k];
        }
        h[12] = 0x08; h[13] = 0x00;
        h[14] = (uint8_t)(w0 >> 8); h[15] = (uint8_t)w0;
        h[16] = (uint8_t)(total >> 8); h[17] = (uint8_t)total;
        h[18] = (uint8_t)(id >> 8); h[19] = (uint8_t)id;
        h[20] = (uint8_t)(w3 >> 8); h[21] = 0;
        h[22] = p.ttl; h[23] = 17;
        h[24] = (uint8_t)(ics >> 8); h[25] = (uint8_t)ics;
        h[26] = (uint8_t)(src >> 24); h[27] = (uint8_t)(src >> 16); h[28] = (uint8_t)(src >> 8); h[29] = (uint8_t)src;
        h[30] = (uint8_t)(dst >> 24); h[31] = (uint8_t)(dst >> 16); h[32] = (uint8_t)(dst >> 8); h[33] = (uint8_t)dst;
        h[34] = (uint8_t)(sp >> 8); h[35] = (uint8_t)sp;
        h[36] = (uint8_t)(dp >> 8); h[37] = (uint8_t)dp;
        h[38] = (uint8_t)(ulen >> 8); h[39] = (uint8_t)ulen;
        h[40] = (uint8_t)(ucs >> 8); h[41] = (uint8_t)ucs;
        if (STAGED) {
            const uint32_t d0 = tid * a.out_stride;
            uint8_t* d = smem + d0;
            uint32_t hw[21];
#pragma unroll
            for (int k = 0; k < 21; k++) hw[k] = (uint32_t)h[2 * k] | ((uint32_t)h[2 * k + 1] << 8);
            lds_put_frame_hw<21>(smem, d0, hw);  // dword writes at either parity of d0
            for (uint32_t k = 0; k < p.payload_len; k++) d[42 + k] = p.payload[k];
            for (uint32_t k = flen; k < a.out_stride; k++) d[k] = 0;
        } else {
            uint8_t* d = a.out + i * (uint64_t)a.out_stride;
#pragma unroll
            for (int k = 0; k < 42; k++) d[k] = h[k];
            for (uint32_t k = 0; k < p.payload_len; k++) d[42 + k] = p.payload[k];
        }
    }
    if (STAGED) {
        __syncthreads();
        build_copy_out(smem, a.out + first * a.out_stride, nf * a.out_stride);
    }
}

// ---- udp_ping IPv6 branch: builder/udp.rs:67-95 over IPv6 (udp.rs:480-505),
// Ipv6PacketBuilder::to_bytes (builder/ipv6.rs:89-152, ipv6.rs:50-75),
// EthernetPacketBuilder; 62 + payload_len bytes per frame.
struct Build6Args {
    nexg_udp6_build p;
    uint8_t* out;
    uint32_t out_stride;
    uint32_t tile_order;  // tile_index order (nexg_internal.hpp), as k_build_udp4
};

// PROBE: udp_ping's IPv6 probe batch: src_ip holds one address (src_shared),
// dst_ip one per frame, ports and MACs from the batch defaults: 16 B read per
// frame.
template <uint32_t MAXS, bool PROBE = false>
__global__ __launch_bounds__(256) void k_build_udp6(Build6Args a) {
    constexpr bool STAGED = MAXS != 0;
    __shared__ __attribute__((aligned(16))) uint8_t smem[STAGED ? kBuildTile * MAXS : 16];
    const nexg_udp6_build& p = a.p;
    const uint64_t first = tile_index(a.tile_order) * kBuildTile;
    const uint64_t left = p.count - first;
    const uint32_t nf = left < kBuildTile ? (uint32_t)left : kBuildTile;
    const uint32_t tid = threadIdx.x;
    const uint64_t i = first + tid;
    const uint32_t flen = 62u + p.payload_len;
    __shared__ uint32_t s_pay;
    const uint64_t pw = shared_payload_sum(p.payload, p.payload_len, &s_pay);
    if (tid < nf) {
        const uint64_t si = PROBE || p.src_shared ? 0u : i;  // one source for the whole batch
        // addresses are 4-B aligned (the ABI checks): dword loads
        const auto* s4 = NEXG_GLOBAL(uint32_t, p.src_ip + 16u * si);
        const auto* d4 = NEXG_GLOBAL(uint32_t, p.dst_ip + 16u * i);
        uint32_t sw[4], dw[4];
#pragma unroll
        for (int k = 0; k < 4; k++) { sw[k] = s4[k]; dw[k] = d4[k]; }
        const uint32_t sp = PROBE ? p.def_src_port : per_or_def(p.src_port, i, p.def_src_port);
        const uint32_t dp = PROBE ? p.def_dst_port : per_or_def(p.dst_port, i, p.def_dst_port);
        const uint32_t ulen = 8u + p.payload_len;
        // util.rs:111-133 pseudo-header: address segments (as LE halves x 256),
        // next header 17, length; then sport, dport, length, payload (skipword 3)
        uint32_t addr_le = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) addr_le += halves(sw[k]) + halves(dw[k]);
        const uint32_t ucs = fold_complement(256ull * addr_le + 17u + ulen + sp + dp + ulen + pw);
        const uint32_t fl = p.flow_label & 0xFFFFFu, tc = p.traffic_class;
        uint32_t hw[31];
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const uint8_t* dm = PROBE ? nullptr : p.dst_mac;
            const uint8_t* sm = PROBE ? nullptr : p.src_mac;
            const uint32_t b0 = per_or_def(dm, i * 6 + 2 * k, p.def_dst_mac[2 * k]);
            const uint32_t b1 = per_or_def(dm, i * 6 + 2 * k + 1, p.def_dst_mac[2 * k + 1]);
            const uint32_t c0 = per_or_def(sm, i * 6 + 2 * k, p.def_src_mac[2 * k]);
            const uint32_t c1 = per_or_def(sm, i * 6 + 2 * k + 1, p.def_src_mac[2 * k + 1]);
            hw[k] = b0 | (b1 << 8);
            hw[3 + k] = c0 | (c1 << 8);
        }
        hw[6] = 0xDD86u;                                              // EtherType 0x86DD
        hw[7] = ((6u << 4) | (tc >> 4)) | ((((tc & 0xFu) << 4) | (fl >> 16)) << 8);
        hw[8] = ((fl >> 8) & 0xFFu) | ((fl & 0xFFu) << 8);
        hw[9] = bswap16(ulen);                                        // payload length
        hw[10] = 17u | ((uint32_t)p.hop_limit << 8);                  // next header, hop limit
#pragma unroll
        for (int k = 0; k < 4; k++) {
            hw[11 + 2 * k] = sw[k] & 0xFFFFu; hw[12 + 2 * k] = sw[k] >> 16;
            hw[19 + 2 * k] = dw[k] & 0xFFFFu; hw[20 + 2 * k] = dw[k] >> 16;
        }
        hw[27] = bswap16(sp);
        hw[28] = bswap16(dp);
        hw[29] = bswap16(ulen);
        hw[30] = bswap16(ucs);  // computed 0 stays 0 (Q18)
        if (STAGED) {
            const uint32_t d0 = tid * a.out_stride;
            uint8_t* d = smem + d0;
            lds_put_frame_hw<31>(smem, d0, hw);
            for (uint32_t k = 0; k < p.payload_len; k++) d[62 + k] = p.payload[k];
            for (uint32_t k = flen; k < a.out_stride; k++) d[k] = 0;
        } else {
            uint8_t* d = a.out + i * (uint64_t)a.out_stride;
#pragma unroll
            for (int k = 0; k < 31; k++) { d[2 * k] = (uint8_t)hw[k]; d[2 * k + 1] = (uint8_t)(hw[k] >> 8); }
            for (uint32_t k = 0; k < p.payload_len; k++) d[62 + k] = p.payload[k];
        }
    }
    if (STAGED) {
        __syncthreads();
        build_copy_out(smem, a.out + first * a.out_stride, nf * a.out_stride);
    }
}

// ---- tcp_ping / icmp_ping: one kernel per (family, L4 kind) ----------------
// The header is a compile-time halfword layout (Ethernet 7, IPv4 10 / IPv6 20,
// TCP 10 / ICMP echo 4) built in registers, then the shared TCP options and
// payload; checksums in closed form: per-frame words + the options word sum
// (host-computed, passed in) + the payload word sum (computed once per
// workgroup into LDS).
enum { kL4Tcp = 6, kL4Icmp = 1 };

struct L4Args {
    nexg_ip_build ip;
    // TCP
    const uint16_t* sport;
    const uint16_t* dport;
    const uint32_t* seq;
    const uint32_t* ack;
    uint32_t def_seq, def_ack;
    uint16_t def_sport, def_dport, window, urg;
    uint32_t flags;
    uint32_t opt_padded;  // bytes, multiple of 4, <= 40
    uint32_t opt_sum;     // BE word sum of the padded options
    uint8_t options[40];
    // ICMP
    const uint16_t* ident;
    const uint16_t* seqno;
    uint16_t def_ident, def_seqno;
    uint32_t icmp_type, icmp_code;
    // shared
    const uint8_t* payload;
    uint32_t payload_len;
    uint64_t count;
    uint8_t* out;
    uint32_t out_stride;
    uint32_t tile_order;  // tile_index order (nexg_internal.hpp), as k_build_udp4
};

// halfword v (memory order: low byte first) at LDS/global byte offset p
__device__ __forceinline__ void put_hw(uint8_t* base, uint32_t p, uint32_t v, bool odd) {
    if (odd) {
        base[p] = (uint8_t)v;
        base[p + 1] = (uint8_t)(v >> 8);
    } else {
        *reinterpret_cast<uint16_t*>(base + p) = (uint16_t)v;
    }
}

// PROBE: a tcp_ping / icmp_ping probe batch (ip.src_shared, every other
// per-frame array NULL): only the destination is read per frame (4 / 16 B);
// source, ports, seq / ack, identifier / sequence, id and MACs are the batch's.
template <int FAM, int KIND, uint32_t MAXS, bool PROBE = false>
__global__ __launch_bounds__(256) void k_build_l4(L4Args a) {
    constexpr bool STAGED = MAXS != 0;
    constexpr int NIP = FAM == 4 ? 10 : 20;             // IP header halfwords
    constexpr int NL4 = KIND == kL4Tcp ? 10 : 4;        // fixed L4 header halfwords
    constexpr int NH = 7 + NIP + NL4;
    static_assert(NH % 2 == 1, "lds_put_halfwords takes an odd halfword count");
    __shared__ __attribute__((aligned(16))) uint8_t smem[STAGED ? kBuildTile * MAXS : 16];
    __shared__ uint32_t s_pay;
    const uint32_t tid = threadIdx.x;
    const uint64_t first = tile_index(a.tile_order) * kBuildTile;
    const uint64_t left = a.count - first;
    const uint32_t nf = left < kBuildTile ? (uint32_t)left : kBuildTile;
    const uint64_t i = first + tid;
    const uint32_t pay_sum = shared_payload_sum(a.payload, a.payload_len, &s_pay);
    const uint32_t l4_hdr = KIND == kL4Tcp ? 20u + a.opt_padded : 8u;
    const uint32_t l4_len = l4_hdr + a.payload_len;
    const uint32_t flen = 14u + 2u * NIP + l4_len;
    if (tid < nf) {
        const nexg_ip_build& ip = a.ip;
        constexpr uint32_t AW = FAM == 4 ? 1u : 4u;  // address dwords
        const uint64_t si = PROBE || ip.src_shared ? 0u : i;  // one source for the whole batch
        uint32_t sw[AW], dw[AW];
#pragma unroll
        for (uint32_t k = 0; k < AW; k++) {
            sw[k] = NEXG_GLOBAL(uint32_t, ip.src_ip)[AW * si + k];
            dw[k] = NEXG_GLOBAL(uint32_t, ip.dst_ip)[AW * i + k];
        }
        uint32_t addr_le = 0;  // address words as LE halves: x256 gives the BE sum (mod 0xFFFF)
#pragma unroll
        for (int k = 0; k < (FAM == 4 ? 1 : 4); k++) addr_le += halves(sw[k]) + halves(dw[k]);
        uint32_t hw[NH];
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const uint8_t* dm = PROBE ? nullptr : ip.dst_mac;
            const uint8_t* sm = PROBE ? nullptr : ip.src_mac;
            const uint32_t b0 = per_or_def(dm, i * 6 + 2 * k, ip.def_dst_mac[2 * k]);
            const uint32_t b1 = per_or_def(dm, i * 6 + 2 * k + 1, ip.def_dst_mac[2 * k + 1]);
            const uint32_t c0 = per_or_def(sm, i * 6 + 2 * k, ip.def_src_mac[2 * k]);
            const uint32_t c1 = per_or_def(sm, i * 6 + 2 * k + 1, ip.def_src_mac[2 * k + 1]);
            hw[k] = b0 | (b1 << 8);
            hw[3 + k] = c0 | (c1 << 8);
        }
        const uint32_t proto = KIND == kL4Tcp ? 6u : (FAM == 4 ? 1u : 58u);
        // ---- L4 header + checksum ----
        uint64_t t;
        constexpr int L = 7 + NIP;  // first L4 halfword
        if (KIND == kL4Tcp) {
            const uint32_t sp = PROBE ? a.def_sport : per_or_def(a.sport, i, a.def_sport);
            const uint32_t dp = PROBE ? a.def_dport : per_or_def(a.dport, i, a.def_dport);
            const uint32_t sq = PROBE ? a.def_seq : per_or_def(a.seq, i, a.def_seq);
            const uint32_t ak = PROBE ? a.def_ack : per_or_def(a.ack, i, a.def_ack);
            const uint32_t w6 = ((l4_hdr / 4u) << 12) | (a.flags & 0xFFu);
            t = sp + dp + (sq >> 16) + (sq & 0xFFFFu) + (ak >> 16) + (ak & 0xFFFFu) + w6 + a.window + a.urg +
                a.opt_sum + pay_sum;
            hw[L + 0] = bswap16(sp); hw[L + 1] = bswap16(dp);
            hw[L + 2] = bswap16(sq >> 16); hw[L + 3] = bswap16(sq & 0xFFFFu);
            hw[L + 4] = bswap16(ak >> 16); hw[L + 5] = bswap16(ak & 0xFFFFu);
            hw[L + 6] = bswap16(w6); hw[L + 7] = bswap16(a.window);
            hw[L + 9] = bswap16(a.urg);
        } else {
            const uint32_t id = PROBE ? a.def_ident : per_or_def(a.ident, i, a.def_ident);
            const uint32_t sq = PROBE ? a.def_seqno : per_or_def(a.seqno, i, a.def_seqno);
            const uint32_t w0 = (a.icmp_type << 8) | a.icmp_code;
            t = w0 + id + sq + pay_sum;
            hw[L + 0] = bswap16(w0);
            hw[L + 2] = bswap16(id); hw[L + 3] = bswap16(sq);
        }
        if (FAM == 6 || KIND == kL4Tcp) t += 256ull * addr_le + proto + l4_len;  // pseudo-header
        const uint32_t cs = fold_complement(t);  // computed 0 stays 0 (Q18)
        hw[KIND == kL4Tcp ? L + 8 : L + 1] = bswap16(cs);
        // ---- IP header ----
        if (FAM == 4) {
            const uint32_t total = 20u + l4_len, id = PROBE ? ip.def_ip_id : per_or_def(ip.ip_id, i, ip.def_ip_id);
            const uint32_t w0 = (0x45u << 8) | ip.tos, w3 = ((uint32_t)(ip.ip_flags & 7u)) << 13;
            const uint32_t w4 = ((uint32_t)ip.ttl << 8) | proto;
            const uint32_t ics = fold_complement(256ull * addr_le + w0 + total + id + w3 + w4);
            hw[6] = 0x0008u;
            hw[7] = bswap16(w0); hw[8] = bswap16(total); hw[9] = bswap16(id); hw[10] = bswap16(w3);
            hw[11] = bswap16(w4); hw[12] = bswap16(ics);
            hw[13] = sw[0] & 0xFFFFu; hw[14] = sw[0] >> 16; hw[15] = dw[0] & 0xFFFFu; hw[16] = dw[0] >> 16;
        } else {
            const uint32_t fl = ip.flow_label & 0xFFFFFu, tc = ip.tos;
            hw[6] = 0xDD86u;
            hw[7] = ((6u << 4) | (tc >> 4)) | ((((tc & 0xFu) << 4) | (fl >> 16)) << 8);
            hw[8] = ((fl >> 8) & 0xFFu) | ((fl & 0xFFu) << 8);
            hw[9] = bswap16(l4_len);
            hw[10] = proto | ((uint32_t)ip.ttl << 8);
#pragma unroll
            for (int k = 0; k < 4; k++) {
                hw[11 + 2 * k] = sw[k] & 0xFFFFu; hw[12 + 2 * k] = sw[k] >> 16;
                hw[19 + 2 * k] = dw[k] & 0xFFFFu; hw[20 + 2 * k] = dw[k] >> 16;
            }
        }
        // ---- write: fixed halfwords, options, payload, zero gap ----
        uint8_t* base = STAGED ? smem : a.out + first * a.out_stride;
        const uint32_t d0 = tid * a.out_stride;
        const bool odd = (a.out_stride & 1u) != 0;
        if (STAGED) {
            lds_put_frame_hw<NH>(base, d0, hw);  // dword writes at either parity
        } else {
#pragma unroll
            for (int k = 0; k < NH; k++) put_hw(base, d0 + 2u * k, hw[k], odd);
        }
        uint32_t p = d0 + 2u * NH;
        if (KIND == kL4Tcp) {
            // unrolled over the 40-B maximum with a uniform guard: constant
            // kernarg offsets become scalar loads, where a run-time index made
            // one vector load + vmcnt(0) wait per option halfword pair
#pragma unroll
            for (uint32_t k = 0; k < 40u; k += 2)
                if (k < a.opt_padded) put_hw(base, p + k, a.options[k] | ((uint32_t)a.options[k + 1] << 8), odd);
            p += a.opt_padded;
        }
        for (uint32_t k = 0; k < a.payload_len; k++) base[p + k] = a.payload[k];
        if (STAGED)
            for (uint32_t k = flen; k < a.out_stride; k++) base[d0 + k] = 0;
    }
    if (STAGED) {
        __syncthreads();
        build_copy_out(smem, a.out + first * a.out_stride, nf * a.out_stride);
    }
}

template <int FAM, int KIND, bool PROBE>
static void launch_l4_form(const L4Args& a, hipStream_t s) {
    const uint64_t blocks = (a.count + kBuildTile - 1) / kBuildTile;
    const bool staged = a.out_stride <= kBuildMaxStride && (reinterpret_cast<uint64_t>(a.out) & 15u) == 0;
    // IPv6: 16-KiB tile + build_lds_pad() -> 5 workgroups per CU (icmp6 echo
    // 0.29 -> 0.26 ms at 16M frames); IPv4 shapes run faster at 8 per CU (tcp
    // SYN 0.21 vs 0.24-0.26 ms, icmp echo 0.132 vs 0.140; profiles/r04/builders/)
    const uint32_t pad = FAM == 6 || PROBE ? build_lds_pad() : 0u;
    if (staged && a.out_stride <= 64u)
        hipLaunchKernelGGL((k_build_l4<FAM, KIND, 64, PROBE>), dim3((uint32_t)blocks), dim3(kBuildTile), pad, s, a);
    else if (staged && a.out_stride <= 80u)  // tcp_ping's 66 B: a 20-KiB tile (7 per CU) instead of 32 KiB (4)
        hipLaunchKernelGGL((k_build_l4<FAM, KIND, 80, PROBE>), dim3((uint32_t)blocks), dim3(kBuildTile),
                           pad > 4096u ? pad - 4096u : 0u, s, a);
    else if (staged)
        hipLaunchKernelGGL((k_build_l4<FAM, KIND, kBuildMaxStride, PROBE>), dim3((uint32_t)blocks), dim3(kBuildTile),
                           0, s, a);
    else
        hipLaunchKernelGGL((k_build_l4<FAM, KIND, 0, PROBE>), dim3((uint32_t)blocks), dim3(kBuildTile), 0, s, a);
}

template <int FAM, int KIND>
static void launch_l4_fam(const L4Args& a, hipStream_t s) {
    // the probe batch: one source, a destination per frame, nothing else per frame
    const bool probe = a.ip.src_shared && !a.ip.ip_id && !a.ip.src_mac && !a.ip.dst_mac &&
                       (KIND == kL4Tcp ? !a.sport && !a.dport && !a.seq && !a.ack : !a.ident && !a.seqno);
    if (probe) launch_l4_form<FAM, KIND, true>(a, s);
    else launch_l4_form<FAM, KIND, false>(a, s);
}

static hipError_t launch_l4(L4Args& a, int kind, hipStream_t s) {
    if (a.count == 0) return hipSuccess;
    a.tile_order = l4_build_tile_order();
    if (kind == kL4Tcp) {
        if (a.ip.family == 4) launch_l4_fam<4, kL4Tcp>(a, s);
        else launch_l4_fam<6, kL4Tcp>(a, s);
    } else {
        if (a.ip.family == 4) launch_l4_fam<4, kL4Icmp>(a, s);
        else launch_l4_fam<6, kL4Icmp>(a, s);
    }
    return hipGetLastError();
}

hipError_t launch_build_tcp(const nexg_tcp_build& p, uint8_t* out, uint32_t out_stride, hipStream_t s) {
    L4Args a{};
    a.ip = p.ip;
    a.sport = p.src_port; a.dport = p.dst_port; a.seq = p.seq; a.ack = p.ack;
    a.def_seq = p.def_seq; a.def_ack = p.def_ack; a.def_sport = p.def_src_port; a.def_dport = p.def_dst_port;
    a.window = p.window; a.urg = p.urgent_ptr; a.flags = p.flags;
    a.opt_padded = (p.options_len + 3u) & ~3u;
    for (uint32_t k = 0; k < 40; k++) a.options[k] = k < p.options_len ? p.options[k] : 0;
    for (uint32_t k = 0; k < a.opt_padded; k += 2) a.opt_sum += ((uint32_t)a.options[k] << 8) | a.options[k + 1];
    a.payload = p.payload; a.payload_len = p.payload_len; a.count = p.count;
    a.out = out; a.out_stride = out_stride;
    return launch_l4(a, kL4Tcp, s);
}

hipError_t launch_build_icmp_echo(const nexg_icmp_echo_build& p, uint8_t* out, uint32_t out_stride,
                                  hipStream_t s) {
    L4Args a{};
    a.ip = p.ip;
    a.ident = p.identifier; a.seqno = p.sequence; a.def_ident = p.def_identifier; a.def_seqno = p.def_sequence;
    a.icmp_type = p.icmp_type; a.icmp_code = p.icmp_code;
    a.payload = p.payload; a.payload_len = p.payload_len; a.count = p.count;
    a.out = out; a.out_stride = out_stride;
    return launch_l4(a, kL4Icmp, s);
}

// ---- arp / ndp probes ------------------------------------------------------
// One lane per frame: the frame's halfwords (memory order, low byte first)
// assembled in registers, written to the LDS tile and copied out coalesced
// like the other builders. 6-B address fields are read bytewise (any
// alignment); IPv6 addresses as dwords (4-B aligned, nexg_ip_build).

__device__ __forceinline__ uint32_t mac_hw(const uint8_t* per, const uint8_t* def, uint64_t i, int k) {
    const uint8_t* m = per ? per + 6u * i : def;
    return (uint32_t)m[2 * k] | ((uint32_t)m[2 * k + 1] << 8);
}

struct ArpArgs {
    nexg_arp_build p;
    uint8_t* out;
    uint32_t out_stride;
};

// builder/arp.rs:18-37 + arp.rs:385-399 behind Ethernet (examples/arp.rs:59-67)
template <uint32_t MAXS>
__global__ __launch_bounds__(256) void k_build_arp(ArpArgs a) {
    constexpr bool STAGED = MAXS != 0;
    __shared__ __attribute__((aligned(16))) uint8_t smem[STAGED ? kBuildTile * MAXS : 16];
    const nexg_arp_build& p = a.p;
    const uint32_t tid = threadIdx.x;
    const uint64_t first = (uint64_t)blockIdx.x * kBuildTile;
    const uint64_t left = p.count - first;
    const uint32_t nf = left < kBuildTile ? (uint32_t)left : kBuildTile;
    const uint64_t i = first + tid;
    if (tid < nf) {
        uint32_t hw[21];
#pragma unroll
        for (int k = 0; k < 3; k++) {
            hw[k] = mac_hw(p.eth_dst, p.def_eth_dst, i, k);
            hw[3 + k] = mac_hw(p.sender_mac, p.def_sender_mac, i, k);
        }
        hw[6] = 0x0608u;  // EtherType 0x0806
        hw[7] = bswap16(p.hardware_type);
        hw[8] = bswap16(p.protocol_type);
        hw[9] = (uint32_t)p.hw_addr_len | ((uint32_t)p.proto_addr_len << 8);
        hw[10] = bswap16(p.operation);
#pragma unroll
        for (int k = 0; k < 3; k++) hw[11 + k] = hw[3 + k];  // sender_hw_addr
        const uint8_t* sip = p.sender_ip ? p.sender_ip + 4u * i : p.def_sender_ip;
        const uint8_t* tip = p.target_ip + 4u * i;
        hw[14] = (uint32_t)sip[0] | ((uint32_t)sip[1] << 8);
        hw[15] = (uint32_t)sip[2] | ((uint32_t)sip[3] << 8);
#pragma unroll
        for (int k = 0; k < 3; k++) hw[16 + k] = mac_hw(p.target_mac, p.def_target_mac, i, k);
        hw[19] = (uint32_t)tip[0] | ((uint32_t)tip[1] << 8);
        hw[20] = (uint32_t)tip[2] | ((uint32_t)tip[3] << 8);
        uint8_t* base = STAGED ? smem : a.out + first * a.out_stride;
        const uint32_t d0 = tid * a.out_stride;
        const bool odd = (a.out_stride & 1u) != 0;
#pragma unroll
        for (int k = 0; k < 21; k++) put_hw(base, d0 + 2u * k, hw[k], odd);
        if (STAGED)
            for (uint32_t k = 42; k < a.out_stride; k++) base[d0 + k] = 0;
    }
    if (STAGED) {
        __syncthreads();
        build_copy_out(smem, a.out + first * a.out_stride, nf * a.out_stride);
    }
}

struct NdpArgs {
    nexg_ndp_ns_build p;
    uint8_t* out;
    uint32_t out_stride;
};

// builder/ndp.rs:30-84 (NS + SourceLLAddr option, icmpv6::checksum) inside
// Ipv6PacketBuilder + EthernetPacketBuilder (examples/ndp.rs:82-108)
template <uint32_t MAXS>
__global__ __launch_bounds__(256) void k_build_ndp_ns(NdpArgs a) {
    constexpr bool STAGED = MAXS != 0;
    constexpr int NH = 43;  // 86 B
    __shared__ __attribute__((aligned(16))) uint8_t smem[STAGED ? kBuildTile * MAXS : 16];
    const nexg_ndp_ns_build& p = a.p;
    const nexg_ip_build& ip = p.ip;
    const uint32_t tid = threadIdx.x;
    const uint64_t first = (uint64_t)blockIdx.x * kBuildTile;
    const uint64_t left = p.count - first;
    const uint32_t nf = left < kBuildTile ? (uint32_t)left : kBuildTile;
    const uint64_t i = first + tid;
    if (tid < nf) {
        uint32_t sw[4], dw[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            sw[k] = reinterpret_cast<const uint32_t*>(ip.src_ip + 16u * i)[k];
            dw[k] = reinterpret_cast<const uint32_t*>(ip.dst_ip + 16u * i)[k];
        }
        uint32_t hw[NH];
        const bool mc = p.eth_dst_multicast != 0;
        // Ethernet: dst (33:33 + target bytes 12..15, or given), src, 0x86DD
        hw[0] = mc ? 0x3333u : mac_hw(ip.dst_mac, ip.def_dst_mac, i, 0);
        hw[1] = mc ? (dw[3] & 0xFFFFu) : mac_hw(ip.dst_mac, ip.def_dst_mac, i, 1);
        hw[2] = mc ? (dw[3] >> 16) : mac_hw(ip.dst_mac, ip.def_dst_mac, i, 2);
#pragma unroll
        for (int k = 0; k < 3; k++) hw[3 + k] = mac_hw(ip.src_mac, ip.def_src_mac, i, k);
        hw[6] = 0xDD86u;
        // IPv6 header (ipv6.rs:50-75): version 6, traffic class, flow label, payload 32, next 58, hop limit
        const uint32_t fl = ip.flow_label & 0xFFFFFu, tc = ip.tos;
        hw[7] = ((6u << 4) | (tc >> 4)) | ((((tc & 0xFu) << 4) | (fl >> 16)) << 8);
        hw[8] = ((fl >> 8) & 0xFFu) | ((fl & 0xFFu) << 8);
        hw[9] = bswap16(32u);
        hw[10] = 58u | ((uint32_t)ip.ttl << 8);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            hw[11 + 2 * k] = sw[k] & 0xFFFFu; hw[12 + 2 * k] = sw[k] >> 16;
            hw[19 + 2 * k] = dw[k] & 0xFFFFu; hw[20 + 2 * k] = dw[k] >> 16;
        }
        // NeighborSolicit: type 135 code 0, checksum, reserved 0, target = dst, option 1 / len 1 / MAC
        constexpr int L = 27;
        hw[L + 0] = 135u;
        hw[L + 2] = 0u; hw[L + 3] = 0u;
#pragma unroll
        for (int k = 0; k < 8; k++) hw[L + 4 + k] = hw[19 + k];
        hw[L + 12] = 0x0101u;
#pragma unroll
        for (int k = 0; k < 3; k++) hw[L + 13 + k] = hw[3 + k];
        // icmpv6::checksum (util.rs:91-137): pseudo-header (src, dst, length 32, next header 58)
        // + the message with its checksum word skipped; memory-order halfwords are
        // little-endian, x256 gives the big-endian sum (mod 0xFFFF)
        uint32_t le = 0;
#pragma unroll
        for (int k = 0; k < 16; k++) le += hw[11 + k];   // src + dst
#pragma unroll
        for (int k = 0; k < 8; k++) le += hw[L + 4 + k];  // target
#pragma unroll
        for (int k = 0; k < 3; k++) le += hw[L + 13 + k]; // MAC
        const uint64_t t = 256ull * le + 58u + 32u + (135u << 8) + 0x0101u;
        hw[L + 1] = bswap16(fold_complement(t));
        uint8_t* base = STAGED ? smem : a.out + first * a.out_stride;
        const uint32_t d0 = tid * a.out_stride;
        const bool odd = (a.out_stride & 1u) != 0;
#pragma unroll
        for (int k = 0; k < NH; k++) put_hw(base, d0 + 2u * k, hw[k], odd);
        if (STAGED)
            for (uint32_t k = 86; k < a.out_stride; k++) base[d0 + k] = 0;
    }
    if (STAGED) {
        __syncthreads();
        build_copy_out(smem, a.out + first * a.out_stride, nf * a.out_stride);
    }
}

hipError_t launch_build_arp(const nexg_arp_build& p, uint8_t* out, uint32_t out_stride, hipStream_t s) {
    if (p.count == 0) return hipSuccess;
    ArpArgs a{p, out, out_stride};
    const dim3 grid((uint32_t)((p.count + kBuildTile - 1) / kBuildTile)), blk(kBuildTile);
    const bool staged = out_stride <= kBuildMaxStride && (reinterpret_cast<uint64_t>(out) & 15u) == 0;
    if (staged && out_stride <= 64u) hipLaunchKernelGGL(k_build_arp<64>, grid, blk, 0, s, a);
    else if (staged) hipLaunchKernelGGL(k_build_arp<kBuildMaxStride>, grid, blk, 0, s, a);
    else hipLaunchKernelGGL(k_build_arp<0>, grid, blk, 0, s, a);
    return hipGetLastError();
}

hipError_t launch_build_ndp_ns(const nexg_ndp_ns_build& p, uint8_t* out, uint32_t out_stride, hipStream_t s) {
    if (p.count == 0) return hipSuccess;
    NdpArgs a{p, out, out_stride};
    const dim3 grid((uint32_t)((p.count + kBuildTile - 1) / kBuildTile)), blk(kBuildTile);
    const bool staged = out_stride <= kBuildMaxStride && (reinterpret_cast<uint64_t>(out) & 15u) == 0;
    if (staged) hipLaunchKernelGGL(k_build_ndp_ns<kBuildMaxStride>, grid, blk, 0, s, a);
    else hipLaunchKernelGGL(k_build_ndp_ns<0>, grid, blk, 0, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------- generators

__global__ void k_gen_lengths(int workload, uint64_t seed, uint64_t first, uint64_t count,
                              uint32_t* lengths) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    uint32_t len = 64, proto = 1;
    if (workload == NEXG_WL_IMIX) imix_class(seed ^ ((first + i) * kPhi), len, proto);
    lengths[i] = len;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

constexpr uint32_t kGenBuf = 1536;  // >= 1500, multiple of 16

// one wave per frame; four waves per block, grid-stride, block-uniform loop
__global__ __launch_bounds__(256) void k_gen_frames(int workload, uint64_t seed, uint64_t first,
                                                    uint64_t count, uint8_t* data,
                                                    const uint64_t* offsets, uint32_t stride) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[4 * kGenBuf];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint8_t* b = smem + wave * kGenBuf;
    const uint64_t nblocks = gridDim.x;
    for (uint64_t base = (uint64_t)blockIdx.x * 4; base < count; base += nblocks * 4) {
        const uint64_t li = base + wave;
        const bool active = li < count;
        const uint64_t s0 = seed ^ ((first + li) * kPhi);
        uint32_t len = 64, proto = 1, d0 = 0;
        if (workload == NEXG_WL_IMIX) d0 = imix_class(s0, len, proto);
        const uint32_t nwords = (len + 7u) / 8u;
        if (active) {
            for (uint32_t k = lane; k < nwords; k += 64) {
                const uint64_t r = draw(s0, d0 + k);
                reinterpret_cast<uint2*>(b)[k] = make_uint2((uint32_t)r, (uint32_t)(r >> 32));
            }
        }
        __syncthreads();
        const bool v6 = proto >= 3u;
        const uint32_t l4p = proto % 3u;  // 0 tcp, 1 udp, 2 icmp
        const uint32_t l4 = v6 ? 54u : 34u, n = len - l4;
        const uint32_t pr = l4p == 0u ? 6u : (l4p == 1u ? 17u : (v6 ? 58u : 1u));
        const uint32_t skip = l4p == 0u ? 8u : (l4p == 1u ? 3u : 1u);
        if (active && lane == 0) {
            b[0] &= 0xFE;
            b[6] &= 0xFE;
            uint8_t* t = b + l4;
            if (!v6) {
                b[12] = 0x08; b[13] = 0x00; b[14] = 0x45;
                b[16] = (uint8_t)((len - 14u) >> 8); b[17] = (uint8_t)(len - 14u);
                b[20] = 0x40; b[21] = 0x00; b[22] = 64; b[23] = (uint8_t)pr;
                b[24] = 0; b[25] = 0;
            } else {
                b[12] = 0x86; b[13] = 0xDD;
                b[14] = (uint8_t)(0x60u | (b[14] & 0x0Fu));
                b[18] = (uint8_t)((len - 54u) >> 8); b[19] = (uint8_t)(len - 54u);
                b[20] = (uint8_t)pr; b[21] = 64;
            }
            if (l4p == 0u) {
                t[12] = 0x50; t[16] = 0; t[17] = 0; t[18] = 0; t[19] = 0;
            } else if (l4p == 1u) {
                t[4] = (uint8_t)(n >> 8); t[5] = (uint8_t)n; t[6] = 0; t[7] = 0;
            } else {
                t[0] = v6 ? 128 : 8; t[1] = 0; t[2] = 0; t[3] = 0;
            }
        }
        __syncthreads();
        // L4 word sum over [l4, len) (checksum field is zero), l4 even
        uint32_t part = 0;
        if (active) {
            const uint32_t A = l4, B = len;
            const uint32_t* w = reinterpret_cast<const uint32_t*>(b);
            for (uint32_t j = (A & ~3u) + 4u * lane; j < B; j += 256u) {
                uint32_t v = w[j >> 2];
                uint32_t lo = A > j ? A - j : 0u, hi = (B - j) < 4u ? B - j : 4u;
                uint32_t m = (hi >= 4u ? 0xFFFFFFFFu : ((1u << (8u * hi)) - 1u)) & (0xFFFFFFFFu << (8u * lo));
                v &= m;
                part += (v & 0xFFFFu) + (v >> 16);
            }
        }
        const uint32_t s_le = wave_sum(part);
        if (active && lane == 0) {
            auto be = [&](uint32_t k) { return ((uint32_t)b[k] << 8) | b[k + 1]; };
            uint64_t addr = 0;
            if (!v6) {
                uint64_t ih = 0;
                for (uint32_t k = 14; k < 34; k += 2) ih += be(k);
                const uint32_t ics = fold_complement(ih);
                b[24] = (uint8_t)(ics >> 8); b[25] = (uint8_t)ics;
                for (uint32_t k = 26; k < 34; k += 2) addr += be(k);
            } else {
                for (uint32_t k = 22; k < 54; k += 2) addr += be(k);
            }
            uint64_t t = ((uint64_t)s_le) << 8;
            if (!(l4p == 2u && !v6)) t += addr + pr + n;
            const uint32_t cs = fold_complement(t);
            uint8_t* f = b + l4 + 2u * skip;
            f[0] = (uint8_t)(cs >> 8); f[1] = (uint8_t)cs;
            const uint64_t c = draw(s0, d0 + nwords);
            if ((c & 15u) == 0u) {
                const uint32_t field = (uint32_t)(c >> 4) & 1u, bit = (uint32_t)(c >> 8) & 15u;
                uint8_t* q = (!v6 && field == 0u) ? b + 24 : f;
                const uint32_t v = (((uint32_t)q[0] << 8) | q[1]) ^ (1u << bit);
                q[0] = (uint8_t)(v >> 8); q[1] = (uint8_t)v;
            }
        }
        __syncthreads();
        if (active) {
            uint8_t* dst = data + (offsets ? offsets[li] : li * (uint64_t)stride);
            if ((reinterpret_cast<uint64_t>(dst) & 3u) == 0u) {
                for (uint32_t k = lane; k < len / 4u; k += 64)
                    reinterpret_cast<uint32_t*>(dst)[k] = reinterpret_cast<const uint32_t*>(b)[k];
                for (uint32_t k = (len & ~3u) + lane; k < len; k += 64) dst[k] = b[k];
            } else {
                for (uint32_t k = lane; k < len; k += 64) dst[k] = b[k];
            }
        }
        __syncthreads();
    }
}

__global__ void k_gen_udp4_params(uint64_t seed, uint64_t first, uint64_t count, uint32_t* src_ip,
                                  uint32_t* dst_ip, uint16_t* sport, uint16_t* dport,
                                  uint16_t* ip_id) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint64_t s0 = seed ^ ((first + i) * kPhi);
    const uint64_t r0 = draw(s0, 0), r1 = draw(s0, 1);
    src_ip[i] = (uint32_t)r0;
    dst_ip[i] = (uint32_t)(r0 >> 32);
    sport[i] = (uint16_t)r1;
    dport[i] = (uint16_t)(r1 >> 16);
    ip_id[i] = (uint16_t)(r1 >> 32);
}

// --------------------------------------------------------------- launchers

hipError_t launch_build_udp4_tuples(const nexg_udp4_build& p, const nexg_udp4_tuple* tuples, uint8_t* out,
                                    uint32_t out_stride, hipStream_t s) {
    if (p.count == 0) return hipSuccess;
    BuildArgs a{p, out, out_stride, tuples, build_tile_order()};
    const uint64_t blocks = (p.count + kBuildTile - 1) / kBuildTile;
    const bool staged = out_stride <= kBuildMaxStride && (reinterpret_cast<uint64_t>(out) & 15u) == 0;
    const uint32_t pad = build_lds_pad();
    if (staged && out_stride <= 64u)
        hipLaunchKernelGGL((k_build_udp4<64, false, false, true>), dim3((uint32_t)blocks), dim3(kBuildTile), pad, s, a);
    else if (staged)
        hipLaunchKernelGGL((k_build_udp4<kBuildMaxStride, false, false, true>), dim3((uint32_t)blocks), dim3(kBuildTile),
                           0, s, a);
    else
        hipLaunchKernelGGL((k_build_udp4<0, false, false, true>), dim3((uint32_t)blocks), dim3(kBuildTile), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_build_udp4(const nexg_udp4_build& p, uint8_t* out, uint32_t out_stride,
                             hipStream_t s) {
    if (p.count == 0) return hipSuccess;
    BuildArgs a{p, out, out_stride, nullptr, build_tile_order()};
    const uint64_t blocks = (p.count + kBuildTile - 1) / kBuildTile;
    const bool staged = out_stride <= kBuildMaxStride && (reinterpret_cast<uint64_t>(out) & 15u) == 0;
    const bool full = p.src_ip && p.src_port && p.dst_port && p.ip_id && !p.src_mac && !p.dst_mac;
    const bool probe = !p.src_ip && !p.src_port && !p.dst_port && !p.ip_id && !p.src_mac && !p.dst_mac;
    // the udp_ping shapes: a 16-KiB tile + build_lds_pad() -> 5 workgroups per CU
    const uint32_t pad = build_lds_pad();
    if (staged && out_stride <= 64u && full)
        hipLaunchKernelGGL((k_build_udp4<64, true>), dim3((uint32_t)blocks), dim3(kBuildTile), pad, s, a);
    else if (staged && out_stride <= 64u && probe)
        hipLaunchKernelGGL((k_build_udp4<64, false, true>), dim3((uint32_t)blocks), dim3(kBuildTile), pad, s, a);
    else if (staged && out_stride <= 64u)
        hipLaunchKernelGGL(k_build_udp4<64>, dim3((uint32_t)blocks), dim3(kBuildTile), 0, s, a);
    else if (staged)
        hipLaunchKernelGGL(k_build_udp4<kBuildMaxStride>, dim3((uint32_t)blocks), dim3(kBuildTile), 0, s, a);
    else
        hipLaunchKernelGGL(k_build_udp4<0>, dim3((uint32_t)blocks), dim3(kBuildTile), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_build_udp6(const nexg_udp6_build& p, uint8_t* out, uint32_t out_stride,
                             hipStream_t s) {
    if (p.count == 0) return hipSuccess;
    Build6Args a{p, out, out_stride, l4_build_tile_order()};
    const uint64_t blocks = (p.count + kBuildTile - 1) / kBuildTile;
    const bool staged = out_stride <= kBuildMaxStride && (reinterpret_cast<uint64_t>(out) & 15u) == 0;
    const bool probe = p.src_shared && !p.src_port && !p.dst_port && !p.src_mac && !p.dst_mac;
    // a 16-KiB tile for the udp_ping shapes + build_lds_pad(): 5 workgroups per CU (0.279 -> 0.253 ms)
    if (staged && out_stride <= 64u && probe)
        hipLaunchKernelGGL((k_build_udp6<64, true>), dim3((uint32_t)blocks), dim3(kBuildTile), build_lds_pad(), s, a);
    else if (staged && out_stride <= 64u)
        hipLaunchKernelGGL(k_build_udp6<64>, dim3((uint32_t)blocks), dim3(kBuildTile), build_lds_pad(), s, a);
    else if (staged)
        hipLaunchKernelGGL(k_build_udp6<kBuildMaxStride>, dim3((uint32_t)blocks), dim3(kBuildTile), 0, s, a);
    else
        hipLaunchKernelGGL(k_build_udp6<0>, dim3((uint32_t)blocks), dim3(kBuildTile), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_gen_lengths(int workload, uint64_t seed, uint64_t first, uint64_t count,
                              uint32_t* lengths, hipStream_t s) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gen_lengths, dim3((uint32_t)((count + 255) / 256)), dim3(256), 0, s,
                       workload, seed, first, count, lengths);
    return hipGetLastError();
}

hipError_t launch_gen_frames(int workload, uint64_t seed, uint64_t first, uint64_t count,
                             uint8_t* data, const uint64_t* offsets, uint32_t stride,
                             hipStream_t s) {
    if (count == 0) return hipSuccess;
    uint64_t blocks = (count + 3) / 4;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_gen_frames, dim3((uint32_t)blocks), dim3(256), 0, s, workload, seed, first,
                       count, data, offsets, stride);
    return hipGetLastError();
}

hipError_t launch_gen_udp4_params(uint64_t seed, uint64_t first, uint64_t count,
                                  uint32_t* src_ip, uint32_t* dst_ip, uint16_t* sport,
                                  uint16_t* dport, uint16_t* ip_id, hipStream_t s) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gen_udp4_params, dim3((uint32_t)((count + 255) / 256)), dim3(256), 0, s,
                       seed, first, count, src_ip, dst_ip, sport, dport, ip_id);
    return hipGetLastError();
}

}  // namespace nexg
