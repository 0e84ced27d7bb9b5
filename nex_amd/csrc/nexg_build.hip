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
#ifdef NEXG_AB_KNOBS
        const char* e = getenv("NEXG_BUILD_LDS_PAD");
#else
        const char* e = nullptr;  // product build: no environment overrides
#endif
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
// Phase timing of the builders' workgroups (measurement builds only:
// -DNEXG_PROBE_TIMING=1, tools/probe_timing.py): thread 0 of workgroup b
// stores s_memtime at phase k into g_build_stamps[8 b + k] (k = 6, 7:
// s_memrealtime at entry and exit); the product library has none of it.
#ifndef NEXG_PROBE_TIMING
#define NEXG_PROBE_TIMING 0
#endif
#if NEXG_PROBE_TIMING
constexpr uint32_t kStampWgs = 1u << 18;
__device__ uint64_t g_build_stamps[8u * kStampWgs];
#define NEXG_BUILD_STAMP(k)                                                                    \
    do {                                                                                       \
        if (threadIdx.x == 0 && blockIdx.x < kStampWgs)                                        \
            g_build_stamps[8u * blockIdx.x + (k)] = (k) >= 6 ? __builtin_amdgcn_s_memrealtime()  \
                                                             : __builtin_amdgcn_s_memtime();   \
    } while (0)
#else
#define NEXG_BUILD_STAMP(k) do { } while (0)
#endif

__device__ __forceinline__ void build_copy_out(const uint8_t* smem, uint8_t* T, uint32_t bytes) {
    const uint32_t tid = threadIdx.x;
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    for (uint32_t c = tid; c < bytes / 16u; c += kBuildTile)
        __builtin_nontemporal_store(reinterpret_cast<const v4u*>(smem)[c], reinterpret_cast<v4u*>(T) + c);
    const uint32_t tail = bytes & ~15u;
    if (tid < bytes - tail) T[tail + tid] = smem[tail + tid];
}

// Loads of one batch-wide value (the shared source, the small payload) by every
// lane of every workgroup: through the scalar cache (constant address space,
// s_load), not as vector loads of one line that every workgroup of the grid
// sends to that line's L2 channel. p is 4-B aligned.
typedef const __attribute__((address_space(4))) uint32_t* uniform_u32_ptr;
__device__ __forceinline__ uniform_u32_ptr uniform_u32(const void* p) {
    return reinterpret_cast<uniform_u32_ptr>(reinterpret_cast<uintptr_t>(p));
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

// A shared payload of at most kSmallPay bytes (icmp_ping's "hello"): every
// lane loads the same dwords (uniform addresses: scalar loads, no barrier)
// and sums them itself, instead of shared_payload_sum's per-workgroup global
// loads, LDS atomic and two barriers in front of every tile.
constexpr uint32_t kSmallPay = 64;
struct SmallPayload {
    uint32_t w[kSmallPay / 4];  // payload byte k = byte k & 3 of w[k >> 2] (bytes past n: 0)
    // k a compile-time index (unrolled loops): no dynamically indexed private array
    __device__ __forceinline__ uint32_t byte(uint32_t k) const { return (w[k >> 2] >> (8u * (k & 3u))) & 0xFFu; }
};

__device__ __forceinline__ void load_small_payload(const uint8_t* pl, uint32_t n, SmallPayload& sp, uint32_t& be_sum) {
    if (n == 0) {  // uniform; pl may be NULL
#pragma unroll
        for (uint32_t k = 0; k < kSmallPay / 4; k++) sp.w[k] = 0;
        be_sum = 0;
        return;
    }
    const uint64_t a = reinterpret_cast<uint64_t>(pl);
    const uint32_t sh = (uint32_t)(a & 3u);
    const uniform_u32_ptr src = uniform_u32(reinterpret_cast<const void*>(a & ~3ull));
    const uint32_t nw = (sh + n + 3u) >> 2;
    uint32_t raw[kSmallPay / 4 + 1];
#pragma unroll
    for (uint32_t k = 0; k < kSmallPay / 4 + 1; k++) raw[k] = src[k < nw ? k : nw - 1u];  // clamped: none past n
    // one empty asm over all 17: the loads issue together, one wait (per-value
    // statements let the compiler sink each load next to its own wait)
    asm volatile("" : "+s"(raw[0]), "+s"(raw[1]), "+s"(raw[2]), "+s"(raw[3]), "+s"(raw[4]), "+s"(raw[5]),
                 "+s"(raw[6]), "+s"(raw[7]), "+s"(raw[8]), "+s"(raw[9]), "+s"(raw[10]), "+s"(raw[11]),
                 "+s"(raw[12]), "+s"(raw[13]), "+s"(raw[14]), "+s"(raw[15]), "+s"(raw[16]));
    static_assert(kSmallPay / 4 + 1 == 17, "the asm above names every raw dword");
#pragma unroll
    for (uint32_t k = 0; k < kSmallPay / 4 + 1; k++) raw[k] = k < nw ? raw[k] : 0u;
#pragma unroll
    for (uint32_t k = 0; k < kSmallPay / 4; k++) {  // realigned to the payload's first byte, masked to n
        const uint32_t x = __builtin_amdgcn_alignbyte(raw[k + 1], raw[k], sh);
        sp.w[k] = 4u * k + 4u <= n ? x : 4u * k >= n ? 0u : x & ((1u << (8u * (n - 4u * k))) - 1u);
    }
    uint32_t s = 0;  // BE words from the payload's start (an even L4 offset), odd tail byte high
#pragma unroll
    for (uint32_t k = 0; k < kSmallPay / 4; k++)  // two BE halfwords per dword (bytes past n are 0)
        s += bswap16(sp.w[k] & 0xFFFFu) + bswap16(sp.w[k] >> 16);
    be_sum = s;
}

// The small payload's words into LDS (s_w, 16 dwords) for byte copies with a
// run-time count: every wave writes the same (uniform) values itself, so no
// barrier is needed before its own reads (a wave's LDS operations execute in
// order). A byte loop over the uniform words in registers was a private array
// with a dynamic index (scratch), and 64 compile-time guarded stores cost 128
// scalar instructions per wave.
__device__ __forceinline__ void stage_small_payload(const SmallPayload& sp, uint32_t* s_w) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t v = 0;
#pragma unroll
    for (uint32_t k = 0; k < kSmallPay / 4; k++) v = lane == k ? sp.w[k] : v;
    if (lane < kSmallPay / 4) s_w[lane] = v;
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
    NEXG_BUILD_STAMP(0);
    NEXG_BUILD_STAMP(6);
    const uint64_t first = tile_index(a.tile_order) * kBuildTile;
    const uint64_t left = p.count - first;
    const uint32_t nf = left < kBuildTile ? (uint32_t)left : kBuildTile;
    const uint32_t tid = threadIdx.x;
    const uint64_t i = first + tid;
    const uint32_t flen = 42u + p.payload_len;
    __shared__ uint32_t s_pay;
    // (the ICMP/TCP builder's wave-0 small-payload path measured slower here:
    // 1-5 B payloads 0.43-0.47 of 8 TB/s against 0.52-0.55 in one session,
    // profiles/r05/payload/: udp_ping's lean per-lane work does not hide it)
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
    NEXG_BUILD_STAMP(1);
    if (STAGED) {
        __syncthreads();
        NEXG_BUILD_STAMP(2);
        NEXG_BUILD_STAMP(3);
        build_copy_out(smem, a.out + first * a.out_stride, nf * a.out_stride);
    }
#if NEXG_PROBE_TIMING
    NEXG_BUILD_STAMP(4);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    NEXG_BUILD_STAMP(5);
    NEXG_BUILD_STAMP(7);
#endif
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
    NEXG_BUILD_STAMP(0);
    NEXG_BUILD_STAMP(6);
    const uint64_t first = tile_index(a.tile_order) * kBuildTile;
    const uint64_t left = p.count - first;
    const uint32_t nf = left < kBuildTile ? (uint32_t)left : kBuildTile;
    const uint32_t tid = threadIdx.x;
    const uint64_t i = first + tid;
    const uint32_t flen = 62u + p.payload_len;
    __shared__ uint32_t s_pay;
    const uint64_t pw = shared_payload_sum(p.payload, p.payload_len, &s_pay);
    if (tid < nf) {
        // addresses are 4-B aligned (the ABI checks): dword loads
        const auto* d4 = NEXG_GLOBAL(uint32_t, p.dst_ip + 16u * i);
        uint32_t sw[4], dw[4];
#pragma unroll
        for (int k = 0; k < 4; k++) dw[k] = d4[k];
        if (PROBE || p.src_shared) {  // one source for the whole batch (uniform branch)
#pragma unroll
            for (int k = 0; k < 4; k++) sw[k] = uniform_u32(p.src_ip)[k];
        } else {
            const auto* s4 = NEXG_GLOBAL(uint32_t, p.src_ip + 16u * i);
#pragma unroll
            for (int k = 0; k < 4; k++) sw[k] = s4[k];
        }
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
    NEXG_BUILD_STAMP(1);
    if (STAGED) {
        __syncthreads();
        NEXG_BUILD_STAMP(2);
        NEXG_BUILD_STAMP(3);
        build_copy_out(smem, a.out + first * a.out_stride, nf * a.out_stride);
    }
#if NEXG_PROBE_TIMING
    NEXG_BUILD_STAMP(4);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    NEXG_BUILD_STAMP(5);
    NEXG_BUILD_STAMP(7);
#endif
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
    NEXG_BUILD_STAMP(0);
    NEXG_BUILD_STAMP(6);
    const uint64_t first = tile_index(a.tile_order) * kBuildTile;
    const uint64_t left = a.count - first;
    const uint32_t nf = left < kBuildTile ? (uint32_t)left : kBuildTile;
    const uint64_t i = first + tid;
    const bool small = a.payload_len <= kSmallPay;  // uniform
    SmallPayload spay{};
    uint32_t pay_sum = 0;
    __shared__ uint32_t s_payw[kSmallPay / 4 + 1];  // the staged words, then their sum
    if (small && STAGED) {
        // staged tile: wave 0 realigns and sums the payload once for the
        // workgroup (the other waves skip ~100 VALU instructions each): icmp_ping's
        // 47-B batch 0.525 -> 0.70 of 8 TB/s written (profiles/r05/payload/)
        if (a.payload_len) {  // uniform
            if (tid < 64u) {
                load_small_payload(a.payload, a.payload_len, spay, pay_sum);
                stage_small_payload(spay, s_payw);
                if (tid == 0) s_payw[kSmallPay / 4] = pay_sum;
            }
            __syncthreads();
            pay_sum = s_payw[kSmallPay / 4];
        }
    } else if (small) {
        load_small_payload(a.payload, a.payload_len, spay, pay_sum);
        if (STAGED && a.payload_len) stage_small_payload(spay, s_payw);
    } else {
        pay_sum = shared_payload_sum(a.payload, a.payload_len, &s_pay);
    }
    const uint32_t l4_hdr = KIND == kL4Tcp ? 20u + a.opt_padded : 8u;
    const uint32_t l4_len = l4_hdr + a.payload_len;
    const uint32_t flen = 14u + 2u * NIP + l4_len;
    if (tid < nf) {
        const nexg_ip_build& ip = a.ip;
        constexpr uint32_t AW = FAM == 4 ? 1u : 4u;  // address dwords
        uint32_t sw[AW], dw[AW];
#pragma unroll
        for (uint32_t k = 0; k < AW; k++) dw[k] = NEXG_GLOBAL(uint32_t, ip.dst_ip)[AW * i + k];
        if (PROBE || ip.src_shared) {  // one source for the whole batch (uniform branch)
#pragma unroll
            for (uint32_t k = 0; k < AW; k++) sw[k] = uniform_u32(ip.src_ip)[k];
        } else {
#pragma unroll
            for (uint32_t k = 0; k < AW; k++) sw[k] = NEXG_GLOBAL(uint32_t, ip.src_ip)[AW * i + k];
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
        if constexpr (KIND == kL4Tcp) {
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
        if (small && STAGED) {
            const uint8_t* pb = reinterpret_cast<const uint8_t*>(s_payw);
            for (uint32_t k = 0; k < a.payload_len; k++) base[p + k] = pb[k];
        } else if (small) {
#pragma unroll
            for (uint32_t k = 0; k < kSmallPay; k++)
                if (k < a.payload_len) base[p + k] = (uint8_t)spay.byte(k);
        } else {
            for (uint32_t k = 0; k < a.payload_len; k++) base[p + k] = a.payload[k];
        }
        if (STAGED)
            for (uint32_t k = flen; k < a.out_stride; k++) base[d0 + k] = 0;
    }
    NEXG_BUILD_STAMP(1);
    if (STAGED) {
        __syncthreads();
        NEXG_BUILD_STAMP(2);
        NEXG_BUILD_STAMP(3);
        build_copy_out(smem, a.out + first * a.out_stride, nf * a.out_stride);
    }
#if NEXG_PROBE_TIMING
    NEXG_BUILD_STAMP(4);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    NEXG_BUILD_STAMP(5);
    NEXG_BUILD_STAMP(7);
#endif
}

template <int FAM, int KIND, bool PROBE>
static void launch_l4_form(const L4Args& a, hipStream_t s) {
    const uint64_t blocks = (a.count + kBuildTile - 1) / kBuildTile;
    const bool staged = a.out_stride <= kBuildMaxStride && (reinterpret_cast<uint64_t>(a.out) & 15u) == 0;
    // IPv6: 16-KiB tile + build_lds_pad() -> 5 workgroups per CU (icmp6 echo
    // 0.29 -> 0.26 ms at 16M frames); IPv4 shapes run faster at 8 per CU (tcp
    // SYN 0.21 vs 0.24-0.26 ms, icmp echo 0.132 vs 0.140; profiles/r04/builders/)
    // ICMP probe batches (odd frame lengths, 47 / 67 B) run faster at 8 per CU:
    // 0.437 / 0.570 of 8 TB/s written against 0.385 / 0.485 (profiles/r05/probe/)
    const uint32_t pad = (FAM == 6 || PROBE) && !(PROBE && KIND == kL4Icmp) ? build_lds_pad() : 0u;
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

static bool try_probe_l4(const L4Args& l, int kind, uint8_t* out, uint32_t out_stride, hipStream_t s, hipError_t& e);

template <int FAM, int KIND>
static hipError_t launch_l4_fam(L4Args& a, hipStream_t s) {
    // the probe batch: one source, a destination per frame, nothing else per
    // frame. It reads 4 / 16 B per frame, as udp_ping's probe batch, and takes
    // that builder's tile order (contiguous eighths); the forms with several
    // parameter arrays keep l4_build_tile_order()
    const bool probe = a.ip.src_shared && !a.ip.ip_id && !a.ip.src_mac && !a.ip.dst_mac &&
                       (KIND == kL4Tcp ? !a.sport && !a.dport && !a.seq && !a.ack : !a.ident && !a.seqno);
    // the template kernel's status (its explicit checks and its launch's
    // hipGetLastError, which also clears HIP's error state) is the result
    hipError_t e = hipSuccess;
    if (probe && try_probe_l4(a, KIND, a.out, a.out_stride, s, e)) return e;
    if (probe) {
        a.tile_order = build_tile_order();
        launch_l4_form<FAM, KIND, true>(a, s);
    } else {
        launch_l4_form<FAM, KIND, false>(a, s);
    }
    return hipGetLastError();
}

static hipError_t launch_l4(L4Args& a, int kind, hipStream_t s) {
    if (a.count == 0) return hipSuccess;
    if ((a.count + kBuildTile - 1) / kBuildTile > 0xFFFFFFFFull) return hipErrorInvalidValue;  // one grid
    a.tile_order = l4_build_tile_order();
    if (kind == kL4Tcp) return a.ip.family == 4 ? launch_l4_fam<4, kL4Tcp>(a, s) : launch_l4_fam<6, kL4Tcp>(a, s);
    return a.ip.family == 4 ? launch_l4_fam<4, kL4Icmp>(a, s) : launch_l4_fam<6, kL4Icmp>(a, s);
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


// ---- probe batches: one template + a per-frame patch ----------------------
// Every frame of a probe batch (one source, a destination per frame, every
// other field the batch's) is one template with the destination address and
// the checksums over it patched. The host builds the template (one frame
// period P = out_stride, with destination, checksums and the device-resident
// source / payload bytes 0) and its base sums and passes it in the kernel
// arguments; a workgroup reads it by scalar loads, merges in the source and
// payload (scalar loads: every workgroup reads the same line, which as vector
// loads makes one L2 channel the bottleneck), lays the period out in LDS and
// fills its tile with it (one ds_write_b128 per 16-B chunk, realigned by
// v_alignbyte), patches each frame (the other builders' closed-form sums: the
// batch base sum plus the destination's halfwords), and copies the tile out
// with 16-B non-temporal stores.
// Used for tcp_ping (IPv4 / IPv6) and udp_ping's IPv6 batch, where it beats
// the per-lane builders (tcp_ping 0.72-0.89 of 8 TB/s written against
// 0.70-0.73); udp_ping's IPv4 batch and the ICMP shapes stay per lane
// (profiles/r05/probe/). A persistent sweep over the tiles and one-wave
// workgroups were measured and lose (writes at 0.65-0.72 of 8 TB/s in a
// sweep, tools/writebench.hip).
#ifndef NEXG_PROBE_TEMPLATE
#define NEXG_PROBE_TEMPLATE 1  // 0: the per-lane builders for probe batches too (A/B builds)
#endif
constexpr uint32_t kProbeMaxP = 128;

struct ProbeArgs {
    uint32_t tmpl[kProbeMaxP / 4];  // one period (the frame with destination, checksums and device bytes 0, zero pad)
    uint64_t ip_sum;           // IPv4 header: congruent sum of every word but the destination's (and a device source's)
    uint64_t l4_sum;           // L4: the same, without the payload
    const uint8_t* dst;        // per-frame destination: DW dwords each, 4-B aligned
    const uint8_t* src;        // the batch's source on the device (DW dwords), written in at src_off; or NULL
    const uint8_t* payload;    // device payload (<= kSmallPay bytes), written in at pay_off
    uint8_t* out;
    uint64_t count;
    uint32_t period;           // out_stride (<= kProbeMaxP)
    uint32_t dst_off, ip_ck_off, l4_ck_off;  // byte offsets in the frame; a checksum offset 0 = none
    uint32_t l4_dst;           // the L4 checksum covers the addresses (all but ICMPv4)
    uint32_t dst_value;        // udp_ping IPv4: dst is a u32 value (bytes reversed in the frame, BE halves summed)
    uint32_t src_off, ip_src;  // device source offset; the source is in the IPv4 header checksum
    uint32_t pay_off, pay_len;
    uint32_t tile_order;
};

// halfword v (big-endian: high byte first in memory) at LDS byte position p
__device__ __forceinline__ void lds_put_be16(uint8_t* lds, uint32_t p, uint32_t v) {
    if (p & 1u) {
        lds[p] = (uint8_t)(v >> 8);
        lds[p + 1] = (uint8_t)v;
    } else {
        *reinterpret_cast<uint16_t*>(lds + p) = (uint16_t)bswap16(v);
    }
}
// dword d of network-order bytes (as loaded little-endian) at LDS position p
__device__ __forceinline__ void lds_put_net32(uint8_t* lds, uint32_t p, uint32_t d) {
    lds_put_be16(lds, p, bswap16(d & 0xFFFFu));
    lds_put_be16(lds, p + 2u, bswap16(d >> 16));
}

// A workgroup of WAVES waves builds a tile of kT = 64 WAVES frames (one per
// lane). KCH = ceil(P / 16): the 16-B pattern chunks per lane (kT frames x P
// bytes = kT P / 16 chunks), written unconditionally. With one wave per
// workgroup the barriers below are wave barriers (no s_barrier).
template <uint32_t DW, uint32_t KCH, uint32_t WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_build_probe(ProbeArgs a) {
    constexpr uint32_t kT = 64u * WAVES;
    extern __shared__ __attribute__((aligned(16))) uint8_t s_tile[];  // kT x P, then the pattern
    const uint32_t t = threadIdx.x, P = a.period;
    // (1) once per workgroup, the period in LDS: wave 0 composes template
    // bytes [0, P + 24) (the period and the start of its next copy, so a 20-B
    // window at any offset < P is contiguous): the template dwords come from
    // the kernel arguments by scalar loads and reach their lanes by a cndmask
    // chain and ds_bpermute; the device payload and source bytes are loaded
    // into place, so they are part of the pattern and not patched per frame
    uint8_t* const tp = s_tile + KCH * 16u * kT;  // 2 x kProbeMaxP + 32 B
    // this lane's destination goes in flight (clamped index: an unconditional
    // load; lanes past the batch's end reload its last frame)
    NEXG_BUILD_STAMP(0);
    NEXG_BUILD_STAMP(6);
    const uint64_t tile = tile_index(a.tile_order);
    uint32_t dw[DW];
    {
        const uint64_t i = tile * kT + t;
        const auto* d4 = NEXG_GLOBAL(uint32_t, a.dst + 4u * DW * (i < a.count ? i : a.count - 1u));
#pragma unroll
        for (uint32_t k = 0; k < DW; k++) dw[k] = d4[k];
    }
    // the batch's device source by scalar loads (uniform addresses through the
    // scalar cache: a vector load of one line by every workgroup of the grid
    // makes that line's L2 channel the bottleneck) and its BE word sum
    uint32_t sx[DW], ssum = 0;
#pragma unroll
    for (uint32_t k = 0; k < DW; k++) sx[k] = 0;
    if (a.src) {  // 4-B aligned
#pragma unroll
        for (uint32_t k = 0; k < DW; k++) sx[k] = uniform_u32(a.src)[k];
#pragma unroll
        for (uint32_t k = 0; k < DW; k++) ssum += bswap16(sx[k] & 0xFFFFu) + bswap16(sx[k] >> 16);
    }
    uint32_t* const psum_lds = reinterpret_cast<uint32_t*>(tp) + (kProbeMaxP + 32u) / 4u;  // past the pattern
    if (t < 64u) {
        // the payload (scalar loads) realigned and summed by wave 0 only; its
        // sum reaches the other waves through LDS
        SmallPayload spay;
        uint32_t psum0;
        load_small_payload(a.payload, a.pay_len, spay, psum0);  // realigned words, 0 past pay_len
        if (t == 0) *psum_lds = psum0;
        // template, source and payload words handed to lane k by cndmask
        // chains, then each pattern byte picked by ds_bpermute from the lane
        // holding it (one per source: the source lane returns its own copy of
        // the operand, so the operand cannot depend on the reading lane)
        uint32_t v = 0, sv = 0, pv = 0;
#pragma unroll
        for (uint32_t k = 0; k < kProbeMaxP / 4; k++) v = t == k ? a.tmpl[k] : v;
#pragma unroll
        for (uint32_t k = 0; k < DW; k++) sv = t == k ? sx[k] : sv;
#pragma unroll
        for (uint32_t k = 0; k < kSmallPay / 4; k++) pv = t == k ? spay.w[k] : pv;
        uint32_t d = 0;
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) {
            const uint32_t j = 4u * t + i, jm = j >= P ? j - P : j;
            const uint32_t pi = jm - a.pay_off, si = jm - a.src_off;  // wrap: huge when before
            const bool in_p = pi < a.pay_len, in_s = a.src && si < 4u * DW;
            const uint32_t xt = (uint32_t)__shfl(v, (int)(jm >> 2));
            const uint32_t xs = (uint32_t)__shfl(sv, (int)((si >> 2) & 63u));
            const uint32_t xp = (uint32_t)__shfl(pv, (int)((pi >> 2) & 63u));
            const uint32_t x = in_p ? xp >> (8u * (pi & 3u)) : in_s ? xs >> (8u * (si & 3u)) : xt >> (8u * (jm & 3u));
            d |= (x & 0xFFu) << (8u * i);
        }
        if (4u * t < P + 24u) reinterpret_cast<uint32_t*>(tp)[t] = d;
    }
    __syncthreads();
    const uint32_t psum = *psum_lds;
    const uint32_t step = (16u * kT) % P, r0 = (16u * t) % P;
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    // the pattern over the tile: chunk c = bytes [(16 c) mod P, + 16) of the
    // period, five dword reads realigned by v_alignbyte
    auto fill = [&]() {
        uint32_t r = r0;
#pragma unroll
        for (uint32_t k = 0; k < KCH; k++) {
            const uint32_t* w = reinterpret_cast<const uint32_t*>(tp + (r & ~3u));
            const uint32_t sh = r & 3u;
            const uint4 c = make_uint4(__builtin_amdgcn_alignbyte(w[1], w[0], sh),
                                       __builtin_amdgcn_alignbyte(w[2], w[1], sh),
                                       __builtin_amdgcn_alignbyte(w[3], w[2], sh),
                                       __builtin_amdgcn_alignbyte(w[4], w[3], sh));
            reinterpret_cast<uint4*>(s_tile)[t + kT * k] = c;
            r += step;
            r = r >= P ? r - P : r;
        }
    };
    // this lane's frame: the destination and the checksums over it
    auto patch = [&](const uint32_t (&cur)[DW]) {
        uint8_t* f = s_tile + t * P;
        uint32_t dsum = 0;
#pragma unroll
        for (uint32_t k = 0; k < DW; k++) dsum += halves(cur[k]);
        uint64_t D;
        if (a.dst_value) {  // a u32 value: network order in the frame, its BE halves summed
            lds_put_be16(f, a.dst_off, cur[0] >> 16);
            lds_put_be16(f, a.dst_off + 2u, cur[0] & 0xFFFFu);
            D = dsum;
        } else {  // network-order bytes as stored: LE halves x 256
#pragma unroll
            for (uint32_t k = 0; k < DW; k++) lds_put_net32(f, a.dst_off + 4u * k, cur[k]);
            D = 256ull * dsum;
        }
        const uint64_t S = ssum;
        if (a.ip_ck_off) lds_put_be16(f, a.ip_ck_off, fold_complement(a.ip_sum + (a.ip_src ? S : 0u) + D));
        if (a.l4_ck_off) lds_put_be16(f, a.l4_ck_off, fold_complement(a.l4_sum + psum + (a.l4_dst ? S + D : 0u)));
    };
    // (2) fill, patch, copy out: one tile per workgroup (a persistent sweep
    // over the tiles writes at 0.65-0.72 of 8 TB/s against 0.77-0.83 for one
    // tile per workgroup, tools/writebench.hip, profiles/r05/writebench/)
    const uint64_t first = (uint64_t)tile * kT;
    const uint32_t nf = a.count - first < kT ? (uint32_t)(a.count - first) : kT;
    NEXG_BUILD_STAMP(1);
    fill();
    __syncthreads();
    NEXG_BUILD_STAMP(2);
    if (t < nf) patch(dw);
    __syncthreads();
    NEXG_BUILD_STAMP(3);
    const uint32_t bytes = nf * P;
    uint8_t* T = a.out + first * P;
    for (uint32_t c = t; c < bytes / 16u; c += kT)
        __builtin_nontemporal_store(reinterpret_cast<const v4u*>(s_tile)[c], reinterpret_cast<v4u*>(T) + c);
    const uint32_t tail = bytes & ~15u;
    if (t < bytes - tail) T[tail + t] = s_tile[tail + t];
#if NEXG_PROBE_TIMING
    NEXG_BUILD_STAMP(4);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // the stores' completion
    NEXG_BUILD_STAMP(5);
    NEXG_BUILD_STAMP(7);
#endif
}

// ---- probe batches, frame per lane: k_build_lane ---------------------------
// The probe template as k_build_probe takes it, but each lane writes its own
// frame into the LDS tile as whole dwords of the tile, so that odd frame
// periods (icmp_ping's 47 B) cost no byte or halfword stores and there is no
// separate fill pass or patch barrier:
//  * the template dwords (the host's, followed by the next frame's first 8
//    bytes) are uniform: the device source and payload are merged into them
//    by scalar loads at compile-time offsets in every wave (no barrier);
//  * lane t's frame starts at tile byte t P, s = t P mod 4 bytes into its
//    first dword. Frame dword F[j] (frame bytes [4j, 4j + 4)) gets the lane's
//    destination and the checksums over it OR-ed in at the shape's
//    compile-time offsets; tile dword (t P >> 2) + j is
//    v_alignbyte(F[j], F[j - 1], 4 - s) (F[j] when s = 0);
//  * a lane writes the dwords from the first one that starts inside its frame
//    to the one holding its last byte; that last dword's other bytes are the
//    next frame's head (the Ethernet addresses: batch constants), so every
//    tile dword has exactly one writer and no lane needs a neighbour's bytes.
// Then one barrier and the tile leaves with 16-B non-temporal stores.
// MINP <= P <= MAXP: the frame dwords every lane writes are known at compile
// time (no exec mask per dword); the last one or two are per lane.
template <int FAM, int KIND, uint32_t MAXP, uint32_t MINP = 0>
__global__ __launch_bounds__(256) void k_build_lane(ProbeArgs a) {
    constexpr uint32_t DW = FAM == 4 ? 1u : 4u;              // destination dwords
    constexpr uint32_t SRC = FAM == 4 ? 26u : 22u;           // source address offset (= 2 mod 4)
    constexpr uint32_t DST = FAM == 4 ? 30u : 38u;           // destination offset (= 2 mod 4)
    constexpr uint32_t L3 = FAM == 4 ? 20u : 40u;
    constexpr uint32_t L4CK = 14u + L3 + (KIND == kL4Tcp ? 16u : 2u);  // L4 checksum offset
    constexpr uint32_t PAY = 14u + L3 + 8u;                  // ICMP payload offset (= 2 mod 4)
    constexpr bool L4DST = !(FAM == 4 && KIND == kL4Icmp);   // ICMPv4 sums the message alone
    constexpr uint32_t NF = MAXP / 4u + 3u;                  // frame dwords + the next frame's head
    static_assert(SRC % 4u == 2u && DST % 4u == 2u && PAY % 4u == 2u, "halfword-shifted fields");
    static_assert(KIND != kL4Icmp || MAXP >= PAY, "the period holds the ICMP header");
    extern __shared__ __attribute__((aligned(16))) uint8_t s_tile[];  // 256 x P + 16
    const uint32_t t = threadIdx.x, P = a.period;
    NEXG_BUILD_STAMP(0);
    NEXG_BUILD_STAMP(6);
    const uint64_t tile = tile_index(a.tile_order);
    const uint64_t first = tile * kBuildTile;
    const uint32_t nf = a.count - first < kBuildTile ? (uint32_t)(a.count - first) : kBuildTile;
    uint32_t dw[DW];
    {  // this lane's destination in flight first (clamped: lanes past the end reload the last)
        const uint64_t i = first + t;
        const auto* d4 = NEXG_GLOBAL(uint32_t, a.dst + 4u * DW * (i < a.count ? i : a.count - 1u));
#pragma unroll
        for (uint32_t k = 0; k < DW; k++) dw[k] = d4[k];
    }
    // uniform: the template with the batch's device source and payload merged
    uint32_t F[NF];
#pragma unroll
    for (uint32_t k = 0; k < NF; k++) F[k] = a.tmpl[k];
    uint32_t ssum = 0;
    {
        uint32_t sx[DW];
#pragma unroll
        for (uint32_t k = 0; k < DW; k++) sx[k] = uniform_u32(a.src)[k];
#pragma unroll
        for (uint32_t k = 0; k < DW; k++) {
            ssum += bswap16(sx[k] & 0xFFFFu) + bswap16(sx[k] >> 16);
            F[SRC / 4u + k] |= sx[k] << 16;
            F[SRC / 4u + k + 1u] |= sx[k] >> 16;
        }
    }
    uint64_t psum = 0;
    if (KIND == kL4Icmp && a.pay_len) {  // uniform: scalar loads and SALU only
        // (load_small_payload's v_alignbyte / v_perm forms put ~250 VALU
        // instructions in every wave; 64-bit scalar shifts, and the payload's
        // word sum as 256 x its LE halves, congruent mod 0xFFFF, stay scalar)
        constexpr uint32_t NP = (MAXP - PAY + 3u) / 4u;  // payload dwords a period can hold
        const uint64_t pa = reinterpret_cast<uint64_t>(a.payload);
        const uint32_t n = a.pay_len, sh = 8u * (uint32_t)(pa & 3u), nw = ((uint32_t)(pa & 3u) + n + 3u) >> 2;
        const uniform_u32_ptr src = uniform_u32(reinterpret_cast<const void*>(pa & ~3ull));
        uint32_t raw[NP + 1];
#pragma unroll
        for (uint32_t k = 0; k < NP + 1u; k++) raw[k] = k < nw ? src[k] : 0u;  // none past the payload
        uint32_t le = 0;
#pragma unroll
        for (uint32_t k = 0; k < NP; k++) {
            const uint32_t x = (uint32_t)((((uint64_t)raw[k + 1] << 32) | raw[k]) >> sh);
            const uint32_t w = 4u * k + 4u <= n ? x : 4u * k >= n ? 0u : x & ((1u << (8u * (n - 4u * k))) - 1u);
            le += (w & 0xFFFFu) + (w >> 16);
            if (PAY / 4u + k < NF) F[PAY / 4u + k] |= w << 16;
            if (PAY / 4u + k + 1u < NF) F[PAY / 4u + k + 1u] |= w >> 16;
        }
        psum = 256ull * le;  // the payload starts at an even offset: BE word sum (mod 0xFFFF)
    }
    const uint64_t S = ssum;
    if (!L4DST) {  // ICMPv4: one checksum for the batch
        const uint32_t ck = fold_complement(a.l4_sum + psum);
        F[L4CK / 4u] |= bswap16(ck) << (8u * (L4CK % 4u));
    }
    if (t < nf) {
        // the lane's frame: destination (network-order bytes, LE halves x 256) and checksums
        uint32_t dsum = 0;
#pragma unroll
        for (uint32_t k = 0; k < DW; k++) {
            dsum += halves(dw[k]);
            F[DST / 4u + k] |= dw[k] << 16;
            F[DST / 4u + k + 1u] |= dw[k] >> 16;
        }
        const uint64_t D = 256ull * dsum;
        if (FAM == 4) F[6] |= bswap16(fold_complement(a.ip_sum + S + D));  // bytes 24-25
        if (L4DST) F[L4CK / 4u] |= bswap16(fold_complement(a.l4_sum + psum + S + D)) << (8u * (L4CK % 4u));
        // frame start s' = 1..4 bytes into tile dword qb = (t P - s') / 4 (s' = 4
        // when t P is dword-aligned), so tile dword qb + j = frame bytes
        // [4j - s', 4j - s' + 4) = v_alignbyte(F[j], F[j - 1], (4 - s') mod 4) for
        // every lane alike; j = 0 is the previous frame's (its writer's), j runs
        // to the dword holding byte P - 1: j <= (P - 1 + s') / 4, which is
        // lane-dependent only for the last one or two j
        const uint32_t b0 = t * P, s1 = ((b0 + 3u) & 3u) + 1u, sh = (4u - s1) & 3u;
        const uint32_t jend = (P - 1u + s1) >> 2, jlo = P >> 2, jhi = (P + 3u) >> 2;
        uint32_t* const tw = reinterpret_cast<uint32_t*>(s_tile) + ((b0 + 4u - s1) >> 2) - 1u;
        // fully unrolled (a `break` here rolls the loop back up with dynamic
        // register indexing of F): j <= MINP / 4 unconditionally, then uniform
        // and per-lane guards
#pragma unroll
        for (uint32_t j = 1; j < NF; j++) {
            const uint32_t v = __builtin_amdgcn_alignbyte(F[j], F[j - 1u], sh);
            if (j <= MINP / 4u) tw[j] = v;
            else if (j <= jlo) tw[j] = v;
            else if (j <= jhi && j <= jend) tw[j] = v;
        }
    }
    NEXG_BUILD_STAMP(1);
    __syncthreads();
    NEXG_BUILD_STAMP(2);
    NEXG_BUILD_STAMP(3);
    build_copy_out(s_tile, a.out + first * P, nf * P);
#if NEXG_PROBE_TIMING
    NEXG_BUILD_STAMP(4);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    NEXG_BUILD_STAMP(5);
    NEXG_BUILD_STAMP(7);
#endif
}

// ---- host: probe templates (the bytes the per-lane builders write, with the
// destination, checksums and payload zero) and their base sums
namespace {
void put_be16(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}
uint64_t be_halves(const uint8_t* p, uint32_t n) {  // BE words of n (even) bytes
    uint64_t s = 0;
    for (uint32_t k = 0; k < n; k += 2) s += ((uint32_t)p[k] << 8) | p[k + 1];
    return s;
}
void probe_eth(uint8_t* t, const uint8_t* dmac, const uint8_t* smac, uint32_t ethertype) {
    for (int k = 0; k < 6; k++) {
        t[k] = dmac[k];
        t[6 + k] = smac[k];
    }
    put_be16(t + 12, ethertype);
}
// IPv4 header (builder/ipv4.rs:94-170) with destination and checksum zero;
// returns the BE word sum of the rest (the header checksum's base)
uint64_t probe_ipv4(uint8_t* h, uint32_t tos, uint32_t total, uint32_t id, uint32_t flags, uint32_t ttl,
                    uint32_t proto, const uint8_t* src) {
    h[0] = 0x45; h[1] = (uint8_t)tos;
    put_be16(h + 2, total);
    put_be16(h + 4, id);
    put_be16(h + 6, (flags & 7u) << 13);
    h[8] = (uint8_t)ttl; h[9] = (uint8_t)proto;
    put_be16(h + 10, 0);
    for (int k = 0; k < 4; k++) { h[12 + k] = src[k]; h[16 + k] = 0; }
    return be_halves(h, 20);
}
// IPv6 header (builder/ipv6.rs:89-152) with the destination zero
void probe_ipv6(uint8_t* h, uint32_t tc, uint32_t flow, uint32_t plen, uint32_t next, uint32_t hop, const uint8_t* src) {
    const uint32_t fl = flow & 0xFFFFFu;
    h[0] = (uint8_t)(0x60u | (tc >> 4)); h[1] = (uint8_t)(((tc & 0xFu) << 4) | (fl >> 16));
    h[2] = (uint8_t)(fl >> 8); h[3] = (uint8_t)fl;
    put_be16(h + 4, plen);
    h[6] = (uint8_t)next; h[7] = (uint8_t)hop;
    for (int k = 0; k < 16; k++) { h[8 + k] = src[k]; h[24 + k] = 0; }
}

bool probe_launch_ok(uint32_t flen, uint32_t period, uint32_t pay_len, const uint8_t* out) {
    return NEXG_PROBE_TEMPLATE && period <= kProbeMaxP && flen <= period && pay_len <= kSmallPay &&
           (reinterpret_cast<uint64_t>(out) & 15u) == 0;
}

// Probe kernel shape (measurement overrides, read once): NEXG_PROBE_WAVES
// waves per workgroup (1 or 4), NEXG_PROBE_WGS workgroups per CU set by the
// dynamic LDS (160 KiB per CU; 0 = only the tile's LDS).
uint32_t probe_env(const char* name, uint32_t def, uint32_t lo, uint32_t hi) {
#ifdef NEXG_AB_KNOBS
    const char* e = getenv(name);
#else
    (void)name;
    const char* e = nullptr;  // product build: no environment overrides
#endif
    const long x = e ? strtol(e, nullptr, 10) : -1;
    return x >= (long)lo && x <= (long)hi ? (uint32_t)x : def;
}
uint32_t probe_waves() {
    static const uint32_t v = probe_env("NEXG_PROBE_WAVES", 4u, 1u, 4u) == 1u ? 1u : 4u;
    return v;
}
uint32_t probe_wgs_per_cu() {
    // 1 or 2 per CU would ask more than a workgroup's 64 KiB of LDS: 3 at least
    static const uint32_t v = [] { const uint32_t w = probe_env("NEXG_PROBE_WGS", 5u, 0u, 64u);
                                   return w && w < 3u ? 3u : w; }();
    return v;
}

// tmpl: one period (P bytes, zero past the frame), one tile per workgroup
hipError_t launch_probe(ProbeArgs& a, const uint8_t* tmpl, uint32_t dw, hipStream_t s) {
    if (a.count == 0) return hipSuccess;
    const uint32_t P = a.period;
    for (uint32_t k = 0; k < kProbeMaxP / 4; k++)
        a.tmpl[k] = (uint32_t)tmpl[4 * k] | ((uint32_t)tmpl[4 * k + 1] << 8) | ((uint32_t)tmpl[4 * k + 2] << 16) |
                    ((uint32_t)tmpl[4 * k + 3] << 24);
    const uint32_t waves = probe_waves(), kT = 64u * waves;
    const uint64_t ntiles = (a.count + kT - 1) / kT;
    if (ntiles > 0xFFFFFFFFull) return hipErrorInvalidValue;
#ifdef NEXG_AB_KNOBS
    // fault injection for the error-path test (tests/test_gpu_probe_batches.py)
    if (probe_env("NEXG_PROBE_FAIL", 0u, 0u, 1u) == 1u) return hipErrorInvalidValue;
#endif
    const uint32_t need = (P + 15u) / 16u;  // 16-B chunks per lane, rounded to an instantiated KCH
    const uint32_t kch = need <= 3u ? 3u : need <= 6u ? need : 8u;
    const uint32_t tile_lds = kch * 16u * kT + 2u * kProbeMaxP + 32u, wgs = probe_wgs_per_cu();
    const uint32_t cap = wgs ? 160u * 1024u / wgs - 1024u : 0u;
    const uint32_t lds = tile_lds > cap ? tile_lds : cap < 65536u ? cap : 65536u;  // a workgroup's LDS limit
    a.tile_order = probe_tile_order();
    const dim3 g((uint32_t)ntiles), b(kT);
#define NEXG_PROBE_LAUNCH(DW, K)                                                     \
    do {                                                                             \
        if (waves == 1u) hipLaunchKernelGGL((k_build_probe<DW, K, 1>), g, b, lds, s, a); \
        else hipLaunchKernelGGL((k_build_probe<DW, K, 4>), g, b, lds, s, a);             \
    } while (0)
    if (dw == 1) {
        if (kch == 3) NEXG_PROBE_LAUNCH(1, 3); else if (kch == 4) NEXG_PROBE_LAUNCH(1, 4);
        else if (kch == 5) NEXG_PROBE_LAUNCH(1, 5); else if (kch == 6) NEXG_PROBE_LAUNCH(1, 6);
        else NEXG_PROBE_LAUNCH(1, 8);
    } else {
        if (kch == 3) NEXG_PROBE_LAUNCH(4, 3); else if (kch == 4) NEXG_PROBE_LAUNCH(4, 4);
        else if (kch == 5) NEXG_PROBE_LAUNCH(4, 5); else if (kch == 6) NEXG_PROBE_LAUNCH(4, 6);
        else NEXG_PROBE_LAUNCH(4, 8);
    }
#undef NEXG_PROBE_LAUNCH
    return hipGetLastError();
}

// Workgroups per CU of k_build_lane, set by its dynamic LDS (NEXG_LANE_WGS
// overrides in the knobs build; 0 = the tile's LDS only): icmp_ping's 47-B
// batch, 16M frames, in one process (profiles/r06/lane/lane_ab2.log): 0.693
// of 8 TB/s written at 3 per CU, 0.663-0.667 at 4, 0.662 at 5, 0.654-0.661
// at 6, against 0.58 for k_build_l4
uint32_t lane_wgs_per_cu() {
    static const uint32_t v = probe_env("NEXG_LANE_WGS", 3u, 0u, 64u);
    return v;
}

// k_build_lane: tmpl = one period P <= kLaneMaxP; the kernel's template is the
// period followed by its first 8 bytes (the next frame's head)
constexpr uint32_t kLaneMaxP = 96;
bool lane_launch_ok(uint32_t flen, uint32_t period, uint32_t pay_len, const uint8_t* out) {
    return period <= kLaneMaxP && flen <= period && pay_len <= kSmallPay && (reinterpret_cast<uint64_t>(out) & 15u) == 0;
}

hipError_t launch_lane(ProbeArgs& a, const uint8_t* tmpl, int fam, int kind, hipStream_t s) {
    if (a.count == 0) return hipSuccess;
    const uint32_t P = a.period;
    uint8_t d[kProbeMaxP] = {0};
    for (uint32_t k = 0; k < P; k++) d[k] = tmpl[k];
    for (uint32_t k = 0; k < 8u; k++) d[P + k] = tmpl[k];
    for (uint32_t k = 0; k < kProbeMaxP / 4; k++)
        a.tmpl[k] = (uint32_t)d[4 * k] | ((uint32_t)d[4 * k + 1] << 8) | ((uint32_t)d[4 * k + 2] << 16) |
                    ((uint32_t)d[4 * k + 3] << 24);
    const uint64_t ntiles = (a.count + kBuildTile - 1) / kBuildTile;
    if (ntiles > 0xFFFFFFFFull) return hipErrorInvalidValue;
#ifdef NEXG_AB_KNOBS
    if (probe_env("NEXG_PROBE_FAIL", 0u, 0u, 1u) == 1u) return hipErrorInvalidValue;
#endif
    // dynamic LDS: the tile (+ the last lane's tail dword), raised to set the
    // workgroups per CU (probe_wgs_per_cu, as k_build_probe)
    const uint32_t tile_lds = kBuildTile * P + 16u, wgs = lane_wgs_per_cu();
    const uint32_t cap = wgs ? 160u * 1024u / wgs - 1024u : 0u;
    const uint32_t lds = tile_lds > cap ? tile_lds : cap < 65536u ? cap : 65536u;  // (1 per CU: 64 KiB)
    a.tile_order = build_tile_order();
    const dim3 g((uint32_t)ntiles), b(kBuildTile);
    // the unrolled frame-dword count follows the period: instances for
    // 44-48 B (icmp_ping, 47 B), 64-68 B (its IPv6 form, 67 B; tcp_ping, 66 B)
    // and any period up to 96 B
    const bool p48 = P >= 44u && P <= 48u, p68 = P >= 64u && P <= 68u;
#define NEXG_LANE(F, K)                                                                           \
    do {                                                                                          \
        if (p68) hipLaunchKernelGGL((k_build_lane<F, K, 68, 64>), g, b, lds, s, a);               \
        else hipLaunchKernelGGL((k_build_lane<F, K, kLaneMaxP>), g, b, lds, s, a);                \
    } while (0)
    if (kind == kL4Icmp && fam == 4 && p48) hipLaunchKernelGGL((k_build_lane<4, kL4Icmp, 48, 44>), g, b, lds, s, a);
    else if (kind == kL4Icmp && fam == 4) NEXG_LANE(4, kL4Icmp);
    else if (kind == kL4Icmp) NEXG_LANE(6, kL4Icmp);
    else if (fam == 4) NEXG_LANE(4, kL4Tcp);
    else NEXG_LANE(6, kL4Tcp);
#undef NEXG_LANE
    return hipGetLastError();
}
}  // namespace

// udp_ping's IPv6 probe batch (src_shared, dst per frame): builder/udp.rs:67-95
// over IPv6 (udp.rs:480-505) as k_build_udp6 sums it
static bool try_probe_udp6(const nexg_udp6_build& p, uint8_t* out, uint32_t out_stride, hipStream_t s, hipError_t& e) {
    const uint32_t flen = 62u + p.payload_len;
    if (!probe_launch_ok(flen, out_stride, p.payload_len, out)) return false;
    ProbeArgs a{};
    uint8_t t[kProbeMaxP] = {0};
    const uint8_t zero[16] = {0};
    const uint32_t ulen = 8u + p.payload_len;
    probe_eth(t, p.def_dst_mac, p.def_src_mac, 0x86DD);
    probe_ipv6(t + 14, p.traffic_class, p.flow_label, ulen, 17, p.hop_limit, zero);
    uint8_t* u = t + 54;
    put_be16(u, p.def_src_port); put_be16(u + 2, p.def_dst_port); put_be16(u + 4, ulen); put_be16(u + 6, 0);
    a.l4_sum = 17u + ulen + (uint64_t)p.def_src_port + p.def_dst_port + ulen;
    a.src = p.src_ip; a.src_off = 22; a.ip_src = 0;
    a.dst = p.dst_ip; a.dst_off = 38;
    a.payload = p.payload; a.pay_off = 62; a.pay_len = p.payload_len;
    a.out = out; a.count = p.count; a.period = out_stride;
    a.l4_ck_off = 60; a.l4_dst = 1;
    e = launch_probe(a, t, 4, s);
    return true;
}

// tcp_ping / icmp_ping probe batches (ip.src_shared, dst per frame): the
// layouts and sums of k_build_l4
static bool try_probe_l4(const L4Args& l, int kind, uint8_t* out, uint32_t out_stride, hipStream_t s, hipError_t& e) {
    const nexg_ip_build& ip = l.ip;
    const bool v4 = ip.family == 4;
    const uint32_t l3 = v4 ? 20u : 40u;
    const uint32_t l4_hdr = kind == kL4Tcp ? 20u + l.opt_padded : 8u;
    const uint32_t l4_len = l4_hdr + l.payload_len;
    const uint32_t flen = 14u + l3 + l4_len;
    // icmp_ping IPv4: k_build_lane (whole-dword tile writes at any frame
    // period); tcp_ping: k_build_probe (0.72-0.89 of 8 TB/s written, round 5).
    // Measurement overrides (knobs build): NEXG_PROBE_ICMP = 1 the template
    // kernel, 2 the per-lane k_build_l4; NEXG_PROBE_LANE_TCP = 1 k_build_lane
    // for tcp_ping (no payload)
    static const uint32_t icmp_path = probe_env("NEXG_PROBE_ICMP", 0u, 0u, 2u);
    static const bool tcp_lane = probe_env("NEXG_PROBE_LANE_TCP", 0u, 0u, 1u) == 1u;
    // (ICMPv6's 67 B ran 0.634-0.637 in k_build_lane against 0.656 per lane in
    // k_build_l4, tcp_ping 0.69-0.70 against 0.80 in k_build_probe: both stay)
    const bool lane = kind == kL4Icmp ? icmp_path == 0u && v4 && lane_launch_ok(flen, out_stride, l.payload_len, out)
                                      : tcp_lane && l.payload_len == 0 && lane_launch_ok(flen, out_stride, 0, out);
    if (!lane && ((kind != kL4Tcp && icmp_path != 1u) || !probe_launch_ok(flen, out_stride, l.payload_len, out)))
        return false;
    ProbeArgs a{};
    uint8_t t[kProbeMaxP] = {0};
    const uint8_t zero[16] = {0};
    const uint32_t proto = kind == kL4Tcp ? 6u : (v4 ? 1u : 58u);
    probe_eth(t, ip.def_dst_mac, ip.def_src_mac, v4 ? 0x0800 : 0x86DD);
    if (v4) a.ip_sum = probe_ipv4(t + 14, ip.tos, 20u + l4_len, ip.def_ip_id, ip.ip_flags, ip.ttl, proto, zero);
    else probe_ipv6(t + 14, ip.tos, ip.flow_label, l4_len, proto, ip.ttl, zero);
    uint8_t* h = t + 14 + l3;
    uint64_t sum;
    if (kind == kL4Tcp) {
        const uint32_t w6 = ((l4_hdr / 4u) << 12) | (l.flags & 0xFFu);
        put_be16(h, l.def_sport); put_be16(h + 2, l.def_dport);
        put_be16(h + 4, l.def_seq >> 16); put_be16(h + 6, l.def_seq & 0xFFFFu);
        put_be16(h + 8, l.def_ack >> 16); put_be16(h + 10, l.def_ack & 0xFFFFu);
        put_be16(h + 12, w6); put_be16(h + 14, l.window); put_be16(h + 16, 0); put_be16(h + 18, l.urg);
        for (uint32_t k = 0; k < l.opt_padded; k++) h[20 + k] = l.options[k];
        sum = (uint64_t)l.def_sport + l.def_dport + (l.def_seq >> 16) + (l.def_seq & 0xFFFFu) + (l.def_ack >> 16) +
              (l.def_ack & 0xFFFFu) + w6 + l.window + l.urg + l.opt_sum;
        a.l4_ck_off = 14 + l3 + 16;
    } else {
        const uint32_t w0 = (l.icmp_type << 8) | l.icmp_code;
        put_be16(h, w0); put_be16(h + 2, 0); put_be16(h + 4, l.def_ident); put_be16(h + 6, l.def_seqno);
        sum = (uint64_t)w0 + l.def_ident + l.def_seqno;
        a.l4_ck_off = 14 + l3 + 2;
    }
    const bool pseudo = !v4 || kind == kL4Tcp;  // ICMPv4 sums the message alone
    if (pseudo) sum += proto + l4_len;
    a.l4_sum = sum;
    a.l4_dst = pseudo ? 1u : 0u;
    a.ip_ck_off = v4 ? 24u : 0u;
    a.ip_src = v4 ? 1u : 0u;
    a.src = ip.src_ip; a.src_off = v4 ? 26u : 22u;
    a.dst = ip.dst_ip; a.dst_off = v4 ? 30u : 38u;
    a.payload = l.payload; a.pay_off = 14 + l3 + l4_hdr; a.pay_len = l.payload_len;
    a.out = out; a.count = l.count; a.period = out_stride;
    e = lane ? launch_lane(a, t, ip.family, kind, s) : launch_probe(a, t, v4 ? 1u : 4u, s);
    return true;
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
    // (the probe batch stays per lane: 0.84-0.85 of 8 TB/s written against
    // 0.69-0.83 for the template kernel, profiles/r05/probe/)
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
    hipError_t e = hipSuccess;
    if (probe && try_probe_udp6(p, out, out_stride, s, e)) return e;
    if (probe) a.tile_order = build_tile_order();  // udp_ping's probe batch order (see launch_l4_fam)
    // a 16-KiB tile for the udp_ping shapes + build_lds_pad(): 5 workgroups per CU (0.279 -> 0.253 ms)
    // (a probe batch reaching here has a misaligned output or a long frame:
    // the per-lane kernel's src_shared branch takes it)
    if (staged && out_stride <= 64u)
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

#if NEXG_PROBE_TIMING
// measurement builds only: copy the builders' workgroup stamps to the host
extern "C" int nexg_debug_build_stamps(uint64_t* host, uint64_t n, int reset) {
    if (n > 8ull * nexg::kStampWgs) n = 8ull * nexg::kStampWgs;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(nexg::g_build_stamps), n * 8u, 0, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    if (reset) {
        void* p = nullptr;
        if (hipGetSymbolAddress(&p, HIP_SYMBOL(nexg::g_build_stamps)) != hipSuccess ||
            hipMemset(p, 0, 8ull * 8u * nexg::kStampWgs) != hipSuccess)
            return -1;
    }
    return 0;
}
#endif
