// nexg_parse.hip — batched Frame::try_from_buf + verification checksums on
// gfx950 (nex-packet/src/frame.rs:299-315, 570-658; util.rs:65-183).
//
// One lane per frame, 256-lane workgroups, one tile of 256 consecutive frames
// per workgroup; HBM is read once, coalesced:
//   TileStride64 / TileStride : fixed-stride batches. The workgroup streams its
//       whole tile (256 x stride bytes, contiguous) with 16-B loads in lane
//       order into per-frame LDS slots, padded to break bank conflicts.
//   SpanTile : packed batches (offset table without lengths, or any other
//       stride). The tile's frames are one contiguous byte span, streamed
//       through LDS in 16-KiB sub-tiles; L4 tail sums come from a prefix scan
//       of chunk sums (k_parse_span).
//   TwoPass : explicit lengths (frames anywhere, in any order): quarter-wave
//       tail sums past byte 80, then one lane per frame on an 80-B head.
#include <stdlib.h>
#include <string.h>

#include "parse_kernels.hpp"

namespace nexg {

// tile_index order named by an env variable (measurement overrides, compiled
// only into the -DNEXG_AB_KNOBS build nex_amd/libnexg_knobs.so that the A/B
// tools and tests/test_gpu_tile_order.py load; the product library has none):
// linear = 0, xcd = 1 (contiguous eighths), xcdK = XCD-local runs of K tiles;
// -1 when unset or unrecognised.
static int64_t order_from_env(const char* name) {
#ifdef NEXG_AB_KNOBS
    const char* e = getenv(name);
    if (!e) return -1;
    if (strncmp(e, "xcd", 3) == 0 && e[3]) return atoi(e + 3);
    if (strncmp(e, "cu", 2) == 0 && e[2]) return (int64_t)(0x80000000u | (uint32_t)atoi(e + 2));  // CU-affine runs
    return strcmp(e, "xcd") == 0 ? 1 : (strcmp(e, "linear") == 0 ? 0 : -1);
#else
    (void)name;
    return -1;
#endif
}

// Tile order of the parse kernels; NEXG_TILE_ORDER overrides (knobs build).
// Fixed-stride tiles (16 KiB at 64 B) take XCD-local runs of 16 tiles at every
// size (profiles/r04/tile_order/: 0.921-0.924 of 8 TB/s at 1 and 3.25 GiB, grid
// order 0.86-0.88, contiguous eighths 0.887-0.894, runs of 4 0.82-0.83). The
// span kernel's 256-frame groups (~90 KB of IMIX each) take XCD-local runs of
// 64 groups (~5.8 MB per run): in one process (profiles/r06/order/) IMIX
// 0.853 -> 0.870 of 8 TB/s, the App. C mix 0.782 -> 0.790, real traffic
// 0.784 -> 0.799 against grid order; runs of 16 / 32 / 128 gained less on one
// of them, runs of 2 and 8 nothing (round 5)
uint32_t tile_order_for(const ParseArgs& a) {
    static const int64_t forced = order_from_env("NEXG_TILE_ORDER");
    if (forced >= 0) return (uint32_t)forced;
    return a.offsets ? 64u : 16u;
}

// Tile order of the udp_ping builder (k_build_udp4) and the write-only stream
// probe; NEXG_BUILD_ORDER overrides. Contiguous eighths (profiles/r04/tile_order/
// builder_tile_order.log, 16M frames): probe batch 0.736-0.744 of 8 TB/s written
// against 0.697-0.701 in grid order, full tuples 0.680 against 0.663; runs of
// 16-64 tiles fall between.
uint32_t build_tile_order() {
    static const int64_t forced = order_from_env("NEXG_BUILD_ORDER");
    return forced >= 0 ? (uint32_t)forced : 1u;
}

// Tile order of the probe-batch template kernel (k_build_probe: tcp_ping and
// udp_ping's IPv6 branch); NEXG_PROBE_ORDER overrides. XCD-local runs of 64
// tiles: 16M frames in one process (profiles/r06/order/build_order2.log)
// tcp_ping 0.740 -> 0.807 of 8 TB/s written, udp6 0.666 -> 0.684 against
// contiguous eighths; runs of 16 lost (0.711). udp_ping's IPv4 probe batch
// (0.889 against 0.846 in runs of 64) and icmp_ping's k_build_lane (0.675
// against 0.639) keep contiguous eighths.
uint32_t probe_tile_order() {
    static const int64_t forced = order_from_env("NEXG_PROBE_ORDER");
    return forced >= 0 ? (uint32_t)forced : 64u;
}

// Tile order of the builders with several per-frame parameter arrays
// (k_build_udp6, k_build_l4); NEXG_L4_ORDER overrides. Grid order: contiguous
// eighths made tcp SYN 0.199 -> 0.230-0.240 ms and tcp_ping 0.247 -> 0.30 at
// 16M frames, icmp4 echo 0.133 -> 0.129 (profiles/r04/builders/order_ab.log).
uint32_t l4_build_tile_order() {
    static const int64_t forced = order_from_env("NEXG_L4_ORDER");
    return forced >= 0 ? (uint32_t)forced : 0u;
}

ParseVariant choose_parse_variant(const ParseArgs& a) {
    const bool aligned = (reinterpret_cast<uint64_t>(a.data) & 15u) == 0;
    if (!a.offsets && aligned && a.stride % 16u == 0 && a.stride > 0 && a.stride <= 128u &&
        a.count * (uint64_t)a.stride <= a.data_bytes) {
        return a.stride == 64u ? ParseVariant::TileStride64 : ParseVariant::TileStride;
    }
    if (!a.lengths && (a.offsets || a.stride > 0)) return ParseVariant::SpanTile;
    // explicit lengths in file order (capture records with their headers in
    // place): one ordered span per group, gaps read through (include/nexg.h)
    if (a.offsets && (a.hints & NEXG_FRAMES_MONOTONE)) return ParseVariant::SpanTile;
    return ParseVariant::TwoPass;
}

#ifndef NEXG_SPAN_SUB
#define NEXG_SPAN_SUB 24576  // span kernel sub-tile bytes (A/B builds override)
#endif
#ifndef NEXG_SPAN_WPE
#define NEXG_SPAN_WPE 5  // span kernel waves per SIMD (its VGPR cap)
#endif

// The span kernel's NEXG_OUT_GROUPED output: every group mixed (head
// NEXG_GROUPED_TILE_RUN), so from NEXG_GROUPED_CODE_OFFSET on it is
// NEXG_OUT_SPARSE's layout (codes, then the exceptions at the next 16-B
// boundary, one run per 256-frame tile): the SPARSE instance writes it there
// and stores the heads.
static ParseArgs grouped_as_sparse(const ParseArgs& a) {
    ParseArgs b = a;
    b.grouped_heads = static_cast<uint8_t*>(a.out);
    b.out = static_cast<uint8_t*>(a.out) + NEXG_GROUPED_CODE_OFFSET(a.count);
    return b;
}

template <int OUT>
static hipError_t launch_parse_out(ParseVariant v, const ParseArgs& a, hipStream_t s) {
    const uint64_t blocks = (a.count + kTile - 1) / kTile;
    dim3 grid((uint32_t)blocks), block(kTile);
    switch (v) {
        case ParseVariant::TileStride64:
            hipLaunchKernelGGL((k_parse<0, OUT, 64, 64, true, true>), grid, block, 0, s, a);
            break;
        case ParseVariant::TileStride:
            hipLaunchKernelGGL((k_parse<0, OUT, 0, 128>), grid, block, 0, s, a);
            break;
        case ParseVariant::LaneWindow:
            hipLaunchKernelGGL((k_parse<1, OUT, 0, 128>), grid, block, 0, s, a);
            break;
        case ParseVariant::SpanTile:
            // 24-KiB sub-tiles at 5 waves/SIMD (31 KB LDS, 5 workgroups per CU:
            // 120 KB in flight per CU): in one process +0.9 % over 20 KiB at 6
            // waves on IMIX and real traffic, the mix equal. 4 waves (24 or 28
            // KiB) run IMIX +1.9 % and real +1.4 % but the App. C mix -5.8 %:
            // its generic section needs the fifth workgroup to hide its latency
            // (profiles/r05/subtile_ab.log; round 2 had measured 20 KiB +2.6 %
            // over 16 KiB and 24 KiB equal, 28-32 KiB slower:
            // profiles/r02_kbench/kbench_subtile.log). Records (about 100
            // VGPRs) run uncapped on 16 KiB: capping them spills 44+ B.
            // (Two-barrier / double-buffered generations measured slower,
            // 0.66-0.69 vs 0.75: tools/kbench.hip keeps them for A/B.)
            if (OUT == NEXG_OUT_RECORD) hipLaunchKernelGGL((k_parse_span<OUT, 1, 16384, 1>), grid, block, 0, s, a);
            else if (OUT == NEXG_OUT_GROUPED)
                hipLaunchKernelGGL((k_parse_span<NEXG_OUT_SPARSE, 1, NEXG_SPAN_SUB, NEXG_SPAN_WPE>), grid, block, 0, s,
                                   grouped_as_sparse(a));
            else hipLaunchKernelGGL((k_parse_span<OUT, 1, NEXG_SPAN_SUB, NEXG_SPAN_WPE>), grid, block, 0, s, a);
            break;
        case ParseVariant::TwoPass:
            hipLaunchKernelGGL((k_tail_sums<OUT, 4>), grid, block, 0, s, a);
            hipLaunchKernelGGL(k_parse_lane80<OUT>, grid, block, 0, s, a);
            break;
    }
    return hipGetLastError();
}

// FrameSlice output: header bytes only, staged exactly as the parse kernels
// stage them (whole tile for small fixed strides, a 128-B lane window plus
// HBM reads for deeper IPv6 extension chains otherwise).
static hipError_t launch_slice(ParseVariant v, const ParseArgs& a, hipStream_t s) {
    const uint64_t blocks = (a.count + kTile - 1) / kTile;
    dim3 grid((uint32_t)blocks), block(kTile);
    if (v == ParseVariant::TileStride64)
        hipLaunchKernelGGL((k_parse<0, NEXG_OUT_SLICE, 64, 64, false, true>), grid, block, 0, s, a);
    else if (v == ParseVariant::TileStride)
        hipLaunchKernelGGL((k_parse<0, NEXG_OUT_SLICE, 0, 128>), grid, block, 0, s, a);
    else
        hipLaunchKernelGGL((k_parse<1, NEXG_OUT_SLICE, 0, 128>), grid, block, 0, s, a);
    return hipGetLastError();
}

hipError_t launch_span_clock(const ParseArgs& a, hipStream_t s) {
    if (a.count == 0) return hipSuccess;
    const uint64_t blocks = (a.count + kTile - 1) / kTile;
    hipLaunchKernelGGL((k_parse_span<NEXG_OUT_SPARSE, 1, NEXG_SPAN_SUB, NEXG_SPAN_WPE, true>), dim3((uint32_t)blocks),
                       dim3(kTile), 0, s, grouped_as_sparse(a));
    return hipGetLastError();
}

hipError_t launch_parse(ParseVariant v, const ParseArgs& a, int out_kind, hipStream_t s) {
    if (a.count == 0) return hipSuccess;
    if (out_kind == NEXG_OUT_SLICE) return launch_slice(v, a, s);
    if (out_kind == NEXG_OUT_FLAGS) return launch_parse_out<NEXG_OUT_FLAGS>(v, a, s);
    // TwoPass with the 2-B / 1-B outputs hands tail sums through a.tail
    if (parse_needs_tail(v, out_kind) && !a.tail) return hipErrorInvalidValue;
    if (out_kind == NEXG_OUT_VERDICT) return launch_parse_out<NEXG_OUT_VERDICT>(v, a, s);
    if (out_kind == NEXG_OUT_SPARSE) return launch_parse_out<NEXG_OUT_SPARSE>(v, a, s);
    if (out_kind == NEXG_OUT_GROUPED) return launch_parse_out<NEXG_OUT_GROUPED>(v, a, s);
    return out_kind == NEXG_OUT_DESC ? launch_parse_out<NEXG_OUT_DESC>(v, a, s)
                                     : launch_parse_out<NEXG_OUT_RECORD>(v, a, s);
}

// nexg_sparse_expand / nexg_grouped_expand: lane per frame; code -> nexg_desc
// (include/nexg.h table), exception codes take the group's next exception in
// frame order. GROUPED: a uniform group's code is its head plus the frame's
// two mask bits; a mixed group's codes and exceptions sit where SPARSE keeps
// them, past the heads and masks.
template <bool GROUPED>
__global__ __launch_bounds__(256) void k_sparse_expand(ParseArgs a, const uint8_t* sparse, nexg_desc* out) {
    __shared__ uint32_t s_wexc[4];  // GROUPED: each wave's exceptions (a NEXG_GROUPED_TILE_RUN tile's run)
    const uint64_t idx = (uint64_t)blockIdx.x * kTile + threadIdx.x;
    const bool valid = idx < a.count;
    uint32_t code = 0xFFu, head = 0;
    const uint8_t* codes = sparse;
    const nexg_desc* exc = reinterpret_cast<const nexg_desc*>(sparse + NEXG_SPARSE_EXC_OFFSET(a.count));
    if (GROUPED) {
        codes = sparse + NEXG_GROUPED_CODE_OFFSET(a.count);
        exc = reinterpret_cast<const nexg_desc*>(sparse + NEXG_GROUPED_EXC_OFFSET(a.count));
    }
    if (valid) {
        head = GROUPED ? sparse[idx >> 6] : 0u;
        if (head && head != NEXG_GROUPED_TILE_RUN) {
            const uint4 m = reinterpret_cast<const uint4*>(sparse + NEXG_GROUPED_MASK_OFFSET(a.count))[idx >> 6];
            const uint32_t b = (uint32_t)idx & 63u;
            const uint32_t ip = b < 32u ? m.x : m.y, l4 = b < 32u ? m.z : m.w;
            code = head | (((ip >> (b & 31u)) & 1u) ? NEXG_SPARSE_IP_OK : 0u) |
                   (((l4 >> (b & 31u)) & 1u) ? NEXG_SPARSE_L4_OK : 0u);
        } else {
            code = codes[idx];
        }
    }
    const uint64_t m = __ballot(code == 0u);
    uint32_t below = 0;  // a tile run: the exceptions of the tile's lower waves
    if (GROUPED) {
        if ((threadIdx.x & 63u) == 0u) s_wexc[threadIdx.x >> 6] = (uint32_t)__builtin_popcountll(m);
        __syncthreads();
        for (uint32_t w = 0; w < (threadIdx.x >> 6); w++) below += s_wexc[w];
    }
    if (!valid) return;
    uint64_t off;
    uint32_t len = 0;
    frame_extent(a, idx, off, len);
    nexg_desc d;
    if (!sparse_decode(code, len, a.opt_flags, a.ip_offset, d))
        d = exc[GROUPED && head == NEXG_GROUPED_TILE_RUN ? (idx & ~255ull) + below + lanes_below(m)
                                                         : (idx & ~63ull) + lanes_below(m)];
    out[idx] = d;
}

hipError_t launch_sparse_expand(const ParseArgs& a, const uint8_t* sparse, nexg_desc* out, bool grouped,
                                hipStream_t s) {
    if (a.count == 0) return hipSuccess;
    const uint64_t blocks = (a.count + kTile - 1) / kTile;
    if (grouped) hipLaunchKernelGGL(k_sparse_expand<true>, dim3((uint32_t)blocks), dim3(kTile), 0, s, a, sparse, out);
    else hipLaunchKernelGGL(k_sparse_expand<false>, dim3((uint32_t)blocks), dim3(kTile), 0, s, a, sparse, out);
    return hipGetLastError();
}

// nexg_decode_options: Ipv4Header.options (ipv4.rs:442-508) and
// TcpHeader.options (tcp.rs:767-818) of each frame as positions, one lane per
// frame, over the headers its record (a prior NEXG_OUT_RECORD parse) locates.
// Not a hot path: byte loads, the 96-B result assembled in private memory.
static_assert(sizeof(nexg_options) == 96, "nexg_options is 96 bytes (include/nexg.h)");

__global__ __launch_bounds__(256) void k_decode_options(ParseArgs a, const nexg_record* recs,
                                                        nexg_options* out) {
    const uint64_t idx = (uint64_t)blockIdx.x * kTile + threadIdx.x;
    if (idx >= a.count) return;
    nexg_options o;
    __builtin_memset(&o, 0, sizeof(o));
    const nexg_record& r = recs[idx];
    const uint32_t flags = r.flags;
    uint64_t off;
    uint32_t len;
    if (frame_extent(a, idx, off, len) && ((flags >> NEXG_STATUS_SHIFT) & 7u) == 0) {
        const uint8_t* g = a.data + off;
        const uint32_t l3 = r.l3_off, ihl4 = 4u * (r.ip_ver_ihl & 0xFu);
        if ((flags & NEXG_L_IPV4) && l3 + ihl4 <= len) {
            const uint8_t* h = g + l3;
            uint32_t i = 20, n = 0;
            while (i < ihl4) {
                const uint32_t num = h[i] & 0x1Fu;
                if (num <= 1u) {  // EOL ends the list, NOP is one byte
                    o.ip_pos[n++] = (uint8_t)(i - 20u);
                    if (num == 0u) break;
                    i += 1;
                    continue;
                }
                if (i + 2 > ihl4) break;
                const uint32_t l = h[i + 1];
                if (l < 2 || i + l > ihl4) break;
                o.ip_pos[n++] = (uint8_t)(i - 20u);
                i += l;
            }
            o.n_ip = (uint8_t)n;
            o.ip_opt_off = (uint16_t)(l3 + 20u);
        }
        const uint32_t l4 = r.l4_off, hl = 4u * (r.l4_code >> 4);
        if ((flags & NEXG_L_TCP) && l4 + hl <= len) {
            const uint8_t* h = g + l4;
            uint32_t p = 20, n = 0;
            while (p < hl) {
                const uint32_t start = p, kind = h[p++];
                if (kind <= 1u) {
                    o.tcp_pos[n++] = (uint8_t)(start - 20u);
                    if (kind == 0u) break;
                    continue;
                }
                if (p >= hl) break;
                const uint32_t l = h[p++];
                if (l < 2 || p + (l - 2) > hl) break;
                o.tcp_pos[n++] = (uint8_t)(start - 20u);
                p += l - 2;
            }
            o.n_tcp = (uint8_t)n;
            o.tcp_opt_off = (uint16_t)(l4 + 20u);
        }
    }
    uint4 v[6];
    __builtin_memcpy(v, &o, sizeof(o));
    uint4* dst = reinterpret_cast<uint4*>(out + idx);
#pragma unroll
    for (int k = 0; k < 6; k++) dst[k] = v[k];
}

hipError_t launch_decode_options(const ParseArgs& a, const nexg_record* recs, nexg_options* out,
                                 hipStream_t s) {
    if (a.count == 0) return hipSuccess;
    const uint64_t blocks = (a.count + kTile - 1) / kTile;
    hipLaunchKernelGGL(k_decode_options, dim3((uint32_t)blocks), dim3(kTile), 0, s, a, recs, out);
    return hipGetLastError();
}

// calibration stream (include/nexg.h nexg_probe_stream): the parse kernels'
// load shape with either the 8-B-per-64-B descriptor store stream or none
// (tiles in the parse kernels' fixed-stride tile order)
// OCC6: the out_per_64 = 9 instance (its own symbol, so a kernel trace tells
// the occupancy-capped run from the 8-per-CU one)
template <bool W8, bool OCC6 = false>
__global__ __launch_bounds__(256) void k_probe_stream(const uint8_t* data, void* out, uint32_t order) {
    __shared__ uint32_t s_x[4];
    extern __shared__ uint32_t s_occ[];  // dynamic LDS: caps workgroups per CU only (out_per_64 = 9)
    const uint32_t t = threadIdx.x;
    if (order == 0xFFFFFFFFu) s_occ[t] = 0u;
    const uint64_t tile = tile_index(order);
    const uint8_t* T = data + tile * 16384u;
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = load16<true>(T + 16u * (t + 256u * k));
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    const uint64_t i = tile * kTile + t;
    if (W8) {
        reinterpret_cast<uint2*>(out)[i] = make_uint2(x, (uint32_t)i);
    } else {
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) x ^= __shfl_xor(x, d, 64);
        if ((t & 63u) == 0) s_x[t >> 6] = x;
        __syncthreads();
        if (t == 0) reinterpret_cast<uint32_t*>(out)[tile] = s_x[0] ^ s_x[1] ^ s_x[2] ^ s_x[3];
    }
}

// write-only calibration stream: the builders' copy-out shape (16-B
// non-temporal stores, 16 KiB per 256-lane workgroup, the builder's tile
// order and workgroups per CU); out[tile][c] = {tile, c, 0, 0}
__global__ __launch_bounds__(256) void k_probe_write(uint8_t* out, uint32_t order) {
    extern __shared__ uint32_t s_cap[];  // dynamic LDS: caps workgroups per CU only
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const uint64_t tile = tile_index(order);
    if (order == 0xFFFFFFFFu) s_cap[threadIdx.x] = 0u;
    v4u* T = reinterpret_cast<v4u*>(out + tile * 16384u);
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
        const uint32_t c = threadIdx.x + 256u * k;
        __builtin_nontemporal_store(v4u{(uint32_t)tile, c, 0u, 0u}, T + c);
    }
}

hipError_t launch_probe_stream(const uint8_t* data, uint64_t tiles, uint32_t mode, void* out, hipStream_t s) {
    if (tiles == 0) return hipSuccess;
    ParseArgs fixed{};
    fixed.stride = 64;
    const uint32_t ro = tile_order_for(fixed), wo = build_tile_order();
    if (mode == 64)  // the builder's LDS footprint: its 16-KiB tile + build_lds_pad()
        hipLaunchKernelGGL(k_probe_write, dim3((uint32_t)tiles), dim3(kTile), 16400u + build_lds_pad(), s,
                           static_cast<uint8_t*>(out), wo);
    else if (mode == 8) hipLaunchKernelGGL(k_probe_stream<true>, dim3((uint32_t)tiles), dim3(kTile), 0, s, data, out, ro);
    else if (mode == 9)  // 6 workgroups per CU: the fixed-stride parse kernel's occupancy
        hipLaunchKernelGGL((k_probe_stream<true, true>), dim3((uint32_t)tiles), dim3(kTile), 160u * 1024u / 6u - 1024u, s,
                           data, out, ro);
    else hipLaunchKernelGGL(k_probe_stream<false>, dim3((uint32_t)tiles), dim3(kTile), 0, s, data, out, ro);
    return hipGetLastError();
}

// dependent-load latency probe (include/nexg.h nexg_probe_latency): a ring
// of 64-B lines, line i holding the index of line (i + kChaseStride) mod n
// (a stride of ~1 MiB: every step another DRAM page), chased by one lane
constexpr uint32_t kChaseStride = 16411;  // prime: one cycle through every line when n is not a multiple
__global__ __launch_bounds__(256) void k_chase_init(uint32_t* buf, uint32_t n, uint64_t* out) {
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (i < n) buf[i * 16u] = (uint32_t)((i + kChaseStride) % n);
    if (i < 4) out[i] = 0;
}
// workgroup 0, lane 0: `steps` dependent loads from line `start`, then
// out[0] = shader-clock ticks, out[1] = 100-MHz ticks, out[3] = the last line
// (keeps the chain live), and the done flag out[2] raised. The other
// workgroups (the loaded case) stream-read the buffer in 16-B chunks until the
// flag is up or `rounds` passes are done, whichever comes first.
__global__ __launch_bounds__(256) void k_chase(const uint32_t* buf, uint32_t n, uint32_t start, uint32_t steps,
                                               uint32_t rounds, uint64_t* out) {
    uint32_t* done = reinterpret_cast<uint32_t*>(out + 2);
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) {
            const auto* b = NEXG_GLOBAL(uint32_t, buf);
            uint32_t j = start % n;
            j = b[(uint64_t)j * 16u];  // first touch outside the timed chain
            const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
            for (uint32_t k = 0; k < steps; k++) j = b[(uint64_t)j * 16u];
            const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
            out[0] = c1 - c0;
            out[1] = r1 - r0;
            out[3] = j;
            __hip_atomic_store(done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    const uint64_t chunks = (uint64_t)n * 4u, lanes = (uint64_t)(gridDim.x - 1u) * 256u;
    uint32_t x = 0;
    for (uint32_t r = 0; r < rounds; r++) {
        if (__hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
        for (uint64_t c = (uint64_t)(blockIdx.x - 1u) * 256u + threadIdx.x; c < chunks; c += lanes) {
            const uint4 v = load16<true>(reinterpret_cast<const uint8_t*>(buf) + 16u * c);
            x ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (x == 0x9e3779b9u) out[3] = x;  // never true on the ring's contents: a pure read stream
}

hipError_t launch_probe_latency(uint32_t* buf, uint32_t lines, uint32_t start, uint32_t steps, uint32_t loaded_wgs,
                                uint32_t rounds, uint64_t* out, hipStream_t s) {
    hipLaunchKernelGGL(k_chase_init, dim3((lines + 255u) / 256u), dim3(256), 0, s, buf, lines, out);
    hipLaunchKernelGGL(k_chase, dim3(1u + loaded_wgs), dim3(256), 0, s, buf, lines, start, steps, rounds, out);
    return hipGetLastError();
}

// util.rs:65-71 checksum(buf, skipword) per buffer; words outside the buffer
// and the skipped word contribute nothing; empty -> 0.
__global__ __launch_bounds__(256) void k_checksum(ParseArgs a, uint32_t skipword, uint16_t* out) {
    const uint64_t idx = (uint64_t)blockIdx.x * kTile + threadIdx.x;
    if (idx >= a.count) return;
    const uint64_t off = a.offsets ? table_off(a, idx, idx) : idx * (uint64_t)a.stride;
    const uint64_t l64 = a.lengths ? (uint64_t)a.lengths[idx]
                                   : (a.offsets ? table_off(a, idx + 1, idx) - off : (uint64_t)a.stride);
    if (l64 == 0 || l64 > 65535u || off > a.data_bytes || l64 > a.data_bytes - off) {
        out[idx] = 0;
        return;
    }
    const uint32_t len = (uint32_t)l64;
    GlobalFrame f{a.data + off};
    FrameOps<GlobalFrame> o{f, (uint32_t)((reinterpret_cast<uint64_t>(f.g)) & 1u)};
    const uint64_t sk = 2ull * skipword;
    uint64_t t;
    if (sk >= len) {
        t = o.wsum(0, len);
    } else {
        t = o.wsum(0, (uint32_t)sk);
        if (sk + 2 < len) t += o.wsum((uint32_t)sk + 2u, len);
    }
    out[idx] = (uint16_t)fold_complement(t);
}

hipError_t launch_checksum(const ParseArgs& a, uint32_t skipword, uint16_t* out, hipStream_t s) {
    if (a.count == 0) return hipSuccess;
    const uint64_t blocks = (a.count + kTile - 1) / kTile;
    hipLaunchKernelGGL(k_checksum, dim3((uint32_t)blocks), dim3(kTile), 0, s, a, skipword, out);
    return hipGetLastError();
}

}  // namespace nexg

