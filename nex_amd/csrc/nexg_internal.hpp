// nexg_internal.hpp — host-side launch interfaces shared between the kernel
// translation units and the C ABI (nexg_api.hip). Not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nexg.h"

namespace nexg {

struct ParseArgs {
    const uint8_t* data;
    uint64_t data_bytes;
    const uint64_t* offsets;
    const uint32_t* lengths;
    uint32_t stride;
    uint64_t count;
    uint32_t opt_flags;
    uint32_t ip_offset;
    void* out;
    uint32_t tile_order = 0;  // fixed-stride tiles: 0 in grid order, 1 XCD-contiguous
    uint32_t hints = 0;       // NEXG_FRAMES_* (include/nexg.h)
    uint32_t* tail = nullptr; // TwoPass tail-sum hand-off (count entries) for outputs
                              // narrower than 4 B per frame; null -> the output itself
    uint64_t* stamps = nullptr;  // k_parse_span<..., TIMING>: 8 clock stamps per workgroup
    uint8_t* grouped_heads = nullptr;  // span kernel, NEXG_OUT_GROUPED run as SPARSE at the code offset: head bytes
                                       // (all NEXG_GROUPED_TILE_RUN: exceptions in one run per 256-frame tile)
    const uint64_t* off_bases = nullptr;  // NEXG_FRAMES_OFFSETS32 over 4 GiB: one full offset per 256 frames
};

// Kernel variants of the parse path.
enum class ParseVariant {
    TileStride64,   // fixed 64-B stride: coalesced tile staging into LDS
    TileStride,     // fixed stride (multiple of 16, <= 128): tile staging
    LaneWindow,     // any layout: per-lane 128-B window, lane sums its own tail
    TwoPass,        // any layout: k_tail_sums (bytes past 80) + k_parse_lane80
    SpanTile,       // packed layouts: 16-KiB sub-tiles through LDS + chunk prefix sums
};

hipError_t launch_parse(ParseVariant v, const ParseArgs& a, int out_kind, hipStream_t s);
// nexg_probe_span_clock: the span kernel's stamped instance (grouped output)
hipError_t launch_span_clock(const ParseArgs& a, hipStream_t s);
// TwoPass hands each frame's tail sum to pass 2 through its own output
// element; outputs narrower than 4 B need a.tail (count u32) instead.
inline bool parse_needs_tail(ParseVariant v, int out_kind) {
    return v == ParseVariant::TwoPass &&
           (out_kind == NEXG_OUT_VERDICT || out_kind == NEXG_OUT_SPARSE || out_kind == NEXG_OUT_GROUPED);
}
uint32_t tile_order_for(const ParseArgs& a);
uint32_t build_tile_order();
uint32_t l4_build_tile_order();
uint32_t probe_tile_order();
uint32_t build_lds_pad();  // dynamic LDS of the udp_ping builds (workgroups per CU)
ParseVariant choose_parse_variant(const ParseArgs& a);

// Tile handled by this workgroup. Workgroups are dispatched to the 8 XCDs
// round-robin (blockIdx % 8).
//  order 0: grid order, tile = b.
//  order 1: each XCD one contiguous eighth of the batch, tile = (b % 8) * (nb / 8) + b / 8.
//  order K >= 2: XCD-local runs of K consecutive tiles, the runs dealt to the
//    XCDs round-robin — XCD x's i-th workgroup takes tile (i / K * 8 + x) * K + i % K.
//    At any moment each XCD streams its own K-tile run of the batch instead of
//    every eighth tile (profiles/r04/tile_order/: K = 16 over 16-KiB tiles is
//    5-7 % faster than grid order at 1 and 3.25 GiB; K = 4 is 5 % slower).
// Workgroups past the last whole group of 8 (order 1) or 8K (order K) keep grid
// order, so the map is a bijection on [0, nb) for every grid size.
__host__ __device__ __forceinline__ uint64_t tile_of(uint32_t b, uint32_t nb, uint32_t order) {
    if (!order) return b;
    if (order & 0x80000000u) {  // CU-affine runs (measurement order "cuR", round 6): XCD-local runs of
        // 32 R tiles in which the XCD's c-th workgroup of a dispatch round (CU c of 32 at launch)
        // takes R consecutive tiles: tile c R + j for the run's (32 j + c)-th workgroup
        const uint32_t R = order & 0x7FFFFFFFu;
        if (R == 0 || R > (nb >> 8)) return b;  // no whole run of 8 x 32 R
        const uint32_t K = 32u * R;
        const uint32_t whole = nb / (8u * K) * (8u * K);
        if (b >= whole) return b;
        const uint32_t i = b >> 3, x = b & 7u, l = i % K;
        return ((uint64_t)(i / K) * 8u + x) * K + (uint64_t)(l % 32u) * R + l / 32u;
    }
    if (order == 1u) {
        const uint32_t q = nb >> 3;
        return b >= (q << 3) ? b : (uint64_t)(b & 7u) * q + (b >> 3);
    }
    const uint32_t K = order;
    if (K > (nb >> 3)) return b;  // no whole group (and 8K cannot overflow below)
    const uint32_t whole = nb / (8u * K) * (8u * K);
    if (b >= whole) return b;
    const uint32_t i = b >> 3, x = b & 7u;
    return ((uint64_t)(i / K) * 8u + x) * K + i % K;
}
__device__ __forceinline__ uint64_t tile_index(uint32_t order) { return tile_of(blockIdx.x, gridDim.x, order); }

hipError_t launch_checksum(const ParseArgs& a, uint32_t skipword, uint16_t* out, hipStream_t s);

hipError_t launch_sparse_expand(const ParseArgs& a, const uint8_t* sparse, nexg_desc* out, bool grouped,
                                hipStream_t s);

hipError_t launch_recompute(const ParseArgs& a, uint32_t which, nexg_fixup* out, hipStream_t s);

hipError_t launch_decode_options(const ParseArgs& a, const nexg_record* recs, nexg_options* out,
                                 hipStream_t s);

hipError_t launch_probe_stream(const uint8_t* data, uint64_t tiles, uint32_t mode, void* out, hipStream_t s);
hipError_t launch_probe_latency(uint32_t* buf, uint32_t lines, uint32_t start, uint32_t steps, uint32_t loaded_wgs,
                                uint32_t rounds, uint64_t* out, hipStream_t s);

hipError_t launch_build_udp4_tuples(const nexg_udp4_build& p, const nexg_udp4_tuple* tuples, uint8_t* out,
                                    uint32_t out_stride, hipStream_t s);
hipError_t launch_build_udp4(const nexg_udp4_build& p, uint8_t* out, uint32_t out_stride,
                             hipStream_t s);

hipError_t launch_build_udp6(const nexg_udp6_build& p, uint8_t* out, uint32_t out_stride,
                             hipStream_t s);

hipError_t launch_build_tcp(const nexg_tcp_build& p, uint8_t* out, uint32_t out_stride, hipStream_t s);
hipError_t launch_build_icmp_echo(const nexg_icmp_echo_build& p, uint8_t* out, uint32_t out_stride,
                                  hipStream_t s);

hipError_t launch_build_arp(const nexg_arp_build& p, uint8_t* out, uint32_t out_stride, hipStream_t s);
hipError_t launch_build_ndp_ns(const nexg_ndp_ns_build& p, uint8_t* out, uint32_t out_stride, hipStream_t s);

hipError_t launch_gen_lengths(int workload, uint64_t seed, uint64_t first, uint64_t count,
                              uint32_t* lengths, hipStream_t s);
hipError_t launch_gen_frames(int workload, uint64_t seed, uint64_t first, uint64_t count,
                             uint8_t* data, const uint64_t* offsets, uint32_t stride,
                             hipStream_t s);
hipError_t launch_gen_udp4_params(uint64_t seed, uint64_t first, uint64_t count,
                                  uint32_t* src_ip, uint32_t* dst_ip, uint16_t* sport,
                                  uint16_t* dport, uint16_t* ip_id, hipStream_t s);

}  // namespace nexg
