// parse_kernels.hpp — the gfx950 parse kernels (one lane per frame, one
// 256-frame tile per workgroup), shared by the library launchers
// (nexg_parse.hip) and the kernel microbenchmarks (tools/kbench.hip).
#pragma once

#include "frame_core.hpp"
#include "nexg_internal.hpp"

namespace nexg {

constexpr uint32_t kTile = 256;

// NEXG_OUT_DESC store shape of the span kernel and the lane-per-frame
// kernels (A/B builds): 2 = a span tile's descriptors staged in LDS and stored
// as 16-B non-temporal pairs, 8-B non-temporal per lane elsewhere; 1 = 8-B
// non-temporal per lane; 0 = 8-B plain per lane. In one process (profiles/
// r05/desc_ab/): 16M IMIX 0.751 / 0.749 / 0.736 of 8 TB/s. The fixed-stride
// tile kernel (k_parse MODE 0) stores plain 8-B descriptors per lane: UDP64
// 0.725 plain against 0.718 non-temporal and 0.703 staged.
#ifndef NEXG_DESC_MODE
#define NEXG_DESC_MODE 2
#endif
// k_parse_span: bytes of the previous sub-tile kept in front (and of pad
// behind): at least the slot, so a head window that starts there is whole
constexpr uint32_t kApron = NEXG_SPAN_SLOT > 96 ? NEXG_SPAN_SLOT : 96;

// Frame read entirely from HBM (checksum utility path).
struct GlobalFrame {
    NEXG_NO_DEFER
    const uint8_t* g;
    NEXG_HD uint32_t u8(uint32_t i) const { return g[i]; }
    NEXG_HD uint64_t le_sum(uint32_t a, uint32_t b) const {
        const uint64_t base = reinterpret_cast<uint64_t>(g);
        return global_le_sum(base + a, base + b);
    }
};

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t u = __shfl_up(v, d, 64);
        if (lane >= d) v += u;
    }
    return v;
}

constexpr uint32_t kPiece = 256;  // bytes per piece = 16 lanes x 16 B

template <int OUT>
__device__ __forceinline__ void store_result(void* out, uint64_t idx, const nexg_record& r) {
    if (OUT == NEXG_OUT_FLAGS) {  // non-temporal: +2.6 % on the 4-B stream (streambench w4_nt)
        __builtin_nontemporal_store(r.flags, reinterpret_cast<uint32_t*>(out) + idx);
    } else if (OUT == NEXG_OUT_VERDICT) {  // include/nexg.h: lossless 2-B form of the flags
        const uint32_t st = (r.flags >> NEXG_STATUS_SHIFT) & 7u;
        const uint16_t v = (uint16_t)(st ? (NEXG_VERDICT_ERR | (st << 3)) : (r.flags & 0xFFFFu));
        __builtin_nontemporal_store(v, reinterpret_cast<uint16_t*>(out) + idx);
    } else if (OUT == NEXG_OUT_DESC) {  // non-temporal, as the flags / verdict streams
        typedef uint32_t v2u __attribute__((ext_vector_type(2)));
        const v2u d{r.flags, (uint32_t)r.payload_off | ((uint32_t)r.payload_len << 16)};
        if (NEXG_DESC_MODE >= 1) __builtin_nontemporal_store(d, reinterpret_cast<v2u*>(out) + idx);
        else reinterpret_cast<v2u*>(out)[idx] = d;
    } else {
        uint4 v[4];
        __builtin_memcpy(v, &r, sizeof(r));
        uint4* dst = reinterpret_cast<uint4*>(out) + idx * 4;
#pragma unroll
        for (int k = 0; k < 4; k++) dst[k] = v[k];
    }
}

// the 1-B-code outputs (NEXG_OUT_SPARSE and its grouped form): whole-wave stores
constexpr bool sparse_like(int out) { return out == NEXG_OUT_SPARSE || out == NEXG_OUT_GROUPED; }

// rank of this lane among the set lanes of m below it (v_mbcnt)
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// NEXG_OUT_SPARSE / NEXG_OUT_GROUPED store (include/nexg.h) of a code already
// known for every lane (0: exception). Called by all 64 lanes of a wave
// together (valid = the lane holds frame idx; idx = 64-frame-group base +
// lane). SPARSE: a ballot compacts the wave's exceptions into exc[group*64 +
// rank]; the 1-B codes of lanes 4q..4q+3 are gathered by DPP quad broadcasts
// and stored as one non-temporal dword by lane 4q. GROUPED: a group whose
// valid lanes share one non-exception code up to the verdict bits stores that
// code as its head byte and its verdicts as two 64-bit ballots (16 B); any
// other group stores head 0, then what SPARSE stores, past the heads and masks.
// The span kernel's grouped output runs as SPARSE with a.grouped_heads set
// (heads NEXG_GROUPED_TILE_RUN, stored by the caller): its exceptions go in one
// run per 256-frame tile, and the whole workgroup must call this together.
template <int OUT, bool GROUP_CHECK = true>
__device__ __forceinline__ void store_sparse_coded(const ParseArgs& a, uint64_t idx, bool valid,
                                                   const nexg_record& r, uint32_t code) {
    uint8_t* const o = reinterpret_cast<uint8_t*>(a.out);
    const uint32_t c = valid ? code : 0u;
    uint8_t* codes = o;
    uint2* x = reinterpret_cast<uint2*>(o + NEXG_SPARSE_EXC_OFFSET(a.count));
    if constexpr (OUT == NEXG_OUT_GROUPED) {
        if ((idx & ~63ull) >= a.count) return;  // a wave past the last group (wave-uniform)
        const uint32_t base = c & ~(NEXG_SPARSE_IP_OK | NEXG_SPARSE_L4_OK);
        const uint32_t c0 = __builtin_amdgcn_readfirstlane(base);  // lane 0 holds the group's first frame
        const bool uniform = GROUP_CHECK && __all(!valid || base == c0) && (c0 & 0xFu) != 0u;
        const uint64_t g = idx >> 6;
        if (GROUP_CHECK && (idx & 63u) == 0u) o[g] = (uint8_t)(uniform ? c0 : 0u);  // else: the caller's
        if (uniform) {
            const uint64_t mi = __ballot(c & NEXG_SPARSE_IP_OK), ml = __ballot(c & NEXG_SPARSE_L4_OK);
            if ((idx & 63u) == 0u)
                __builtin_nontemporal_store(u32x4{(uint32_t)mi, (uint32_t)(mi >> 32), (uint32_t)ml, (uint32_t)(ml >> 32)},
                                            reinterpret_cast<u32x4*>(o + NEXG_GROUPED_MASK_OFFSET(a.count)) + g);
            return;
        }
        codes = o + NEXG_GROUPED_CODE_OFFSET(a.count);
        x = reinterpret_cast<uint2*>(o + NEXG_GROUPED_EXC_OFFSET(a.count));
    }
    const bool exc = valid && code == 0u;
    const uint64_t m = __ballot(exc);
    uint64_t slot = (idx & ~63ull) + lanes_below(m);
    if (OUT == NEXG_OUT_SPARSE && a.grouped_heads) {
        // the span kernel's grouped output (heads NEXG_GROUPED_TILE_RUN): the
        // 256-frame tile's exceptions as one run. Every thread of the
        // workgroup calls this together; each group's exceptions written apart
        // cost 1.5-3 % on the real-traffic / App. C batches
        __shared__ uint32_t s_wexc[4];
        if ((threadIdx.x & 63u) == 0u) s_wexc[threadIdx.x >> 6] = (uint32_t)__builtin_popcountll(m);
        __syncthreads();
        uint32_t below = 0;
        for (uint32_t w = 0; w < (threadIdx.x >> 6); w++) below += s_wexc[w];
        slot = (idx & ~255ull) + below + lanes_below(m);
        // non-temporal: real traffic 0.9236-0.9253 -> 0.9083-0.9098 ms, the
        // App. C mix 0.896-0.899 -> 0.901 (profiles/r06/writes/exc_nt_ab.log)
        typedef uint32_t v2u __attribute__((ext_vector_type(2)));
        if (exc) __builtin_nontemporal_store(v2u{r.flags, (uint32_t)r.payload_off | ((uint32_t)r.payload_len << 16)},
                                             reinterpret_cast<v2u*>(x + slot));
    } else if (exc) {
        x[slot] = make_uint2(r.flags, (uint32_t)r.payload_off | ((uint32_t)r.payload_len << 16));
    }
    const uint32_t c1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x55, 0xF, 0xF, false);  // quad_perm 1111
    const uint32_t c2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0xAA, 0xF, 0xF, false);  // quad_perm 2222
    const uint32_t c3 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0xFF, 0xF, 0xF, false);  // quad_perm 3333
    if ((idx & 3u) == 0u && idx < a.count)
        __builtin_nontemporal_store(c | (c1 << 8) | (c2 << 16) | (c3 << 24), reinterpret_cast<uint32_t*>(codes + idx));
}

// store_sparse_coded with the code taken from the record (known: the code
// when the caller already proved the shape, the fast paths)
template <int OUT>
__device__ __forceinline__ void store_sparse(const ParseArgs& a, uint64_t idx, bool valid, const nexg_record& r,
                                             uint32_t known = 0u) {
    const uint32_t code = !valid ? 0u : known ? known : sparse_encode(r, a.opt_flags, a.ip_offset);
    store_sparse_coded<OUT>(a, idx, valid, r, code);
}

// every lane of the wave calls this together (see store_sparse)
template <int OUT>
__device__ __forceinline__ void store_out(const ParseArgs& a, uint64_t idx, bool valid, const nexg_record& r) {
    if constexpr (sparse_like(OUT)) store_sparse<OUT>(a, idx, valid, r);
    else if (valid) store_result<OUT>(a.out, idx, r);
}

// Record output of a 256-frame tile through LDS: each thread has written its
// 64-B record at stage + t * PITCH (call after a barrier); the tile's nf
// records leave as contiguous 16-B stores (1 KiB per wave instruction)
// instead of four 64-B-strided ones per thread.
template <uint32_t PITCH>
__device__ __forceinline__ void copy_out_records(const uint8_t* stage, void* out, uint64_t first, uint32_t nf) {
    uint4* dst = reinterpret_cast<uint4*>(out) + first * 4u;
    for (uint32_t c = threadIdx.x; c < nf * 4u; c += kTile)
        dst[c] = *reinterpret_cast<const uint4*>(stage + (c >> 2) * PITCH + 16u * (c & 3u));
}

// NEXG_OUT_DESC output of a tile through LDS: each thread has written its
// 8-B descriptor at the start of its PITCH-byte slot (call after a barrier);
// the tile's nf descriptors leave as contiguous 16-B non-temporal stores, two
// descriptors per thread (threads 0..127), instead of 8-B stores per thread.
// An output at 8 mod 16 (the API asks 8-B alignment) takes two 8-B stores.
template <uint32_t PITCH>
__device__ __forceinline__ void copy_out_descs(const uint8_t* stage, void* out, uint64_t first, uint32_t nf) {
    typedef uint32_t v2u __attribute__((ext_vector_type(2)));
    const uint32_t c = threadIdx.x, f = 2u * c;
    if (f >= nf) return;
    const uint2 d0 = *reinterpret_cast<const uint2*>(stage + f * PITCH);
    const bool pair = f + 1u < nf;
    const uint2 d1 = pair ? *reinterpret_cast<const uint2*>(stage + (f + 1u) * PITCH) : d0;
    if (pair && (reinterpret_cast<uint64_t>(out) & 15u) == 0) {
        __builtin_nontemporal_store(u32x4{d0.x, d0.y, d1.x, d1.y}, reinterpret_cast<u32x4*>(out) + (first + f) / 2u);
    } else {
        __builtin_nontemporal_store(v2u{d0.x, d0.y}, reinterpret_cast<v2u*>(out) + first + f);
        if (pair) __builtin_nontemporal_store(v2u{d1.x, d1.y}, reinterpret_cast<v2u*>(out) + first + f + 1u);
    }
}

__device__ __forceinline__ void stage_desc(uint8_t* slot, const nexg_record& r) {
    *reinterpret_cast<uint2*>(slot) = make_uint2(r.flags, (uint32_t)r.payload_off | ((uint32_t)r.payload_len << 16));
}

__device__ __forceinline__ void stage_record(uint8_t* slot, const nexg_record& r) {
    uint4 v[4];
    __builtin_memcpy(v, &r, sizeof(r));
#pragma unroll
    for (int k = 0; k < 4; k++) reinterpret_cast<uint4*>(slot)[k] = v[k];
}

// Offset i of the batch's table (include/nexg.h): u64 entries, or with
// NEXG_FRAMES_OFFSETS32 u32 entries, completed from the 256-frame group base
// of frame g when the batch is over 4 GiB (g = i, or for a packed frame's end
// the frame itself: its end lies within 4 GiB of its own group's base)
__device__ __forceinline__ uint64_t table_off(const ParseArgs& a, uint64_t i, uint64_t g) {
    if (!(a.hints & NEXG_FRAMES_OFFSETS32)) return NEXG_GLOBAL(uint64_t, a.offsets)[i];
    const uint32_t o = NEXG_GLOBAL(uint32_t, a.offsets)[i];
    if (!a.off_bases) return o;
    const uint64_t b = NEXG_GLOBAL(uint64_t, a.off_bases)[g >> 8];
    return b + (uint32_t)(o - (uint32_t)b);
}

// MODE 0: fixed stride tile staging (STRIDE = 0 -> runtime stride).
// MODE 1: per-lane window staging.
template <int MODE, int OUT, int STRIDE, int WIN, bool FAST = true, bool NT = false>
__global__ __launch_bounds__(256) void k_parse(ParseArgs a) {
    constexpr uint32_t PITCH = WIN + 16;
    __shared__ __attribute__((aligned(16))) uint8_t smem[kTile * PITCH];
    const uint32_t tid = threadIdx.x;
    const uint64_t first = (MODE == 0 ? tile_index(a.tile_order) : (uint64_t)blockIdx.x) * kTile;
    const uint64_t left = a.count - first;
    const uint32_t nf = left < kTile ? (uint32_t)left : kTile;
    const uint64_t idx = first + tid;
    uint8_t* slot = smem + tid * PITCH;
    const uint8_t* g = nullptr;
    uint32_t len = 0, o = 0, wlen = 0;
    bool bad = false;
    if (MODE == 0) {
        const uint32_t S = STRIDE ? (uint32_t)STRIDE : a.stride;
        const uint8_t* T = a.data + first * S;
        const uint32_t chunks = nf * (S / 16u);
        // every 16-B load of the tile issued before the first LDS write (a
        // load -> wait -> write loop keeps one load per lane in flight)
        constexpr uint32_t KMAX = (STRIDE ? (uint32_t)STRIDE : (uint32_t)WIN) / 16u;
        uint4 v[KMAX];
        if (STRIDE && nf == kTile) {  // full tile of a compile-time stride: straight line
#pragma unroll
            for (uint32_t k = 0; k < KMAX; k++) v[k] = load16<NT>(T + (uint64_t)(tid + k * kTile) * 16u);
#pragma unroll
            for (uint32_t k = 0; k < KMAX; k++) {
                const uint32_t byte = (tid + k * kTile) * 16u;
                const uint32_t f = byte / S;
                *reinterpret_cast<uint4*>(smem + f * PITCH + (byte - f * S)) = v[k];
            }
        } else {
#pragma unroll
            for (uint32_t k = 0; k < KMAX; k++) {
                const uint32_t c = tid + k * kTile;
                if (c < chunks) v[k] = load16<NT>(T + (uint64_t)c * 16u);
            }
#pragma unroll
            for (uint32_t k = 0; k < KMAX; k++) {
                const uint32_t c = tid + k * kTile;
                if (c < chunks) {
                    const uint32_t byte = c * 16u;
                    const uint32_t f = byte / S;
                    *reinterpret_cast<uint4*>(smem + f * PITCH + (byte - f * S)) = v[k];
                }
            }
        }
        __syncthreads();
        if (tid < nf) {
            g = T + (uint64_t)tid * S;
            len = a.lengths ? a.lengths[idx] : S;
            wlen = len < S ? len : S;
            bad = len > 65535u || (first + tid) * S + len > a.data_bytes;
        }
    } else {
        // SPARSE stores need every lane of the wave; other outputs leave early
        if (!sparse_like(OUT) && tid >= nf) return;
        const uint64_t off = tid < nf ? (a.offsets ? table_off(a, idx, idx) : idx * (uint64_t)a.stride) : 0u;
        const uint64_t l64 = tid >= nf ? 0u
                             : a.lengths ? (uint64_t)a.lengths[idx]
                                         : (a.offsets ? table_off(a, idx + 1, idx) - off : (uint64_t)a.stride);
        bad = l64 > 65535u || off > a.data_bytes || l64 > a.data_bytes - off;
        if (!bad && tid < nf) {
            len = (uint32_t)l64;
            g = a.data + off;
            o = (uint32_t)(reinterpret_cast<uint64_t>(g) & 15u);
            const uint8_t* A0 = g - o;
            wlen = len < (uint32_t)WIN ? len : (uint32_t)WIN;
            const uint32_t chunks = (o + wlen + 15u) >> 4;
            constexpr uint32_t KW = (uint32_t)WIN / 16u + 1u;  // window + alignment slack
            uint4 v[KW];
#pragma unroll
            for (uint32_t k = 0; k < KW; k++)  // all loads in flight before the first LDS write
                if (k < chunks) v[k] = *reinterpret_cast<const uint4*>(A0 + 16u * k);
#pragma unroll
            for (uint32_t k = 0; k < KW; k++)
                if (k < chunks) *reinterpret_cast<uint4*>(slot + 16u * k) = v[k];
        }
    }
    // MODE 0 + RECORD / DESC: every thread stays for the coalesced copy-out
    constexpr bool kStaged = MODE == 0 && OUT == NEXG_OUT_RECORD && PITCH >= 64;
    constexpr bool kPlainDesc = MODE == 0 && OUT == NEXG_OUT_DESC;  // see NEXG_DESC_MODE
    if constexpr (OUT == NEXG_OUT_SLICE) {  // FrameSlice boundaries from the same staging
        if (tid < nf) {
            nexg_slice sl;
            if (bad) {
                sl = nexg_slice{};
                sl.flags = (uint32_t)NEXG_ERR_BAD_EXTENT << NEXG_STATUS_SHIFT;
            } else {
                WinFrame f{slot, g, o, wlen};
                slice_frame(f, len, a.opt_flags, a.ip_offset, sl);
            }
            reinterpret_cast<nexg_slice*>(a.out)[idx] = sl;
        }
        return;
    }
    nexg_record r;
    bool have = false;
    if (tid < nf) {
        if (MODE == 0 && STRIDE == 64 && FAST && !bad && len == 64u) {
            // register copy of the whole frame: 4 x ds_read_b128 (pitch 80: conflict-free)
            uint32_t w[16];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint4 v = *reinterpret_cast<const uint4*>(slot + 16 * k);
                w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
            }
            have = fast_udp4_64(w, a.opt_flags, r);
        }
        if (!have) {
            if (bad) {
                r = nexg_record{};
                r.flags = (uint32_t)NEXG_ERR_BAD_EXTENT << NEXG_STATUS_SHIFT;
            } else {
                WinFrame f{slot, g, o, wlen};
                parse_frame(f, (uint32_t)(reinterpret_cast<uint64_t>(g) & 1u), len, a.opt_flags, a.ip_offset, r);
            }
        }
        if (kStaged) stage_record(slot, r);  // own slot: no other thread reads it
        else if (kPlainDesc)
            reinterpret_cast<uint2*>(a.out)[idx] =
                make_uint2(r.flags, (uint32_t)r.payload_off | ((uint32_t)r.payload_len << 16));
        else if constexpr (!sparse_like(OUT)) store_result<OUT>(a.out, idx, r);
    }
    if constexpr (sparse_like(OUT)) {
        // fast_udp4_64 proved IPv4/UDP with the datagram to the frame end (payload
        // [42, 64)): the code is the shape and the two verdicts
        const uint32_t known = have ? NEXG_SHAPE_V4_UDP | ((r.flags & NEXG_C_IP_OK) ? NEXG_SPARSE_IP_OK : 0u) |
                                          ((r.flags & NEXG_C_L4_OK) ? NEXG_SPARSE_L4_OK : 0u)
                                    : 0u;
        store_sparse<OUT>(a, idx, tid < nf, r, known);
    }
    if (kStaged) {
        __syncthreads();
        copy_out_records<PITCH>(smem, a.out, first, nf);
    }
}

// wave-scope LDS visibility: the wave's LDS ops run in order; this only stops
// the compiler from moving LDS accesses across the point
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr uint32_t kLaneWin = 80;  // register window of k_parse_lane80

// Per-frame slot the two-kernel IMIX path hands the tail sum through: the
// first 4 bytes of the frame's own output element (overwritten by pass 2).
// Outputs narrower than 4 B (verdict, sparse codes) hand off through a.tail.
template <int OUT>
__device__ __forceinline__ uint32_t* handoff_slot(const ParseArgs& a, uint64_t idx) {
    if (OUT == NEXG_OUT_VERDICT || sparse_like(OUT)) return a.tail + idx;
    return reinterpret_cast<uint32_t*>(a.out) + idx * (OUT == NEXG_OUT_FLAGS ? 1u : OUT == NEXG_OUT_DESC ? 2u : 16u);
}

// Each layout's loads in one block of uniform control flow, issued together
// (the one-expression form compiled the packed case to offsets[idx], a wait,
// then offsets[idx + 1]: two dependent round trips at every workgroup's start)
__device__ __forceinline__ bool frame_extent(const ParseArgs& a, uint64_t idx, uint64_t& off, uint32_t& len) {
    uint64_t l64;
    if (a.offsets && !a.lengths && (a.hints & NEXG_FRAMES_OFFSETS32)) {  // packed, u32 table
        const auto* op = NEXG_GLOBAL(uint32_t, a.offsets);
        const uint32_t o0 = op[idx], o1 = op[idx + 1];
        uint64_t b = 0;
        if (a.off_bases) b = NEXG_GLOBAL(uint64_t, a.off_bases)[idx >> 8];
        off = b + (uint32_t)(o0 - (uint32_t)b);
        l64 = (uint32_t)(o1 - o0);  // < 4 GiB by the table's contract
    } else if (a.offsets && !a.lengths) {  // packed: the next frame's offset ends this one
        const auto* op = NEXG_GLOBAL(uint64_t, a.offsets);
        const uint64_t o0 = op[idx], o1 = op[idx + 1];
        off = o0;
        l64 = o1 - o0;
    } else if (a.offsets && (a.hints & NEXG_FRAMES_OFFSETS32)) {
        const uint64_t o0 = table_off(a, idx, idx);
        const uint32_t l = NEXG_GLOBAL(uint32_t, a.lengths)[idx];
        off = o0;
        l64 = l;
    } else if (a.offsets) {
        const uint64_t o0 = NEXG_GLOBAL(uint64_t, a.offsets)[idx];
        const uint32_t l = NEXG_GLOBAL(uint32_t, a.lengths)[idx];
        off = o0;
        l64 = l;
    } else {
        off = idx * (uint64_t)a.stride;
        l64 = a.lengths ? (uint64_t)NEXG_GLOBAL(uint32_t, a.lengths)[idx] : (uint64_t)a.stride;
    }
    const bool bad = l64 > 65535u || off > a.data_bytes || l64 > a.data_bytes - off;
    len = bad ? 0u : (uint32_t)l64;
    return !bad;
}

// Pass 1 of the offset-table path: little-endian sum of every frame's bytes
// [80, len), streamed by quarter-waves in 256-B pieces (16 aligned 16-B chunks);
// no parse state, so registers and LDS stay small and many waves keep
// loads in flight. Result -> handoff_slot.
template <int OUT, uint32_t PU = 8>
__global__ __launch_bounds__(256) void k_tail_sums(ParseArgs a) {
    __shared__ uint32_t s_pfx[4][65];
    __shared__ uint32_t s_acc[4][64];
    __shared__ uint32_t s_ta[4][64];  // tail start relative to the wave base
    __shared__ uint32_t s_tb[4][64];  // tail end   relative to the wave base
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    uint32_t* pfx = s_pfx[wv];
    uint32_t* acc = s_acc[wv];
    uint32_t* tail_a = s_ta[wv];
    uint32_t* tail_b = s_tb[wv];
    const uint64_t wfirst = (uint64_t)blockIdx.x * kTile + 64u * wv;
    if (wfirst >= a.count) return;
    const uint64_t left = a.count - wfirst;
    const uint32_t nf = left < 64u ? (uint32_t)left : 64u;
    const uint64_t idx = wfirst + lane;
    uint32_t np = 0;
    uint64_t off = 0;
    uint32_t len = 0;
    const bool have = lane < nf && frame_extent(a, idx, off, len) && len > kLaneWin;
    // wave base: lowest 256-B aligned tail start of the wave (wave-uniform)
    uint64_t myA = have ? reinterpret_cast<uint64_t>(a.data) + off + kLaneWin : ~0ull;
    uint64_t wbase = myA;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t o2 = __shfl_xor(wbase, d, 64);
        wbase = o2 < wbase ? o2 : wbase;
    }
    wbase &= ~(uint64_t)(kPiece - 1);
    bool fits = true;
    if (have) {
        const uint64_t ra = myA - wbase, rb = ra + (len - kLaneWin);
        fits = rb < (1ull << 31);
        if (fits) {
            np = (uint32_t)(((rb - 1) / kPiece) - (ra / kPiece) + 1);
            tail_a[lane] = (uint32_t)ra;
            tail_b[lane] = (uint32_t)rb;
        }
    }
    if (!__all(fits)) {  // wave spans >2 GiB (unordered offsets): each lane sums its own tail
        if (have) *handoff_slot<OUT>(a, idx) = (uint32_t)global_le_sum(myA, myA + len - kLaneWin);
        return;
    }
    acc[lane] = 0;
    const uint32_t incl = wave_incl_scan(np);
    pfx[lane] = incl - np;
    const uint32_t total = __shfl(incl, 63, 64);
    if (lane == 63) pfx[64] = total;
    wave_lds_sync();
    const uint32_t grp = lane >> 4, gl = lane & 15u;
    const uint32_t pb = (uint32_t)((uint64_t)total * grp / 4u);
    const uint32_t pe = (uint32_t)((uint64_t)total * (grp + 1u) / 4u);
    const uint8_t* wb = reinterpret_cast<const uint8_t*>(wbase);
    if (pb < pe) {
        uint32_t lo = 0, hi = 64;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (pfx[mid] <= pb) lo = mid; else hi = mid;
        }
        uint32_t fi = lo;
        uint32_t cf = lo, ce = pfx[lo + 1];
        uint32_t ca = tail_a[lo], cb = tail_b[lo];
        uint32_t cpb = (ca & ~(kPiece - 1)) - pfx[lo] * kPiece;  // mod 2^32
        uint32_t run = 0;
        for (uint32_t p0 = pb; p0 < pe; p0 += PU) {
            uint4 v[PU];
            uint32_t C[PU], AA[PU], BB[PU], F[PU];
#pragma unroll
            for (uint32_t u = 0; u < PU; u++) {
                const uint32_t pp = p0 + u;
                while (pp < pe && pp >= ce) {
                    cf++;
                    ce = pfx[cf + 1];
                    ca = tail_a[cf];
                    cb = tail_b[cf];
                    cpb = (ca & ~(kPiece - 1)) - pfx[cf] * kPiece;
                }
                F[u] = cf;
                AA[u] = ca;
                BB[u] = cb;
                C[u] = cpb + pp * kPiece + 16u * gl;
            }
#pragma unroll
            for (uint32_t u = 0; u < PU; u++) {
                v[u] = make_uint4(0, 0, 0, 0);
                if (p0 + u < pe && C[u] < BB[u] && C[u] + 16u > AA[u]) v[u] = load16<true>(wb + C[u]);
            }
#pragma unroll
            for (uint32_t u = 0; u < PU; u++) {
                if (p0 + u >= pe) break;
                if (F[u] != fi) {
                    uint32_t s = run;
                    s += __shfl_xor(s, 8, 16);
                    s += __shfl_xor(s, 4, 16);
                    s += __shfl_xor(s, 2, 16);
                    s += __shfl_xor(s, 1, 16);
                    if (gl == 0 && s) atomicAdd(&acc[fi], s);
                    run = 0;
                    fi = F[u];
                }
                const uint32_t c = C[u], A = AA[u], B = BB[u];
                if (c < B && c + 16u > A) {
                    if (c >= A && c + 16u <= B) {
                        run += halves(v[u].x) + halves(v[u].y) + halves(v[u].z) + halves(v[u].w);
                    } else {
                        if (c + 0 < B) run += halves(v[u].x & range_mask(c + 0, A, B));
                        if (c + 4 < B) run += halves(v[u].y & range_mask(c + 4, A, B));
                        if (c + 8 < B) run += halves(v[u].z & range_mask(c + 8, A, B));
                        if (c + 12 < B) run += halves(v[u].w & range_mask(c + 12, A, B));
                    }
                }
            }
        }
        uint32_t s = run;
        s += __shfl_xor(s, 8, 16);
        s += __shfl_xor(s, 4, 16);
        s += __shfl_xor(s, 2, 16);
        s += __shfl_xor(s, 1, 16);
        if (gl == 0 && s) atomicAdd(&acc[fi], s);
    }
    wave_lds_sync();
    if (have) *handoff_slot<OUT>(a, idx) = acc[lane];
}

// Pass 2: one lane per frame. The first 80 bytes are loaded straight into
// registers (six aligned 16-B loads, dword realignment by selects) and the
// six canonical IMIX shapes finish in fast_canonical80 with the pass-1 tail
// sum; any other frame runs the generic parse_frame from HBM.
template <int OUT>
__global__ __launch_bounds__(256) void k_parse_lane80(ParseArgs a) {
    const uint64_t idx = (uint64_t)blockIdx.x * kTile + threadIdx.x;
    const bool valid = idx < a.count;
    if (!sparse_like(OUT) && !valid) return;  // sparse stores need the whole wave
    uint64_t off = 0;
    uint32_t len = 0;
    nexg_record r{};
    const bool ext = valid && frame_extent(a, idx, off, len);
    if (valid && !ext) r.flags = (uint32_t)NEXG_ERR_BAD_EXTENT << NEXG_STATUS_SHIFT;
    const uint64_t abs = reinterpret_cast<uint64_t>(a.data) + off;
    const uint64_t dend = reinterpret_cast<uint64_t>(a.data) + a.data_bytes;
    bool done = !ext;
    if (ext && abs + kLaneWin <= dend) {
        // six 16-B aligned loads cover [abs, abs + 84) at any alignment (the
        // sixth only while it still overlaps the batch bytes); realigned by
        // dword selects (q) and v_alignbyte (byte shift)
        const uint32_t tail = len > kLaneWin ? *handoff_slot<OUT>(a, idx) : 0u;
        const uint64_t a16 = abs & ~15ull;
        const uint32_t q = (uint32_t)(abs >> 2) & 3u, sh = (uint32_t)abs & 3u;
        uint32_t u[24];
#pragma unroll
        for (int k = 0; k < 6; k++) {
            const uint4 v = (k < 5 || a16 + 80u < dend) ? load16<true>(reinterpret_cast<const void*>(a16 + 16u * k))
                                                        : make_uint4(0, 0, 0, 0);
            u[4 * k] = v.x; u[4 * k + 1] = v.y; u[4 * k + 2] = v.z; u[4 * k + 3] = v.w;
        }
        uint32_t d[21];
#pragma unroll
        for (int j = 0; j < 21; j++) d[j] = q == 0 ? u[j] : q == 1 ? u[j + 1] : q == 2 ? u[j + 2] : u[j + 3];
        uint32_t w[20];  // bytes past len left in place: fast_canonical80 never reads them
#pragma unroll
        for (int k = 0; k < 20; k++) w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
        // k_tail_sums weights by absolute parity (see k_parse_span)
        done = fast_canonical80(w, len, a.opt_flags, (uint64_t)tail << (8u * (sh & 1u)), len, r);
    }
    if (!done) {
        GlobalFrame f{a.data + off};
        parse_frame(f, (uint32_t)(abs & 1u), len, a.opt_flags, a.ip_offset, r);
    }
    store_out<OUT>(a, idx, valid, r);
}

}  // namespace nexg

namespace nexg {

// ---- packed-span path (offset tables without a lengths array, any stride) ----
//
// A workgroup owns 256 consecutive frames (one per thread). Packed frames are
// contiguous, so their bytes form one span [off[f0], off[f0+256]). The span is
// streamed through LDS in 16-KiB sub-tiles with plain coalesced 16-B loads:
// every byte of the batch is fetched exactly once, by the one workgroup that
// owns it (no head/tail split). Per sub-tile the 1024 chunk
// LE-halfword sums are prefix-scanned; a frame's L4 tail sum is then the
// difference of two prefix values Q(p) = Σ_{i<p} byte_i·256^(i mod 2) taken at
// p = start+80 and p = end (ones-complement sums are linear, and 2^32 wrapping
// is exact for a ≤64-KiB frame). Each frame's head window is copied from LDS
// into registers at any byte alignment and finished by fast_canonical80; the
// frames it declines are bucketed by (family, L4 protocol) across the
// workgroup and parsed densely by the generic core on 80-B LDS slots
// (SpanFrame), their L4 sums taken from the same prefix scan.

NEXG_HD uint32_t chunk_le_sum(const uint4& v) {
    return halves_acc(v.w, halves_acc(v.z, halves_acc(v.y, halves_acc(v.x, 0u))));
}

// LE halfword sum of the first m (< 16) bytes of the 16-B LDS chunk at c
NEXG_HD uint32_t chunk_prefix_sum(const uint8_t* c, uint32_t m) {
    const uint4 v = *reinterpret_cast<const uint4*>(c);
    auto msk = [&](uint32_t d) {  // bytes [4d, m) of dword d
        return m >= 4u * d + 4u ? 0xFFFFFFFFu : (m <= 4u * d ? 0u : ((1u << (8u * (m - 4u * d))) - 1u));
    };
    return halves_acc(v.w & msk(3), halves_acc(v.z & msk(2), halves_acc(v.y & msk(1), halves(v.x & msk(0)))));
}

// little-endian halfword sum of the bytes of the 16-B chunk v at absolute
// address c that lie in [A, B)
NEXG_HD uint32_t chunk_range_sum(const uint4& v, uint64_t c, uint64_t A, uint64_t B) {
    if (c >= B || c + 16u <= A) return 0u;
    if (c >= A && c + 16u <= B) return chunk_le_sum(v);
    uint32_t s = halves(v.x & range_mask(c, A, B));
    if (c + 4 < B) s += halves(v.y & range_mask(c + 4, A, B));
    if (c + 8 < B) s += halves(v.z & range_mask(c + 8, A, B));
    if (c + 12 < B) s += halves(v.w & range_mask(c + 12, A, B));
    return s;
}

// k_parse_span's generic-pass bucket of a declined frame, from its head
// window dwords 3 (bytes 12..15) and 5 (bytes 20..23): IPv4 TCP / UDP / ICMP /
// other, IPv6 TCP / UDP / ICMPv6 / other, anything else (FROM_IP included)
constexpr uint32_t kBuckets = 9;
NEXG_HD uint32_t span_bucket(uint32_t w3, uint32_t w5, uint32_t opt_flags) {
    if (opt_flags & NEXG_PARSE_FROM_IP) return 8u;
    const uint32_t et = ((w3 & 0xFFu) << 8) | ((w3 >> 8) & 0xFFu);
    if (et == 0x0800u) {
        const uint32_t p = w5 >> 24;
        return p == 6u ? 0u : p == 17u ? 1u : p == 1u ? 2u : 3u;
    }
    if (et == 0x86DDu) {
        const uint32_t p = w5 & 0xFFu;
        return p == 6u ? 4u : p == 17u ? 5u : p == 58u ? 6u : 7u;
    }
    return 8u;
}

// inclusive wave64 scan on DPP (row_shr 1/2/4/8, row_bcast 15/31): no LDS traffic
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return v;
}

// Per-workgroup clock stamps of k_parse_span's calibration instance
// (TIMING = true, launched only by nexg_probe_span_clock; the product
// instances compile no stamp): stamps[8 * workgroup + k] = s_memtime (shader
// clock ticks of the workgroup's XCD) at k = 0 entry, 1 span check, 2 end of
// the sub-tile loop, 3 end of the fast path, 4 end of the generic section,
// 5 exit; k = 6 / 7 = s_memrealtime (100 MHz) at entry / exit. The clock a
// workgroup ran at is (t5 - t0) / (rt7 - rt6) x 100 MHz (MI355X_MICROARCH.md
// 'DVFS give-back' item 6).
#define NEXG_SPAN_STAMP(k) \
    do { if constexpr (TIMING) { if (t == 0) a.stamps[blockIdx.x * 8ull + (k)] = __builtin_amdgcn_s_memtime(); } } while (0)
#define NEXG_SPAN_RTSTAMP(k) \
    do { if constexpr (TIMING) { if (t == 0) a.stamps[blockIdx.x * 8ull + (k)] = __builtin_amdgcn_s_memrealtime(); } } while (0)

// NB = 2: sub-tile k stages into buffer k&1, so the barrier that publishes
// sub-tile k also retires every lookup into sub-tile k-2's buffer (3 barriers
// per sub-tile, ~42 KB LDS); NB = 1 (the library's): one buffer and a 4th
// barrier (~25 KB LDS, 6 workgroups per CU).
#ifndef NEXG_SPAN_NT
#define NEXG_SPAN_NT true  // sub-tile fetch cache policy (A/B builds override)
#endif
#ifndef NEXG_SPAN_PF
#define NEXG_SPAN_PF 0  // offset-table prefetch distance in same-XCD dispatches (A/B builds)
#endif
#ifndef NEXG_SPAN_DEPTH
#define NEXG_SPAN_DEPTH 1  // sub-tiles in flight beside the one being scanned (A/B builds: 2)
#endif
template <int OUT, int NB = 1, uint32_t SUB = 16384, int WPE = 1, bool TIMING = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_parse_span(ParseArgs a) {
    // each stage buffer: [96-B apron | SUB bytes | 96-B pad]; the apron holds
    // the previous sub-tile's last 96 bytes, so a head window that starts
    // there is read in the sub-tile where it ends (one gather, no straddle)
    // (after the loop the bytes become per-lane 80-B SpanFrame / record slots)
    constexpr uint32_t kStage = kApron + SUB + kApron > kTile * SpanFrame::kSlot ? kApron + SUB + kApron
                                                                                 : kTile * SpanFrame::kSlot;
    __shared__ __attribute__((aligned(16))) uint8_t s_bytes[NB][kStage];
    __shared__ __attribute__((aligned(16))) uint32_t s_pfx[NB][(SUB / 16u) + 4];  // [1024] = total
    __shared__ uint32_t s_wsum[NB][4];
    __shared__ uint64_t s_span[2];
    __shared__ uint32_t s_hist[2 * kBuckets + 1];  // generic-pass bucket counts, bases, total
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    NEXG_SPAN_RTSTAMP(6);
    NEXG_SPAN_STAMP(0);
    const uint64_t f0 = tile_index(a.tile_order) * kTile;
    const uint64_t idx = f0 + t;
    const uint32_t nf = a.count - f0 < kTile ? (uint32_t)(a.count - f0) : kTile;
    const uint64_t base = reinterpret_cast<uint64_t>(a.data);
    uint64_t off = 0;
    uint32_t len = 0;
    const bool have = t < nf;
    // NEXG_OUT_GROUPED runs as the SPARSE instance on the grouped output's
    // code / exception area (the same layout from NEXG_GROUPED_CODE_OFFSET on)
    // with every group stored mixed: head NEXG_GROUPED_TILE_RUN (the tile's
    // exceptions in one run, store_sparse_coded). A GROUPED instance of this kernel
    // ran the App. C mix 7 % slower than SPARSE on the same batch (register
    // allocation of the generic section: a spill inside its loop,
    // profiles/r05/grouped_as_sparse/)
    if (OUT == NEXG_OUT_SPARSE && a.grouped_heads && lane == 0 && have) a.grouped_heads[idx >> 6] = NEXG_GROUPED_TILE_RUN;
    if (OUT == NEXG_OUT_GROUPED && lane == 0 && have) reinterpret_cast<uint8_t*>(a.out)[idx >> 6] = 0;
#if NEXG_SPAN_PF
    // warm this XCD's L2 with the offset table of the group its workgroup
    // NEXG_SPAN_PF dispatches later will take (same XCD: block + 8 k): one
    // u64 per 64-B line of that group's 2 KiB, read now, used after the loop
    uint64_t pfv = 0;
    const uint64_t pfb = (uint64_t)blockIdx.x + 8ull * NEXG_SPAN_PF;
    if (a.offsets && !a.lengths && !(a.hints & NEXG_FRAMES_OFFSETS32) && pfb < gridDim.x && t < 33u) {
        const uint64_t pg = tile_of((uint32_t)pfb, gridDim.x, a.tile_order) * kTile + 8u * t;
        if (pg <= a.count) pfv = NEXG_GLOBAL(uint64_t, a.offsets)[pg];
    }
#endif
    const bool ok = have && frame_extent(a, idx, off, len);
    if (t == 0) s_span[0] = off;
    if (t == nf - 1) s_span[1] = off + len;
    __syncthreads();
    const uint64_t lo = s_span[0], hi = s_span[1];
    const uint64_t A0 = (base + lo) & ~15ull;
    const uint32_t span = (uint32_t)(((base + hi + 15u) & ~15ull) - A0);
    // the first sub-tile goes in flight before the group's packed check (one
    // barrier less of start-up latency); only when [lo, hi] is a plausible
    // range of the batch, so every load stays inside its 16-B blocks
    constexpr int CPT = SUB / 4096u;  // 16-B chunks per thread per sub-tile
    uint4 cur[CPT];
#if NEXG_SPAN_DEPTH == 2
    uint4 nxt[CPT];
#endif
    auto fetch = [&](uint32_t S, uint4 (&v)[CPT]) {
#pragma unroll
        for (int i = 0; i < CPT; i++) {
            const uint32_t c = S + 16u * (t + 256u * i);
            v[i] = c < span ? load16g<NEXG_SPAN_NT>(A0 + c) : make_uint4(0, 0, 0, 0);
        }
    };
    const bool plausible = hi >= lo && hi <= a.data_bytes && hi - lo <= (1ull << 30);
    if (plausible) {
        fetch(0, cur);
#if NEXG_SPAN_DEPTH == 2
        fetch(SUB, nxt);  // (chunks past the span load nothing)
#endif
    }
    // packed contract: every frame of the group lies inside [lo, hi], and the
    // span is small enough for 32-bit span-relative arithmetic
    const bool inside = !have || (ok && off >= lo && off + len <= hi);
    const bool span_ok = __syncthreads_and(inside) && plausible;
    NEXG_SPAN_STAMP(1);
    nexg_record r{};
    if (!span_ok) {  // not packed here: every lane parses its own frame from HBM
        if (have) {
            if (!ok) {
                r.flags = (uint32_t)NEXG_ERR_BAD_EXTENT << NEXG_STATUS_SHIFT;
            } else {
                GlobalFrame f{a.data + off};
                parse_frame(f, (uint32_t)((base + off) & 1u), len, a.opt_flags, a.ip_offset, r);
            }
        }
        store_out<OUT>(a, idx, have, r);
        NEXG_SPAN_STAMP(5);
        NEXG_SPAN_RTSTAMP(7);
        return;
    }
    // span-relative positions: head, tail start (head + 80), end
    const uint32_t hr = (uint32_t)(base + off - A0);
    const bool want_tail = have && len > kLaneWin;
    // every frame's head window is gathered (any byte alignment: 21 aligned
    // LDS dwords, realigned by v_alignbyte after the loop); fast_canonical80
    // itself declines FROM_IP. One generic call site below: a second parse_frame
    // instance on another branch costs 15 VGPRs (6 -> 5 waves/SIMD).
    const uint32_t sh = (uint32_t)((base + off) & 3u);
    uint32_t qa = 0, qb = 0, run = 0;
    uint32_t qend = len;  // frame-relative position of the second prefix value
    constexpr uint32_t NW = SpanFrame::kSlot / 4u + 1u;  // head window dwords (one of alignment slack)
    uint32_t u[NW];
#pragma unroll
    for (int j = 0; j < (int)NW; j++) u[j] = 0;

    uint32_t buf = 0;
    // one sub-tile: stage v (this sub-tile's chunks) into LDS, refill v with the
    // sub-tile NEXG_SPAN_DEPTH ahead, scan, gather
    auto sub_tile = [&](const uint32_t S, uint4 (&v)[CPT]) {
        uint8_t* sb = s_bytes[buf] + kApron;
        uint32_t* sp = s_pfx[buf];
        // (1) stage bytes + chunk sums, put the next sub-tile in flight. The
        // threads owning the last 6 chunks first move the previous sub-tile's
        // (NB = 1: this buffer's, before they overwrite it) into the apron.
        if (S > 0 && t >= kTile - kApron / 16u) {
            const uint8_t* prev = s_bytes[NB == 2 ? buf ^ 1u : buf] + kApron + SUB - kApron;
            *reinterpret_cast<uint4*>(sb - kApron + 16u * (t - (kTile - kApron / 16u))) =
                *reinterpret_cast<const uint4*>(prev + 16u * (t - (kTile - kApron / 16u)));
        }
#pragma unroll
        for (int i = 0; i < CPT; i++) {
            const uint32_t c = t + 256u * i;
            *reinterpret_cast<uint4*>(sb + 16u * c) = v[i];
            sp[c] = chunk_le_sum(v[i]);
        }
        const uint32_t E = S + SUB;
        if (S + NEXG_SPAN_DEPTH * SUB < span) fetch(S + NEXG_SPAN_DEPTH * SUB, v);
        __syncthreads();
        // (2) block exclusive scan of the 1024 chunk sums (4 consecutive per thread)
        uint32_t cs[CPT];
        uint32_t own = 0;
#pragma unroll
        for (int i = 0; i < CPT; i++) own += (cs[i] = sp[CPT * t + i]);
        const uint32_t incl = wave_incl_scan_dpp(own);
        if (lane == 63u) s_wsum[buf][wv] = incl;
        __syncthreads();
        const uint4 ws = *reinterpret_cast<const uint4*>(s_wsum[buf]);
        const uint32_t wbase = (wv > 0 ? ws.x : 0u) + (wv > 1 ? ws.y : 0u) + (wv > 2 ? ws.z : 0u);
        const uint32_t total = ws.x + ws.y + ws.z + ws.w;
        uint32_t ex = wbase + incl - own;
#pragma unroll
        for (int i = 0; i < CPT; i++) {
            sp[CPT * t + i] = ex;
            ex += cs[i];
        }
        if (t == 0) sp[(SUB / 16u)] = total;
        __syncthreads();
        // (3) prefix values at this sub-tile's positions, head window copy
        const bool last = E >= span;
        auto q_at = [&](uint32_t d) {  // d = position - S, 0 <= d <= SUB
            const uint32_t c = d >> 4, m = d & 15u;
            return run + sp[c] + (m ? chunk_prefix_sum(sb + 16u * c, m) : 0u);
        };
        // 84-B dword-aligned head window [dh, dh + 84): gathered exactly once,
        // in the first sub-tile that holds all of it (apron included: dh >= -80),
        // or in the last one (bytes past the span end are masked by len)
        const int dh = (int)((hr & ~3u) - S);
        constexpr int kWin = (int)SpanFrame::kSlot;
        if (have && dh >= -kWin && (dh <= (int)SUB - kWin - 4 || (last && dh < (int)SUB))) {
#pragma unroll
            for (int j = 0; j < (int)NW; j++) u[j] = *reinterpret_cast<const uint32_t*>(sb + dh + 4 * j);
            // A padded frame's L4 range ends at the IP end, not the frame end:
            // take the second prefix value there instead (at or past the window
            // end, so in this sub-tile or a later one), so SpanFrame sums that
            // range from the scan too (untagged Ethernet only).
            qend = span_tail_end(__builtin_amdgcn_alignbyte(u[4], u[3], sh),
                                 __builtin_amdgcn_alignbyte(u[5], u[4], sh), len, a.opt_flags);
        }
        const uint32_t da = hr + kLaneWin - S, db = hr + qend - S;  // wrap: < 0 -> huge
        if (want_tail && (da < SUB || (last && da == SUB))) qa = q_at(da);
        if (have && (db < SUB || (last && db == SUB))) qb = q_at(db);
        run += total;
        if (NB == 1) __syncthreads();
    };
#if NEXG_SPAN_DEPTH == 2
    // two sub-tiles in flight: the loop unrolled by two over two register sets
    // (a copy between them would wait for the loads in flight)
    static_assert(NB == 1, "depth 2 runs on one stage buffer");
    for (uint32_t S = 0; S < span; S += 2u * SUB) {
        sub_tile(S, cur);
        if (S + SUB < span) sub_tile(S + SUB, nxt);
    }
#else
    for (uint32_t S = 0; S < span; S += SUB, buf = NB == 2 ? buf ^ 1u : 0u) sub_tile(S, cur);
#endif
    if (NB == 2) __syncthreads();  // the stage buffers become per-lane slots below
#if NEXG_SPAN_PF
    if (pfv == ~0ull) s_hist[0] = 1u;  // consumes the prefetch (long returned); s_hist is rewritten below
#endif
    NEXG_SPAN_STAMP(2);
    uint8_t* const slots = &s_bytes[0][0];  // 80 B per lane from here on
    // (A) every lane: the canonical fast path on its head window
    uint32_t code = 0, key = 0;
    bool gen = false;
    const uint32_t tq = want_tail ? qb - qa : 0u;
    if (have) {
        // the realigned window; bytes past len (the next frame's) are left in
        // place: fast_canonical80 never reads them, the slot copy masks them
        uint32_t w[20];
#pragma unroll
        for (int k = 0; k < 20; k++) w[k] = __builtin_amdgcn_alignbyte(u[k + 1], u[k], sh);
        // Q weights bytes by absolute parity; fast_canonical80 wants the
        // frame-relative LE sum: x256 (mod 0xFFFF) for a frame at an odd address
        const uint64_t tail = (sh & 1u) ? (uint64_t)tq * 256u : (uint64_t)tq;
        if (fast_canonical80(w, len, a.opt_flags, tail, qend, r)) {
            if (sparse_like(OUT)) code = canonical80_code(r);
            if (OUT == NEXG_OUT_RECORD) stage_record(slots + SpanFrame::kSlot * t, r);
        } else {  // declined: the window goes to this lane's slot for pass (B), zero past len
            gen = true;
            constexpr int NS = (int)SpanFrame::kSlot / 4;
            uint32_t x[NS];
#pragma unroll
            for (int k = 0; k < NS; k++) {
                const uint32_t v = k < 20 ? w[k] : __builtin_amdgcn_alignbyte(u[k + 1], u[k], sh);
                x[k] = 4u * k < len ? (v & range_mask(4u * k, 0, len)) : 0u;
            }
            key = span_bucket(x[3], x[5], a.opt_flags);
#pragma unroll
            for (int k = 0; k < NS / 4; k++)
                reinterpret_cast<uint4*>(slots + SpanFrame::kSlot * t)[k] =
                    make_uint4(x[4 * k], x[4 * k + 1], x[4 * k + 2], x[4 * k + 3]);
        }
    }
    // (B) the declined frames of the workgroup, bucketed by (family, L4
    // protocol) and handed out densely in bucket order, so a wave runs one or
    // two generic parse paths for 64 frames instead of the union of every
    // path for the few declined lanes of each wave. Items: {span position,
    // len | tail end << 16, tail sum, owner lane} in the idle prefix buffer;
    // results go back through the owner's slot.
    NEXG_SPAN_STAMP(3);
    if (__syncthreads_or(gen)) {
        if (t < kBuckets) s_hist[t] = 0;
        __syncthreads();
        const uint32_t rank = gen ? atomicAdd(&s_hist[key], 1u) : 0u;
        __syncthreads();
        if (t == 0) {
            uint32_t acc = 0;
            for (uint32_t k = 0; k < kBuckets; k++) {
                const uint32_t c = s_hist[k];
                s_hist[kBuckets + k] = acc;
                acc += c;
            }
            s_hist[2 * kBuckets] = acc;
        }
        __syncthreads();
        uint4* const items = reinterpret_cast<uint4*>(&s_pfx[0][0]);
        if (gen) items[s_hist[kBuckets + key] + rank] = make_uint4(hr, len | qend << 16, tq, t);
        const uint32_t ngen = s_hist[2 * kBuckets];
        __syncthreads();
        const bool work = t < ngen;
        nexg_record rr{};
        SpanDeferred dfr{};
        uint32_t owner = 0, ghr = 0;
        if (work) {
            const uint4 it = items[t];
            ghr = it.x;
            owner = it.w;
            SpanFrame f{slots + SpanFrame::kSlot * owner, reinterpret_cast<const uint8_t*>(A0 + ghr), it.y >> 16,
                        ghr & 1u, it.z};
            parse_frame(f, ghr & 1u, it.y & 0xFFFFu, a.opt_flags, a.ip_offset, rr);
            dfr = f.d;
        }
        // deferred checksum ranges (SpanFrame): four at a time, one per 16-lane
        // group (row), each lane summing up to four 16-B loads in flight per
        // step (1 KiB per group, L2-hot), rows reduced by xor shuffles
        uint32_t mine = 0;
        const uint32_t grp = lane >> 4, gl = lane & 15u;
        for (uint64_t m = __ballot(dfr.which() != 0u); m;) {
            const uint64_t cur = m;
            uint64_t rest = cur;
            uint32_t pick = 64u;  // this group's deferred lane (64: none)
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) {
                const uint32_t b = rest ? (uint32_t)__builtin_ctzll(rest) : 64u;
                pick = k == grp ? b : pick;
                rest &= rest - 1;
            }
            m = rest;
            const int src = (int)(pick & 63u);
            const uint32_t rg = (uint32_t)__shfl((int)dfr.rng, src, 64);
            const uint64_t A = A0 + (uint32_t)__shfl((int)ghr, src, 64) + (rg & 0xFFFFu);
            const uint64_t B = pick < 64u ? A + (rg >> 16) : A;
            uint32_t s = 0;
            for (uint64_t c = (A & ~15ull) + 16u * gl; c < B; c += 1024u) {
                uint4 v[4];
#pragma unroll
                for (uint32_t k = 0; k < 4; k++)
                    v[k] = c + 256u * k < B ? load16(reinterpret_cast<const void*>(c + 256u * k)) : make_uint4(0, 0, 0, 0);
#pragma unroll
                for (uint32_t k = 0; k < 4; k++) s += chunk_range_sum(v[k], c + 256u * k, A, B);
            }
            s += __shfl_xor(s, 8, 16);
            s += __shfl_xor(s, 4, 16);
            s += __shfl_xor(s, 2, 16);
            s += __shfl_xor(s, 1, 16);
            const uint32_t rk = (uint32_t)__builtin_popcountll(cur & ((1ull << lane) - 1ull));
            const uint32_t tot = (uint32_t)__shfl((int)s, (int)((rk & 3u) << 4), 64);
            if (((cur >> lane) & 1ull) && rk < 4u) mine = tot;
        }
        if (dfr.which()) span_patch(dfr, mine, rr);
        if (work) {  // each slot is read and written by its one worker only
            uint8_t* os = slots + SpanFrame::kSlot * owner;
            if (OUT == NEXG_OUT_RECORD) {
                stage_record(os, rr);
            } else {
                const uint32_t c = sparse_like(OUT) ? sparse_encode(rr, a.opt_flags, a.ip_offset) : 0u;
                *reinterpret_cast<uint4*>(os) =
                    make_uint4(rr.flags, (uint32_t)rr.payload_off | ((uint32_t)rr.payload_len << 16), c, 0u);
            }
        }
        __syncthreads();
        if (gen && OUT != NEXG_OUT_RECORD) {
            const uint4 v = *reinterpret_cast<const uint4*>(slots + SpanFrame::kSlot * t);
            r.flags = v.x;
            r.payload_off = (uint16_t)v.y;
            r.payload_len = (uint16_t)(v.y >> 16);
            code = v.z;
        }
    }
    // (the span kernel's batches mix shapes: its grouped output stores every
    // group as a mixed one — head NEXG_GROUPED_TILE_RUN, stored at the start — which keeps the
    // uniformity test and the head store out of the generic section's register
    // budget: with them the App. C mix ran 10 % slower, profiles/r03/grouped)
    NEXG_SPAN_STAMP(4);
    if (sparse_like(OUT)) store_sparse_coded<OUT, false>(a, idx, have, r, code);
    else if (OUT == NEXG_OUT_DESC && NEXG_DESC_MODE == 2) {  // 256 x 8 B through the slots: 16-B NT stores
        // own slot only (the generic section's reads of other lanes' slots
        // ended at its last barrier)
        if (have) stage_desc(slots + SpanFrame::kSlot * t, r);
        __syncthreads();
        copy_out_descs<SpanFrame::kSlot>(slots, a.out, f0, nf);
    } else if (OUT != NEXG_OUT_RECORD) store_out<OUT>(a, idx, have, r);
    if (OUT == NEXG_OUT_RECORD) {  // 256 x 64 B records through the slots (pitch 80 B)
        static_assert(kStage >= kTile * SpanFrame::kSlot, "record staging needs kTile slots");
        __syncthreads();
        copy_out_records<SpanFrame::kSlot>(slots, a.out, f0, nf);
    }
    NEXG_SPAN_STAMP(5);
    NEXG_SPAN_RTSTAMP(7);
}


// (A persistent variant that prefetched the next group's first sub-tile by
// LDS-DMA was measured in round 5 and removed: every variant spilled, DESIGN.md
// §6 round 5; it is in the history at commit 2c6e6f3.)

}  // namespace nexg
