// nexg_parse.hip — batched Frame::try_from_buf + verification checksums on
// gfx950 (nex-packet/src/frame.rs:299-315, 570-658; util.rs:65-183).
//
// One lane per frame, 256-lane workgroups, one tile of 256 consecutive frames
// per workgroup. Header bytes are staged in LDS so the branchy per-protocol
// parse reads LDS, not HBM; HBM is read once, coalesced where the layout
// allows:
//   TileStride64 / TileStride : fixed-stride batches. The workgroup streams its
//       whole tile (256 x stride bytes, contiguous) with 16-B loads in lane
//       order into per-frame LDS slots, padded to break bank conflicts.
//   LaneWindow : offset-table batches (IMIX). Each lane stages the first
//       128 B of its frame (16-B aligned chunks) into its own LDS slot; bytes
//       past the window (long payloads) are summed straight from HBM.
#include "frame_core.hpp"
#include "nexg_internal.hpp"

namespace nexg {

constexpr uint32_t kTile = 256;

// Frame read entirely from HBM (checksum utility path).
struct GlobalFrame {
    const uint8_t* g;
    NEXG_HD uint32_t u8(uint32_t i) const { return g[i]; }
    NEXG_HD uint64_t le_sum(uint32_t a, uint32_t b) const {
        const uint64_t base = reinterpret_cast<uint64_t>(g);
        return global_le_sum(base + a, base + b);
    }
};

template <int OUT>
__device__ __forceinline__ void store_result(void* out, uint64_t idx, const nexg_record& r) {
    if (OUT == NEXG_OUT_DESC) {
        uint2 d = make_uint2(r.flags, (uint32_t)r.payload_off | ((uint32_t)r.payload_len << 16));
        reinterpret_cast<uint2*>(out)[idx] = d;
    } else {
        uint4 v[4];
        __builtin_memcpy(v, &r, sizeof(r));
        uint4* dst = reinterpret_cast<uint4*>(out) + idx * 4;
#pragma unroll
        for (int k = 0; k < 4; k++) dst[k] = v[k];
    }
}

// MODE 0: fixed stride tile staging (STRIDE = 0 -> runtime stride).
// MODE 1: per-lane window staging.
template <int MODE, int OUT, int STRIDE, int WIN>
__global__ __launch_bounds__(256) void k_parse(ParseArgs a) {
    constexpr uint32_t PITCH = WIN + 16;
    __shared__ __attribute__((aligned(16))) uint8_t smem[kTile * PITCH];
    const uint32_t tid = threadIdx.x;
    const uint64_t first = (uint64_t)blockIdx.x * kTile;
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
        for (uint32_t c = tid; c < chunks; c += kTile) {
            const uint4 v = *reinterpret_cast<const uint4*>(T + (uint64_t)c * 16u);
            const uint32_t byte = c * 16u;
            const uint32_t f = byte / S;
            *reinterpret_cast<uint4*>(smem + f * PITCH + (byte - f * S)) = v;
        }
        __syncthreads();
        if (tid >= nf) return;
        g = T + (uint64_t)tid * S;
        len = a.lengths ? a.lengths[idx] : S;
        wlen = len < S ? len : S;
        bad = len > 65535u || (first + tid) * S + len > a.data_bytes;
    } else {
        if (tid >= nf) return;
        const uint64_t off = a.offsets ? a.offsets[idx] : idx * (uint64_t)a.stride;
        const uint64_t l64 = a.lengths ? (uint64_t)a.lengths[idx]
                                       : (a.offsets ? a.offsets[idx + 1] - off : (uint64_t)a.stride);
        bad = l64 > 65535u || off > a.data_bytes || l64 > a.data_bytes - off;
        if (!bad) {
            len = (uint32_t)l64;
            g = a.data + off;
            o = (uint32_t)(reinterpret_cast<uint64_t>(g) & 15u);
            const uint8_t* A0 = g - o;
            wlen = len < (uint32_t)WIN ? len : (uint32_t)WIN;
            const uint32_t chunks = (o + wlen + 15u) >> 4;
            for (uint32_t k = 0; k < chunks; k++)
                *reinterpret_cast<uint4*>(slot + 16u * k) = *reinterpret_cast<const uint4*>(A0 + 16u * k);
        }
    }
    nexg_record r;
    if (bad) {
        r = nexg_record{};
        r.flags = (uint32_t)NEXG_ERR_BAD_EXTENT << NEXG_STATUS_SHIFT;
    } else {
        WinFrame f{slot, g, o, wlen};
        parse_frame(f, (uint32_t)(reinterpret_cast<uint64_t>(g) & 1u), len, a.opt_flags, a.ip_offset, r);
    }
    store_result<OUT>(a.out, idx, r);
}

// util.rs:65-71 checksum(buf, skipword) per buffer; words outside the buffer
// and the skipped word contribute nothing; empty -> 0.
__global__ __launch_bounds__(256) void k_checksum(ParseArgs a, uint32_t skipword, uint16_t* out) {
    const uint64_t idx = (uint64_t)blockIdx.x * kTile + threadIdx.x;
    if (idx >= a.count) return;
    const uint64_t off = a.offsets ? a.offsets[idx] : idx * (uint64_t)a.stride;
    const uint64_t l64 = a.lengths ? (uint64_t)a.lengths[idx]
                                   : (a.offsets ? a.offsets[idx + 1] - off : (uint64_t)a.stride);
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

ParseVariant choose_parse_variant(const ParseArgs& a) {
    const bool aligned = (reinterpret_cast<uint64_t>(a.data) & 15u) == 0;
    if (!a.offsets && aligned && a.stride % 16u == 0 && a.stride > 0 && a.stride <= 128u &&
        a.count * (uint64_t)a.stride <= a.data_bytes) {
        return a.stride == 64u ? ParseVariant::TileStride64 : ParseVariant::TileStride;
    }
    return ParseVariant::LaneWindow;
}

template <int OUT>
static hipError_t launch_parse_out(ParseVariant v, const ParseArgs& a, hipStream_t s) {
    const uint64_t blocks = (a.count + kTile - 1) / kTile;
    dim3 grid((uint32_t)blocks), block(kTile);
    switch (v) {
        case ParseVariant::TileStride64:
            hipLaunchKernelGGL((k_parse<0, OUT, 64, 64>), grid, block, 0, s, a);
            break;
        case ParseVariant::TileStride:
            hipLaunchKernelGGL((k_parse<0, OUT, 0, 128>), grid, block, 0, s, a);
            break;
        case ParseVariant::LaneWindow:
            hipLaunchKernelGGL((k_parse<1, OUT, 0, 128>), grid, block, 0, s, a);
            break;
    }
    return hipGetLastError();
}

hipError_t launch_parse(ParseVariant v, const ParseArgs& a, int out_kind, hipStream_t s) {
    if (a.count == 0) return hipSuccess;
    return out_kind == NEXG_OUT_DESC ? launch_parse_out<NEXG_OUT_DESC>(v, a, s)
                                     : launch_parse_out<NEXG_OUT_RECORD>(v, a, s);
}

hipError_t launch_checksum(const ParseArgs& a, uint32_t skipword, uint16_t* out, hipStream_t s) {
    if (a.count == 0) return hipSuccess;
    const uint64_t blocks = (a.count + kTile - 1) / kTile;
    hipLaunchKernelGGL(k_checksum, dim3((uint32_t)blocks), dim3(kTile), 0, s, a, skipword, out);
    return hipGetLastError();
}

}  // namespace nexg
