// kbench.hip — kernel microbenchmarks for the parse hot path (one process,
// interleaved variants, hipEvent timing). Frames come from the product
// generator (libnexg.so C ABI); every parse variant's output is compared
// byte-for-byte with the product kernel's.
//   build: make -C tools kbench      run: tools/kbench [frames]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../nex_amd/csrc/parse_kernels.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

using namespace nexg;

// Measured-and-rejected span kernel generation (moved out of the product
// library): kept here only for the A/B rows below.
namespace nexg {
// k_parse_span with two barriers per sub-tile instead of four (NB = 1), or
// one (NB = 2, double-buffered stage). The scan needs no exchange of chunk
// sums: chunk c = t + 256 i (the coalesced load order) sits in scan block
// b = c / 64 = 4 i + wave, whose 64 chunks are exactly one wave's i-th
// loads, so each wave scans its blocks in registers (DPP), stores the
// in-block exclusive prefixes and the block totals, and after the one
// publishing barrier a lookup adds the totals of the blocks before its
// chunk (NBLK predicated adds). NB = 2 stages sub-tile k into buffer k & 1:
// the barrier that publishes sub-tile k+1 also retires every lookup into
// sub-tile k, so buffer k & 1 is free again when sub-tile k+2 arrives.
template <int OUT, uint32_t SUB = 16384, int NB = 1, int WPE = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_parse_span2(ParseArgs a) {
    constexpr uint32_t CPT = SUB / 4096u;  // 16-B chunks per thread per sub-tile
    constexpr uint32_t NBLK = 4u * CPT;    // 64-chunk scan blocks per sub-tile
    static_assert(CPT >= 1 && SUB % 4096u == 0, "sub-tile is a multiple of 4 KiB");
    __shared__ __attribute__((aligned(16))) uint8_t s_bytes[NB][SUB];
    __shared__ __attribute__((aligned(16))) uint32_t s_pfx[NB][SUB / 16u];
    __shared__ __attribute__((aligned(16))) uint32_t s_tot[NB][NBLK];
    __shared__ uint64_t s_span[2];
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    const uint64_t f0 = (uint64_t)blockIdx.x * kTile;
    const uint64_t idx = f0 + t;
    const uint32_t nf = a.count - f0 < kTile ? (uint32_t)(a.count - f0) : kTile;
    const uint64_t base = reinterpret_cast<uint64_t>(a.data);
    uint64_t off = 0;
    uint32_t len = 0;
    const bool have = t < nf;
    const bool ok = have && frame_extent(a, idx, off, len);
    if (t == 0) s_span[0] = off;
    if (t == nf - 1) s_span[1] = off + len;
    __syncthreads();
    const uint64_t lo = s_span[0], hi = s_span[1];
    const bool inside = !have || (ok && off >= lo && off + len <= hi);
    const bool span_ok = __syncthreads_and(inside) && hi >= lo && hi - lo <= (1ull << 30);
    nexg_record r{};
    if (!span_ok) {  // not one ordered span here: every lane parses its own frame from HBM
        if (have) {
            if (!ok) {
                r.flags = (uint32_t)NEXG_ERR_BAD_EXTENT << NEXG_STATUS_SHIFT;
            } else {
                GlobalFrame f{a.data + off};
                parse_frame(f, (uint32_t)((base + off) & 1u), len, a.opt_flags, a.ip_offset, r);
            }
        }
        store_out<OUT>(a, idx, have, r);
        return;
    }
    const uint64_t A0 = (base + lo) & ~15ull;
    const uint32_t span = (uint32_t)(((base + hi + 15u) & ~15ull) - A0);
    const uint32_t hr = (uint32_t)(base + off - A0);
    const bool want_tail = have && len > kLaneWin;
    const bool fast = have && ((base + off) & 3u) == 0 && !(a.opt_flags & NEXG_PARSE_FROM_IP);
    uint32_t qa = 0, qb = 0, run = 0;
    uint32_t w[20];
#pragma unroll
    for (int j = 0; j < 20; j++) w[j] = 0;

    uint4 cur[CPT];
    auto fetch = [&](uint32_t S) {
#pragma unroll
        for (uint32_t i = 0; i < CPT; i++) {
            const uint32_t c = S + 16u * (t + 256u * i);
            cur[i] = c < span ? load16<true>(reinterpret_cast<const void*>(A0 + c)) : make_uint4(0, 0, 0, 0);
        }
    };
    fetch(0);
    uint32_t buf = 0;
    for (uint32_t S = 0; S < span; S += SUB, buf = NB == 2 ? buf ^ 1u : 0u) {
        uint8_t* sb = s_bytes[buf];
        uint32_t* sp = s_pfx[buf];
        uint32_t* st = s_tot[buf];
        // (1) stage bytes; in-block exclusive prefixes and block totals in registers
#pragma unroll
        for (uint32_t i = 0; i < CPT; i++) {
            const uint32_t c = t + 256u * i;
            *reinterpret_cast<uint4*>(sb + 16u * c) = cur[i];
            const uint32_t cs = chunk_le_sum(cur[i]);
            const uint32_t inc = wave_incl_scan_dpp(cs);
            sp[c] = inc - cs;
            if (lane == 63u) st[4u * i + wv] = inc;
        }
        const uint32_t E = S + SUB;
        if (E < span) fetch(E);
        __syncthreads();
        // (2) prefix values at this sub-tile's positions, head window copy
        // (block totals re-read from LDS as broadcasts: no registers held)
        const bool last = E >= span;
        auto q_at = [&](uint32_t d) {  // d = position - S, 0 <= d <= SUB
            const uint32_t c = d >> 4, m = d & 15u, b = c >> 6;
            uint32_t q = run;
#pragma unroll
            for (uint32_t k = 0; k < NBLK; k += 4) {
                const uint4 v = *reinterpret_cast<const uint4*>(st + k);
                q += (k < b ? v.x : 0u) + (k + 1 < b ? v.y : 0u) + (k + 2 < b ? v.z : 0u) + (k + 3 < b ? v.w : 0u);
            }
            if (c < SUB / 16u) q += sp[c] + (m ? chunk_prefix_sum(sb + 16u * c, m) : 0u);
            return q;
        };
        const uint32_t da = hr + kLaneWin - S, db = hr + len - S;  // wrap: < 0 -> huge
        if (want_tail && (da < SUB || (last && da == SUB))) qa = q_at(da);
        if (have && (db < SUB || (last && db == SUB))) qb = q_at(db);
        const uint32_t dh = hr - S;
        if (fast) {
            if (dh <= SUB - kLaneWin) {  // whole window in this sub-tile (the usual case)
#pragma unroll
                for (int j = 0; j < 20; j++) w[j] = *reinterpret_cast<const uint32_t*>(sb + dh + 4u * j);
            } else if (dh < SUB || dh + kLaneWin - 1u < kLaneWin - 1u) {  // straddles a sub-tile edge
#pragma unroll
                for (int j = 0; j < 20; j++) {
                    const uint32_t d = dh + 4u * j;
                    if (d < SUB) w[j] = *reinterpret_cast<const uint32_t*>(sb + d);
                }
            }
        }
#pragma unroll
        for (uint32_t k = 0; k < NBLK; k += 4) {
            const uint4 v = *reinterpret_cast<const uint4*>(st + k);
            run += v.x + v.y + v.z + v.w;
        }
        if (NB == 1) __syncthreads();
    }
    if (have) {
        bool done = false;
        if (fast) {
#pragma unroll
            for (int k = 0; k < 20; k++) w[k] = 4u * k < len ? (w[k] & range_mask(4u * k, 0, len)) : 0u;
            done = fast_canonical80(w, len, a.opt_flags, want_tail ? (uint32_t)(qb - qa) : 0u, len, r);
        }
        if (!done) {
            GlobalFrame f{a.data + off};
            parse_frame(f, (uint32_t)((base + off) & 1u), len, a.opt_flags, a.ip_offset, r);
        }
    }
    if (OUT != NEXG_OUT_RECORD) store_out<OUT>(a, idx, have, r);
    if (OUT == NEXG_OUT_RECORD) {  // 256 x 64 B records through the (now idle) byte buffer
        static_assert(OUT != NEXG_OUT_RECORD || NB * SUB >= kTile * 64u, "record staging needs 16 KiB");
        uint8_t* stage = &s_bytes[0][0];
        __syncthreads();  // NB = 2: the other buffer may still be read; NB = 1: already idle
        if (have) stage_record(stage + 64u * t, r);
        __syncthreads();
        copy_out_records<64>(stage, a.out, f0, nf);
    }
}

}  // namespace nexg

// 64 B in, 8 B out per frame, coalesced: the traffic ceiling of the layout
template <bool NT>
__global__ __launch_bounds__(256) void k_readpeak(const uint8_t* data, uint64_t count, uint2* out) {
    const uint64_t first = (uint64_t)blockIdx.x * 256;
    const uint4* T = reinterpret_cast<const uint4*>(data + first * 64);
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint4 v = load16<NT>(T + threadIdx.x + 256 * k);
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[first + threadIdx.x] = make_uint2(x, 0);
}

// float4 copy: read N, write N (reference point from the microarch guide)
__global__ __launch_bounds__(256) void k_copy(const uint4* in, uint4* out, uint64_t n16) {
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (; i < n16; i += stride) out[i] = in[i];
}

// LDS staging exactly as the product kernel, then a trivial per-lane reduce
__global__ __launch_bounds__(256) void k_stageonly(const uint8_t* data, uint64_t count, uint2* out) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[256 * 80];
    const uint64_t first = (uint64_t)blockIdx.x * 256;
    const uint8_t* T = data + first * 64;
    for (uint32_t c = threadIdx.x; c < 1024; c += 256) {
        const uint4 v = reinterpret_cast<const uint4*>(T)[c];
        *reinterpret_cast<uint4*>(smem + (c >> 2) * 80 + (c & 3) * 16) = v;
    }
    __syncthreads();
    uint32_t x = 0;
    for (int k = 0; k < 4; k++) {
        uint4 v = *reinterpret_cast<const uint4*>(smem + threadIdx.x * 80 + 16 * k);
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[first + threadIdx.x] = make_uint2(x, 0);
}

// one lane per frame, 4 strided 16-B loads straight from HBM (no LDS)
__global__ __launch_bounds__(256) void k_lanedirect(const uint8_t* data, uint64_t count, uint2* out,
                                                    uint32_t flags) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint4* p = reinterpret_cast<const uint4*>(data + i * 64);
    uint32_t w[16];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint4 v = p[k];
        w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
    }
    nexg_record r;
    if (!fast_udp4_64(w, flags, r)) r.flags = 0xdead;
    out[i] = make_uint2(r.flags, (uint32_t)r.payload_off | ((uint32_t)r.payload_len << 16));
}


// Ablation of k_parse_span's streaming skeleton on the same packed batch:
// LEVEL 0 = stage each 16-KiB sub-tile into LDS (+ chunk sums) with the next
// one in flight, one barrier; 1 = + the block scan and its two barriers;
// 2 = + the head-window copy and the 4th barrier. One 8-B result per frame.
template <int LEVEL>
__global__ __launch_bounds__(256) void k_span_skeleton(ParseArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t sb[16384];
    __shared__ __attribute__((aligned(16))) uint32_t sp[1028];
    __shared__ uint32_t s_wsum[4];
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    const uint64_t f0 = (uint64_t)blockIdx.x * 256;
    const uint64_t nf = a.count - f0 < 256 ? a.count - f0 : 256;
    const uint64_t base = reinterpret_cast<uint64_t>(a.data);
    const uint64_t lo = a.offsets[f0], hi = a.offsets[f0 + nf];
    const uint64_t off = t < nf ? a.offsets[f0 + t] : lo;
    const uint64_t A0 = (base + lo) & ~15ull;
    const uint32_t span = (uint32_t)(((base + hi + 15u) & ~15ull) - A0);
    const uint32_t hr = (uint32_t)(base + off - A0);
    uint4 cur[4];
    auto fetch = [&](uint32_t S) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t c = S + 16u * (t + 256u * i);
            cur[i] = c < span ? load16<true>(reinterpret_cast<const void*>(A0 + c)) : make_uint4(0, 0, 0, 0);
        }
    };
    fetch(0);
    uint32_t acc = 0, run = 0, w[20];
#pragma unroll
    for (int j = 0; j < 20; j++) w[j] = 0;
    for (uint32_t S = 0; S < span; S += 16384) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t c = t + 256u * i;
            *reinterpret_cast<uint4*>(sb + 16u * c) = cur[i];
            sp[c] = chunk_le_sum(cur[i]);
        }
        if (S + 16384 < span) fetch(S + 16384);
        __syncthreads();
        if (LEVEL >= 1) {
            uint32_t cs[4], own = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) own += (cs[i] = sp[4 * t + i]);
            const uint32_t incl = wave_incl_scan_dpp(own);
            if (lane == 63u) s_wsum[wv] = incl;
            __syncthreads();
            const uint4 ws = *reinterpret_cast<const uint4*>(s_wsum);
            uint32_t ex = (wv > 0 ? ws.x : 0u) + (wv > 1 ? ws.y : 0u) + (wv > 2 ? ws.z : 0u) + incl - own;
#pragma unroll
            for (int i = 0; i < 4; i++) { sp[4 * t + i] = ex; ex += cs[i]; }
            run += ws.x + ws.y + ws.z + ws.w;
            __syncthreads();
        } else {
            acc += sp[(t * 7u) & 1023u];
        }
        if (LEVEL >= 2) {
            const uint32_t dh = hr - S;
            if (dh <= 16384u - 80u) {
#pragma unroll
                for (int j = 0; j < 20; j++) w[j] = *reinterpret_cast<const uint32_t*>(sb + dh + 4u * j);
            }
            __syncthreads();
        } else if (LEVEL == 0) {
            __syncthreads();
        }
    }
    uint32_t x = acc ^ run;
#pragma unroll
    for (int j = 0; j < 20; j++) x ^= w[j];
    if (t < nf) reinterpret_cast<uint2*>(a.out)[f0 + t] = make_uint2(x, 0);
}

// One-shot chunk skeleton: a workgroup per 16-KiB chunk of the packed byte
// stream (all four loads per lane in flight at once), LDS staging + chunk
// sums + block scan as in k_parse_span, 8 B written per 512 B read (near the
// IMIX descriptor ratio). Premise check for a chunk-decomposed IMIX kernel.
__global__ __launch_bounds__(256) void k_chunk_skeleton(const uint8_t* data, uint64_t nchunks, uint2* out) {
    __shared__ __attribute__((aligned(16))) uint8_t sb[16384];
    __shared__ __attribute__((aligned(16))) uint32_t sp[1028];
    __shared__ uint32_t s_wsum[4];
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    const uint8_t* T = data + (uint64_t)blockIdx.x * 16384u;
    uint4 v[4];
#pragma unroll
    for (int i = 0; i < 4; i++) v[i] = load16<true>(T + 16u * (t + 256u * i));
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t c = t + 256u * i;
        *reinterpret_cast<uint4*>(sb + 16u * c) = v[i];
        sp[c] = chunk_le_sum(v[i]);
    }
    __syncthreads();
    uint32_t cs[4], own = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) own += (cs[i] = sp[4 * t + i]);
    const uint32_t incl = wave_incl_scan_dpp(own);
    if (lane == 63u) s_wsum[wv] = incl;
    __syncthreads();
    const uint4 ws = *reinterpret_cast<const uint4*>(s_wsum);
    uint32_t ex = (wv > 0 ? ws.x : 0u) + (wv > 1 ? ws.y : 0u) + (wv > 2 ? ws.z : 0u) + incl - own;
#pragma unroll
    for (int i = 0; i < 4; i++) { sp[4 * t + i] = ex; ex += cs[i]; }
    __syncthreads();
    if (t < 32) {  // 32 results x 8 B per 16 KiB (the caller's out holds nchunks x 32)
        uint32_t x = sp[(t * 32u) & 1023u];
#pragma unroll
        for (int j = 0; j < 20; j++) x ^= *reinterpret_cast<const uint32_t*>(sb + 512u * t + 4u * j);
        out[(uint64_t)blockIdx.x * 32 + t] = make_uint2(x, 0);
    }
}

struct Var {
    std::string name;
    std::function<void()> run;
    double bytes;  // algorithmic bytes per launch
    std::vector<float> ms;
};

int main(int argc, char** argv) {
    const uint64_t count = argc > 1 ? strtoull(argv[1], nullptr, 0) : (16ull << 20);
    const int reps = 20, rounds = 7;
    nexg_ctx* ctx;
    if (nexg_ctx_create(0, &ctx) != 0) { printf("ctx failed\n"); return 1; }
    uint8_t* data;
    uint2 *out, *ref;
    uint4* cpy;
    void* rec;
    CK(hipMalloc(&data, count * 64));
    CK(hipMalloc(&out, count * 8));
    CK(hipMalloc(&ref, count * 8));
    CK(hipMalloc(&cpy, count * 64));
    CK(hipMalloc(&rec, count * 64));
    if (nexg_gen_frames(ctx, 1, 0x6E6578, 0, count, data, nullptr, 64, nullptr) != 0) return 1;
    CK(hipDeviceSynchronize());
    ParseArgs a{};
    a.data = data; a.data_bytes = count * 64; a.stride = 64; a.count = count; a.out = out;
    const dim3 grid((uint32_t)(count / 256)), blk(256);
    std::vector<Var> vars;
    auto parse = [&](auto kern) { return [=]() { hipLaunchKernelGGL(kern, grid, blk, 0, 0, a); }; };
    vars.push_back({"prod_fast", parse(k_parse<0, NEXG_OUT_DESC, 64, 64, true, false>), count * 64.0});
    vars.push_back({"prod_fast_nt", parse(k_parse<0, NEXG_OUT_DESC, 64, 64, true, true>), count * 64.0});
    vars.push_back({"flags_fast_nt", parse(k_parse<0, NEXG_OUT_FLAGS, 64, 64, true, true>), count * 64.0});
    vars.push_back({"verdict_fast_nt", parse(k_parse<0, NEXG_OUT_VERDICT, 64, 64, true, true>), count * 64.0});
    uint8_t* sparse_out;
    CK(hipMalloc(&sparse_out, NEXG_SPARSE_BYTES(count)));
    {
        ParseArgs sa = a;
        sa.out = sparse_out;
        vars.push_back({"sparse_fast_nt", [=]() { hipLaunchKernelGGL((k_parse<0, NEXG_OUT_SPARSE, 64, 64, true, true>), grid, blk, 0, 0, sa); }, count * 64.0});
    }
    vars.push_back({"prod_generic", parse(k_parse<0, NEXG_OUT_DESC, 64, 64, false, false>), count * 64.0});
    vars.push_back({"span_udp64_nb2", parse(k_parse_span<NEXG_OUT_DESC, 2>), count * 64.0});
    vars.push_back({"span_udp64_nb1", parse(k_parse_span<NEXG_OUT_DESC, 1>), count * 64.0});
    vars.push_back({"lanewindow_generic", parse(k_parse<1, NEXG_OUT_DESC, 0, 128, false, false>), count * 64.0});
    vars.push_back({"lane_direct_fast", [=]() { hipLaunchKernelGGL(k_lanedirect, grid, blk, 0, 0, data, count, out, 0u); }, count * 64.0});
    vars.push_back({"stage_only", [=]() { hipLaunchKernelGGL(k_stageonly, grid, blk, 0, 0, data, count, out); }, count * 64.0});
    vars.push_back({"readpeak", [=]() { hipLaunchKernelGGL(k_readpeak<false>, grid, blk, 0, 0, data, count, out); }, count * 64.0});
    vars.push_back({"readpeak_nt", [=]() { hipLaunchKernelGGL(k_readpeak<true>, grid, blk, 0, 0, data, count, out); }, count * 64.0});
    vars.push_back({"copy_float4", [=]() { hipLaunchKernelGGL(k_copy, dim3(256 * 32), blk, 0, 0, (const uint4*)data, cpy, count * 4); }, count * 128.0});

    // correctness of parse variants vs the product kernel (full descriptors)
    hipLaunchKernelGGL((k_parse<0, NEXG_OUT_DESC, 64, 64, false, false>), grid, blk, 0, 0, ParseArgs{data, count * 64, nullptr, nullptr, 64, count, 0, 0, ref});
    CK(hipDeviceSynchronize());
    std::vector<uint2> h_ref(count), h_out(count);
    CK(hipMemcpy(h_ref.data(), ref, count * 8, hipMemcpyDeviceToHost));
    for (auto& v : vars) {
        if (v.name.rfind("prod", 0) != 0 && v.name.rfind("lane", 0) != 0 && v.name.rfind("span", 0) != 0) continue;
        if (v.name.find("flags") != std::string::npos) continue;  // 4-B output, not comparable
        CK(hipMemset(out, 0, count * 8));
        v.run();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h_out.data(), out, count * 8, hipMemcpyDeviceToHost));
        uint64_t bad = 0;
        for (uint64_t i = 0; i < count; i++) bad += memcmp(&h_out[i], &h_ref[i], 8) != 0;
        printf("check %-20s mismatches=%llu\n", v.name.c_str(), (unsigned long long)bad);
    }
    {  // sparse codes expand (nexg_sparse_expand) to exactly the product descriptors
        CK(hipMemset(out, 0, count * 8));
        ParseArgs sa = a;
        sa.out = sparse_out;
        hipLaunchKernelGGL((k_parse<0, NEXG_OUT_SPARSE, 64, 64, true, true>), grid, blk, 0, 0, sa);
        nexg_frames fr{data, count * 64, nullptr, nullptr, 64, 0, count};
        if (nexg_sparse_expand(ctx, &fr, nullptr, sparse_out, reinterpret_cast<nexg_desc*>(out), nullptr) != 0) return 1;
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h_out.data(), out, count * 8, hipMemcpyDeviceToHost));
        uint64_t bad = 0;
        for (uint64_t i = 0; i < count; i++) bad += memcmp(&h_out[i], &h_ref[i], 8) != 0;
        printf("check %-20s mismatches=%llu\n", "sparse_fast_nt", (unsigned long long)bad);
    }
    // ---- IMIX (offset table) ----
    const uint64_t icount = count;
    uint32_t* ilen;
    uint64_t* ioff;
    CK(hipMalloc(&ilen, icount * 4));
    CK(hipMalloc(&ioff, (icount + 1) * 8));
    if (nexg_gen_lengths(ctx, 2, 0x6E6578, 0, icount, ilen, nullptr) != 0) return 1;
    std::vector<uint32_t> hl(icount);
    std::vector<uint64_t> ho(icount + 1, 0);
    CK(hipMemcpy(hl.data(), ilen, icount * 4, hipMemcpyDeviceToHost));
    for (uint64_t i = 0; i < icount; i++) ho[i + 1] = ho[i] + hl[i];
    CK(hipMemcpy(ioff, ho.data(), (icount + 1) * 8, hipMemcpyHostToDevice));
    uint8_t* idata;
    CK(hipMalloc(&idata, ho[icount] + 64));
    if (nexg_gen_frames(ctx, 2, 0x6E6578, 0, icount, idata, ioff, 0, nullptr) != 0) return 1;
    CK(hipDeviceSynchronize());
    ParseArgs ia{};
    ia.data = idata; ia.data_bytes = ho[icount]; ia.offsets = ioff; ia.count = icount; ia.out = out;
    const double ibytes = (double)ho[icount];
    auto iparse = [&](auto kern) { return [=]() { hipLaunchKernelGGL(kern, grid, blk, 0, 0, ia); }; };
    std::vector<Var> ivars;
    ivars.push_back({"imix_2pass_u4", [=]() {
        hipLaunchKernelGGL((k_tail_sums<NEXG_OUT_DESC, 4>), grid, blk, 0, 0, ia);
        hipLaunchKernelGGL(k_parse_lane80<NEXG_OUT_DESC>, grid, blk, 0, 0, ia); }, ibytes});
    ivars.push_back({"imix_span_nb2", iparse(k_parse_span<NEXG_OUT_DESC, 2>), ibytes});
    ivars.push_back({"imix_flags_span_nb1", iparse(k_parse_span<NEXG_OUT_FLAGS, 1>), ibytes});
    ivars.push_back({"imix_span_nb1", iparse(k_parse_span<NEXG_OUT_DESC, 1>), ibytes});
    ivars.push_back({"imix_span2_16k", iparse(k_parse_span2<NEXG_OUT_DESC, 16384, 1>), ibytes});
    ivars.push_back({"imix_span2_16k_w6", iparse(k_parse_span2<NEXG_OUT_DESC, 16384, 1, 6>), ibytes});
    ivars.push_back({"imix_span2_8k_nb2", iparse(k_parse_span2<NEXG_OUT_DESC, 8192, 2>), ibytes});
    ivars.push_back({"imix_span2_8k_nb1", iparse(k_parse_span2<NEXG_OUT_DESC, 8192, 1>), ibytes});
    ivars.push_back({"imix_span2_12k_nb1", iparse(k_parse_span2<NEXG_OUT_DESC, 12288, 1>), ibytes});
    {
        ParseArgs sa = ia;
        sa.out = sparse_out;
        ivars.push_back({"imix_sparse_span2_16k", [=]() { hipLaunchKernelGGL((k_parse_span2<NEXG_OUT_SPARSE, 16384, 1>), grid, blk, 0, 0, sa); }, ibytes});
        ivars.push_back({"imix_sparse_span2_8k_nb2", [=]() { hipLaunchKernelGGL((k_parse_span2<NEXG_OUT_SPARSE, 8192, 2>), grid, blk, 0, 0, sa); }, ibytes});
        ivars.push_back({"imix_sparse_span_v1", [=]() { hipLaunchKernelGGL((k_parse_span<NEXG_OUT_SPARSE, 1>), grid, blk, 0, 0, sa); }, ibytes});
        ivars.push_back({"imix_sparse_span_v1_w7", [=]() { hipLaunchKernelGGL((k_parse_span<NEXG_OUT_SPARSE, 1, 16384, 7>), grid, blk, 0, 0, sa); }, ibytes});
        ivars.push_back({"imix_sparse_span_v1_w6", [=]() { hipLaunchKernelGGL((k_parse_span<NEXG_OUT_SPARSE, 1, 16384, 6>), grid, blk, 0, 0, sa); }, ibytes});
        // larger sub-tiles: more bytes in flight per workgroup, fewer workgroups per CU
        ivars.push_back({"imix_sparse_span_20k_w6", [=]() { hipLaunchKernelGGL((k_parse_span<NEXG_OUT_SPARSE, 1, 20480, 6>), grid, blk, 0, 0, sa); }, ibytes});
        ivars.push_back({"imix_sparse_span_20k_w5", [=]() { hipLaunchKernelGGL((k_parse_span<NEXG_OUT_SPARSE, 1, 20480, 5>), grid, blk, 0, 0, sa); }, ibytes});
        ivars.push_back({"imix_sparse_span_24k_w5", [=]() { hipLaunchKernelGGL((k_parse_span<NEXG_OUT_SPARSE, 1, 24576, 5>), grid, blk, 0, 0, sa); }, ibytes});
        ivars.push_back({"imix_sparse_span_24k_w4", [=]() { hipLaunchKernelGGL((k_parse_span<NEXG_OUT_SPARSE, 1, 24576, 4>), grid, blk, 0, 0, sa); }, ibytes});
        ivars.push_back({"imix_sparse_span_28k_w5", [=]() { hipLaunchKernelGGL((k_parse_span<NEXG_OUT_SPARSE, 1, 28672, 5>), grid, blk, 0, 0, sa); }, ibytes});
        ivars.push_back({"imix_sparse_span_32k_w4", [=]() { hipLaunchKernelGGL((k_parse_span<NEXG_OUT_SPARSE, 1, 32768, 4>), grid, blk, 0, 0, sa); }, ibytes});
        ivars.push_back({"imix_sparse_span_32k_w5", [=]() { hipLaunchKernelGGL((k_parse_span<NEXG_OUT_SPARSE, 1, 32768, 5>), grid, blk, 0, 0, sa); }, ibytes});
        ivars.push_back({"imix_desc_span_20k_w6", [=]() { hipLaunchKernelGGL((k_parse_span<NEXG_OUT_DESC, 1, 20480, 6>), grid, blk, 0, 0, ia); }, ibytes});
        ivars.push_back({"imix_desc_span_16k_w6", [=]() { hipLaunchKernelGGL((k_parse_span<NEXG_OUT_DESC, 1, 16384, 6>), grid, blk, 0, 0, ia); }, ibytes});
    }
    ivars.push_back({"imix_span_nb1_8k", iparse(k_parse_span<NEXG_OUT_DESC, 1, 8192>), ibytes});
    ivars.push_back({"imix_span_nb2_8k", iparse(k_parse_span<NEXG_OUT_DESC, 2, 8192>), ibytes});
    ivars.push_back({"imix_span_nb1_32k", iparse(k_parse_span<NEXG_OUT_DESC, 1, 32768>), ibytes});
    ivars.push_back({"imix_span_rec", [=]() {
        ParseArgs r2 = ia; r2.out = rec;
        hipLaunchKernelGGL((k_parse_span<NEXG_OUT_RECORD, 1>), grid, blk, 0, 0, r2); }, ibytes});
    ivars.push_back({"ABL_span_stage", iparse(k_span_skeleton<0>), ibytes});
    ivars.push_back({"ABL_span_stage_scan", iparse(k_span_skeleton<1>), ibytes});
    ivars.push_back({"ABL_span_stage_scan_head", iparse(k_span_skeleton<2>), ibytes});
    ivars.push_back({"ABL_chunk_oneshot", [=]() { hipLaunchKernelGGL(k_chunk_skeleton, dim3((uint32_t)(ho[icount] / 16384)), blk, 0, 0, idata, ho[icount] / 16384, out); }, (double)(ho[icount] / 16384 * 16384)});
    ivars.push_back({"ABL_tails_only_u4", [=]() { hipLaunchKernelGGL((k_tail_sums<NEXG_OUT_DESC, 4>), grid, blk, 0, 0, ia); }, ibytes});
    ivars.push_back({"ABL_lane80_only", [=]() { hipLaunchKernelGGL(k_parse_lane80<NEXG_OUT_DESC>, grid, blk, 0, 0, ia); }, ibytes});
    hipLaunchKernelGGL((k_parse<1, NEXG_OUT_DESC, 0, 128>), grid, blk, 0, 0, ParseArgs{idata, ho[icount], ioff, nullptr, 0, icount, 0, 0, ref});
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h_ref.data(), ref, count * 8, hipMemcpyDeviceToHost));
    for (auto& v : ivars) {
        if (v.name.rfind("ABL", 0) == 0 || v.name.rfind("udp64", 0) == 0 || v.name.find("_rec") != std::string::npos ||
            v.name.find("flags") != std::string::npos) continue;
        if (v.name.find("sparse") != std::string::npos) {  // codes -> nexg_sparse_expand -> descriptors
            nexg_frames fr{idata, ho[icount], ioff, nullptr, 0, 0, icount};
            CK(hipMemset(out, 0, count * 8));
            v.run();
            if (nexg_sparse_expand(ctx, &fr, nullptr, sparse_out, reinterpret_cast<nexg_desc*>(out), nullptr) != 0) return 1;
        } else {
            CK(hipMemset(out, 0, count * 8));
            v.run();
        }
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h_out.data(), out, count * 8, hipMemcpyDeviceToHost));
        uint64_t bad = 0;
        for (uint64_t i = 0; i < count; i++) bad += memcmp(&h_out[i], &h_ref[i], 8) != 0;
        printf("check %-20s mismatches=%llu\n", v.name.c_str(), (unsigned long long)bad);
    }
    for (auto& v : ivars) vars.push_back(v);
    printf("imix bytes %.3f GB, mean frame %.1f B\n", ibytes / 1e9, ibytes / icount);

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; r++) {
        for (auto& v : vars) {
            v.run();
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < reps; i++) v.run();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            v.ms.push_back(ms / reps);
        }
    }
    printf("%-22s %10s %10s %10s %8s\n", "variant", "med_us", "min_us", "GB/s(med)", "frac8T");
    for (auto& v : vars) {
        std::sort(v.ms.begin(), v.ms.end());
        double med = v.ms[v.ms.size() / 2];
        double gbs = v.bytes / (med * 1e-3) / 1e9;
        printf("%-22s %10.1f %10.1f %10.1f %8.3f\n", v.name.c_str(), med * 1e3, v.ms[0] * 1e3, gbs, gbs / 8000.0);
    }
    return 0;
}
