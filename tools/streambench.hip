// streambench.hip — read-stream ceiling for the 64-B-in / 8-B-out layout
// (the UDP64 parse's traffic shape) under different kernel structures.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <functional>
#include <memory>
#include <string>
#include <vector>
#include "../nex_amd/csrc/frame_core.hpp"
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
using namespace nexg;

// L = 16-B loads per thread; tile = 256*L*16 bytes per block, one-shot grid
template <int L, bool NT>
__global__ __launch_bounds__(256) void k_rp(const uint8_t* data, uint64_t n16, uint2* out) {
    const uint64_t base = (uint64_t)blockIdx.x * 256 * L;
    uint32_t x = 0;
    uint4 v[L];
#pragma unroll
    for (int k = 0; k < L; k++) v[k] = load16<NT>(data + 16 * (base + threadIdx.x + 256 * k));
#pragma unroll
    for (int k = 0; k < L; k++) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    // 8 B per 64 B read, coalesced
    uint2* o = out + (base / 4);
#pragma unroll
    for (int k = 0; k < L / 4; k++) o[threadIdx.x + 256 * k] = make_uint2(x, k);
}

// read only: the output is written only on an impossible value (pure read ceiling)
template <int L>
__global__ __launch_bounds__(256) void k_ro(const uint8_t* data, uint64_t n16, uint2* out) {
    const uint64_t base = (uint64_t)blockIdx.x * 256 * L;
    uint32_t x = 0;
    uint4 v[L];
#pragma unroll
    for (int k = 0; k < L; k++) v[k] = load16<true>(data + 16 * (base + threadIdx.x + 256 * k));
#pragma unroll
    for (int k = 0; k < L; k++) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    if (x == 0x9e3779b9u) out[threadIdx.x] = make_uint2(x, 0);
}

// write-side variants of k_rp<4,true>: W = bytes written per 64-B frame
// (8, 4, 1), SP = store policy (0 plain, 1 nt, 2 sc0 sc1 nt)
typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
template <int W, int SP>
__global__ __launch_bounds__(256) void k_wv(const uint8_t* data, uint64_t n16, uint8_t* out) {
    const uint64_t base = (uint64_t)blockIdx.x * 1024;
    uint32_t x = 0;
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = load16<true>(data + 16 * (base + threadIdx.x + 256 * k));
#pragma unroll
    for (int k = 0; k < 4; k++) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    const uint64_t fr = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (W == 8) {
        u32x2v d = {x, (uint32_t)fr};
        u32x2v* o = reinterpret_cast<u32x2v*>(out) + fr;
        if (SP == 0) *o = d;
        else if (SP == 1) __builtin_nontemporal_store(d, o);
        else asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1 nt" :: "v"(o), "v"(d) : "memory");
    } else if (W == 4) {
        uint32_t* o = reinterpret_cast<uint32_t*>(out) + fr;
        if (SP == 0) *o = x;
        else __builtin_nontemporal_store(x, o);
    } else {
        // 1 B per frame: 4 frames per dword via a lane shuffle, 64 B per wave
        uint32_t b = x & 0xff;
        uint32_t b1 = __shfl_down(b, 1, 64), b2 = __shfl_down(b, 2, 64), b3 = __shfl_down(b, 3, 64);
        if ((threadIdx.x & 3) == 0) {
            uint32_t* o = reinterpret_cast<uint32_t*>(out) + fr / 4;
            const uint32_t w = b | (b1 << 8) | (b2 << 16) | (b3 << 24);
            if (SP == 0) *o = w; else __builtin_nontemporal_store(w, o);
        }
    }
}

// 64 B read + 64 B written per frame (the record output's shape), store policy
template <bool NTS>
__global__ __launch_bounds__(256) void k_rec(const uint8_t* data, uint64_t n16, uint8_t* out) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const uint64_t base = (uint64_t)blockIdx.x * 1024;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint64_t c = base + threadIdx.x + 256 * k;
        uint4 v = load16<true>(data + 16 * c);
        v.x ^= 0x9e3779b9u;
        v4u w = {v.x, v.y, v.z, v.w};
        if (NTS) __builtin_nontemporal_store(w, reinterpret_cast<v4u*>(out) + c);
        else reinterpret_cast<v4u*>(out)[c] = w;
    }
}

// 8 B per frame as 16-B non-temporal stores by half the lanes (through LDS)
__global__ __launch_bounds__(256) void k_wv16nt(const uint8_t* data, uint64_t n16, uint8_t* out) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) uint2 s_d[256];
    const uint64_t base = (uint64_t)blockIdx.x * 1024;
    uint32_t x = 0;
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = load16<true>(data + 16 * (base + threadIdx.x + 256 * k));
#pragma unroll
    for (int k = 0; k < 4; k++) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    s_d[threadIdx.x] = make_uint2(x, (uint32_t)(blockIdx.x * 256 + threadIdx.x));
    __syncthreads();
    if (threadIdx.x < 128) {
        const uint4 d = reinterpret_cast<const uint4*>(s_d)[threadIdx.x];
        v4u w = {d.x, d.y, d.z, d.w};
        __builtin_nontemporal_store(w, reinterpret_cast<v4u*>(out) + (uint64_t)blockIdx.x * 128 + threadIdx.x);
    }
}

// 8 B per 64-B frame written as 16-B stores by half the lanes (through LDS)
__global__ __launch_bounds__(256) void k_wv16(const uint8_t* data, uint64_t n16, uint8_t* out) {
    __shared__ __attribute__((aligned(16))) uint2 s_d[256];
    const uint64_t base = (uint64_t)blockIdx.x * 1024;
    uint32_t x = 0;
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = load16<true>(data + 16 * (base + threadIdx.x + 256 * k));
#pragma unroll
    for (int k = 0; k < 4; k++) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    const uint64_t fr = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    s_d[threadIdx.x] = make_uint2(x, (uint32_t)fr);
    __syncthreads();
    if (threadIdx.x < 128)
        reinterpret_cast<uint4*>(out)[(uint64_t)blockIdx.x * 128 + threadIdx.x] =
            reinterpret_cast<const uint4*>(s_d)[threadIdx.x];
}

// descriptor stream into a small wrapping output window (wmask + 1 entries):
// are writes that stay cache-resident cheaper than writes that reach HBM?
__global__ __launch_bounds__(256) void k_wwin(const uint8_t* data, uint64_t n16, uint2* out, uint64_t wmask) {
    const uint64_t base = (uint64_t)blockIdx.x * 1024;
    uint32_t x = 0;
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = load16<true>(data + 16 * (base + threadIdx.x + 256 * k));
#pragma unroll
    for (int k = 0; k < 4; k++) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    const uint64_t fr = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    out[fr & wmask] = make_uint2(x, (uint32_t)fr);
}

// T tiles per workgroup, the T descriptor blocks written together at the end
template <int T>
__global__ __launch_bounds__(256) void k_wbatch(const uint8_t* data, uint64_t n16, uint2* out) {
    const uint64_t base = (uint64_t)blockIdx.x * 1024 * T;
    uint32_t x[T];
#pragma unroll
    for (int tt = 0; tt < T; tt++) {
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = load16<true>(data + 16 * (base + 1024ull * tt + threadIdx.x + 256 * k));
        x[tt] = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) x[tt] ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
#pragma unroll
    for (int tt = 0; tt < T; tt++) out[base / 4 + 256 * tt + threadIdx.x] = make_uint2(x[tt], tt);
}

// persistent: grid-stride over tiles of 1024 chunks, software prefetch of the next tile
__global__ __launch_bounds__(256) void k_rp_persist(const uint8_t* data, uint64_t ntiles, uint2* out) {
    uint4 cur[4], nxt[4];
    uint64_t t = blockIdx.x;
    if (t >= ntiles) return;
#pragma unroll
    for (int k = 0; k < 4; k++) cur[k] = load16<true>(data + 16 * (t * 1024 + threadIdx.x + 256 * k));
    for (; t < ntiles; t += gridDim.x) {
        const uint64_t tn = t + gridDim.x;
        if (tn < ntiles) {
#pragma unroll
            for (int k = 0; k < 4; k++) nxt[k] = load16<true>(data + 16 * (tn * 1024 + threadIdx.x + 256 * k));
        }
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) x ^= cur[k].x ^ cur[k].y ^ cur[k].z ^ cur[k].w;
        out[t * 256 + threadIdx.x] = make_uint2(x, 0);
#pragma unroll
        for (int k = 0; k < 4; k++) cur[k] = nxt[k];
    }
}

// LDS-DMA: global_load_lds_dwordx4 (1 KiB per wave instruction) into LDS, then read back
__global__ __launch_bounds__(256) void k_rp_ldsdma(const uint8_t* data, uint64_t n16, uint2* out) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[16384];
    const uint64_t base = (uint64_t)blockIdx.x * 1024;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t chunk = wave * 256 + k * 64;  // this wave's 4 KB, 1 KB per instruction
        __builtin_amdgcn_global_load_lds(
            reinterpret_cast<const void*>(data + 16 * (base + chunk + lane)),
            (__attribute__((address_space(3))) void*)(smem + 16 * chunk), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint4 v = *reinterpret_cast<const uint4*>(smem + 64 * threadIdx.x + 16 * ((k + (threadIdx.x >> 2)) & 3));
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[blockIdx.x * 256 + threadIdx.x] = make_uint2(x, 0);
}


// LDS-DMA ring, wave-private: each wave keeps R slots of 4 KiB (64 x 64 B) in
// flight via global_load_lds_dwordx4 (nt) and consumes them in order.
template <int R, int WPB>
__global__ __launch_bounds__(64 * WPB) void k_rp_ring(const uint8_t* data, uint64_t nunits, uint2* out) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[WPB * R * 4096];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint8_t* ring = smem + wave * R * 4096;
    const uint64_t gw = (uint64_t)blockIdx.x * WPB + wave, nw = (uint64_t)gridDim.x * WPB;
    // contiguous range of units per wave
    const uint64_t per = (nunits + nw - 1) / nw;
    const uint64_t u0 = gw * per, u1 = u0 + per < nunits ? u0 + per : nunits;
    if (u0 >= u1) return;
    auto issue = [&](uint64_t u, int slot) {
        const uint8_t* src = data + u * 4096;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            // LDS image: frame f (=lane) chunk c stored at 64 f + 16 c; instruction k
            // covers frames 16k..16k+15 -> lane l writes LDS 1024 k + 16 l
            const uint32_t f = 16 * k + (lane >> 2), c = lane & 3;
            __builtin_amdgcn_global_load_lds(
                reinterpret_cast<const void*>(src + 64 * f + 16 * c),
                (__attribute__((address_space(3))) void*)(ring + slot * 4096 + 1024 * k), 16, 0, 2);
        }
    };
    uint64_t u = u0;
    for (int i = 0; i < R; i++)
        if (u0 + i < u1) issue(u0 + i, i);
    int slot = 0;
    for (; u < u1; u++) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (R - 1)) : "memory");
        uint32_t x = 0;
        {
            // opaque LDS reads: keeps the compiler from draining vmcnt before them
            const uint32_t a = (uint32_t)(uintptr_t)(ring + slot * 4096 + 64 * lane);
            const uint32_t r = 16 * ((lane >> 2) & 3);
            const uint32_t a0 = a + r, a1 = a + ((r + 16) & 63), a2 = a + ((r + 32) & 63), a3 = a + ((r + 48) & 63);
            u32x4 v0, v1, v2, v3;
            asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %5\n\tds_read_b128 %2, %6\n\tds_read_b128 %3, %7\n\ts_waitcnt lgkmcnt(0)"
                         : "=v"(v0), "=v"(v1), "=v"(v2), "=v"(v3)
                         : "v"(a0), "v"(a1), "v"(a2), "v"(a3) : "memory");
            x = v0.x ^ v0.y ^ v0.z ^ v0.w ^ v1.x ^ v1.y ^ v1.z ^ v1.w ^ v2.x ^ v2.y ^ v2.z ^ v2.w ^ v3.x ^ v3.y ^ v3.z ^ v3.w;
        }
        out[u * 64 + lane] = make_uint2(x, 0);
        if (u + R < u1) issue(u + R, slot);
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain: keeps the count exact at the tail
        slot = slot + 1 == R ? 0 : slot + 1;
    }
}


// each workgroup streams T consecutive 16-KiB tiles, next tile prefetched into registers
template <int T>
__global__ __launch_bounds__(256) void k_rp_multi(const uint8_t* data, uint64_t n16, uint2* out) {
    const uint64_t base = (uint64_t)blockIdx.x * 1024 * T;
    uint4 cur[4], nxt[4];
#pragma unroll
    for (int k = 0; k < 4; k++) cur[k] = load16<true>(data + 16 * (base + threadIdx.x + 256 * k));
    for (int tt = 0; tt < T; tt++) {
        const uint64_t b = base + 1024ull * tt;
        if (tt + 1 < T) {
#pragma unroll
            for (int k = 0; k < 4; k++) nxt[k] = load16<true>(data + 16 * (b + 1024 + threadIdx.x + 256 * k));
        }
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) x ^= cur[k].x ^ cur[k].y ^ cur[k].z ^ cur[k].w;
        out[b / 4 + threadIdx.x] = make_uint2(x, 0);
#pragma unroll
        for (int k = 0; k < 4; k++) cur[k] = nxt[k];
    }
}


// cache-policy bits on the 16-B loads (one asm block: 4 loads + wait), XCD-aware tile order
#define RP_ASM_KERNEL(NAME, BITS)                                                              \
__global__ __launch_bounds__(256) void NAME(const uint8_t* data, uint64_t n16, uint2* out, int xcd) { \
    uint64_t b = blockIdx.x;                                                                   \
    if (xcd) { const uint64_t per = gridDim.x / 8; b = (blockIdx.x % 8) * per + blockIdx.x / 8; } \
    const uint64_t base = b * 1024;                                                            \
    const uint8_t* p0 = data + 16 * (base + threadIdx.x);                                      \
    u32x4 v0, v1, v2, v3;                                                                      \
    asm volatile("global_load_dwordx4 %0, %4, off " BITS "\n\t"                                \
                 "global_load_dwordx4 %1, %5, off " BITS "\n\t"                                \
                 "global_load_dwordx4 %2, %6, off " BITS "\n\t"                                \
                 "global_load_dwordx4 %3, %7, off " BITS "\n\t"                                \
                 "s_waitcnt vmcnt(0)"                                                          \
                 : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3)                                  \
                 : "v"(p0), "v"(p0 + 4096), "v"(p0 + 8192), "v"(p0 + 12288) : "memory");       \
    const uint32_t x = v0.x ^ v0.y ^ v0.z ^ v0.w ^ v1.x ^ v1.y ^ v1.z ^ v1.w ^                  \
                       v2.x ^ v2.y ^ v2.z ^ v2.w ^ v3.x ^ v3.y ^ v3.z ^ v3.w;                   \
    out[b * 256 + threadIdx.x] = make_uint2(x, 0);                                             \
}
RP_ASM_KERNEL(k_rp_nt, "nt")
RP_ASM_KERNEL(k_rp_sc0nt, "sc0 nt")
RP_ASM_KERNEL(k_rp_sc1nt, "sc1 nt")
RP_ASM_KERNEL(k_rp_sc01nt, "sc0 sc1 nt")
RP_ASM_KERNEL(k_rp_sc01, "sc0 sc1")
RP_ASM_KERNEL(k_rp_plain, "")

int main(int argc, char** argv) {
    const uint64_t count = argc > 1 ? strtoull(argv[1], 0, 0) : (16ull << 20), bytes = count * 64, n16 = bytes / 16;
    uint8_t* data;
    uint2* out;
    CK(hipMalloc(&data, bytes));
    CK(hipMalloc(&out, count * 8));
    uint8_t* rec;
    CK(hipMalloc(&rec, count * 64));
    CK(hipMemset(data, 1, bytes));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    struct V { std::string name; std::function<void()> f; std::vector<float> ms; };
    std::vector<V> vs;
    vs.push_back({"rp_L4_nt", [=]() { hipLaunchKernelGGL((k_rp<4, true>), dim3(n16 / 1024), dim3(256), 0, 0, data, n16, out); }});
    vs.push_back({"rp_L4", [=]() { hipLaunchKernelGGL((k_rp<4, false>), dim3(n16 / 1024), dim3(256), 0, 0, data, n16, out); }});
    vs.push_back({"rp_L8_nt", [=]() { hipLaunchKernelGGL((k_rp<8, true>), dim3(n16 / 2048), dim3(256), 0, 0, data, n16, out); }});
    vs.push_back({"rp_L16_nt", [=]() { hipLaunchKernelGGL((k_rp<16, true>), dim3(n16 / 4096), dim3(256), 0, 0, data, n16, out); }});
    for (int per : {4, 8, 16}) {
        const uint32_t g = cus * per;
        vs.push_back({"persist_x" + std::to_string(per), [=]() { hipLaunchKernelGGL(k_rp_persist, dim3(g), dim3(256), 0, 0, data, n16 / 1024, out); }});
    }
    vs.push_back({"multi2", [=]() { hipLaunchKernelGGL(k_rp_multi<2>, dim3(n16 / 2048), dim3(256), 0, 0, data, n16, out); }});
    vs.push_back({"multi4", [=]() { hipLaunchKernelGGL(k_rp_multi<4>, dim3(n16 / 4096), dim3(256), 0, 0, data, n16, out); }});
    vs.push_back({"multi8", [=]() { hipLaunchKernelGGL(k_rp_multi<8>, dim3(n16 / 8192), dim3(256), 0, 0, data, n16, out); }});
    vs.push_back({"multi16", [=]() { hipLaunchKernelGGL(k_rp_multi<16>, dim3(n16 / 16384), dim3(256), 0, 0, data, n16, out); }});
    {
        const dim3 g(n16 / 1024);
        vs.push_back({"asm_nt", [=]() { hipLaunchKernelGGL(k_rp_nt, g, dim3(256), 0, 0, data, n16, out, 0); }});
        vs.push_back({"asm_nt_xcd", [=]() { hipLaunchKernelGGL(k_rp_nt, g, dim3(256), 0, 0, data, n16, out, 1); }});
        vs.push_back({"asm_sc0nt", [=]() { hipLaunchKernelGGL(k_rp_sc0nt, g, dim3(256), 0, 0, data, n16, out, 0); }});
        vs.push_back({"asm_sc1nt", [=]() { hipLaunchKernelGGL(k_rp_sc1nt, g, dim3(256), 0, 0, data, n16, out, 0); }});
        vs.push_back({"asm_sc01nt", [=]() { hipLaunchKernelGGL(k_rp_sc01nt, g, dim3(256), 0, 0, data, n16, out, 0); }});
        vs.push_back({"asm_sc01", [=]() { hipLaunchKernelGGL(k_rp_sc01, g, dim3(256), 0, 0, data, n16, out, 0); }});
        vs.push_back({"asm_plain", [=]() { hipLaunchKernelGGL(k_rp_plain, g, dim3(256), 0, 0, data, n16, out, 0); }});
    }
    for (int R : {2, 4, 8}) {
        const uint64_t nunits = count / 64;
        const uint32_t g4 = cus * (R == 8 ? 1 : (R == 4 ? 2 : 4));
        if (R == 2) vs.push_back({"ring_R2_W4", [=]() { hipLaunchKernelGGL((k_rp_ring<2, 4>), dim3(g4), dim3(256), 0, 0, data, nunits, out); }});
        if (R == 4) vs.push_back({"ring_R4_W4", [=]() { hipLaunchKernelGGL((k_rp_ring<4, 4>), dim3(g4), dim3(256), 0, 0, data, nunits, out); }});
        if (R == 8) vs.push_back({"ring_R8_W4", [=]() { hipLaunchKernelGGL((k_rp_ring<8, 4>), dim3(g4), dim3(256), 0, 0, data, nunits, out); }});
    }
    vs.push_back({"readonly_L4_nt", [=]() { hipLaunchKernelGGL((k_ro<4>), dim3(n16 / 1024), dim3(256), 0, 0, data, n16, out); }});
    vs.push_back({"readonly_L8_nt", [=]() { hipLaunchKernelGGL((k_ro<8>), dim3(n16 / 2048), dim3(256), 0, 0, data, n16, out); }});
    {
        uint8_t* o8 = reinterpret_cast<uint8_t*>(out);
        const dim3 g(n16 / 1024);
        vs.push_back({"w8_plain", [=]() { hipLaunchKernelGGL((k_wv<8, 0>), g, dim3(256), 0, 0, data, n16, o8); }});
        for (int lg : {16, 19, 22, 24}) {  // 512 KiB, 4 MiB, 32 MiB, 128 MiB windows
            const uint64_t m = (1ull << lg) - 1;
            vs.push_back({"w8_win" + std::to_string(8ull << lg >> 20) + "MiB", [=]() { hipLaunchKernelGGL(k_wwin, g, dim3(256), 0, 0, data, n16, out, m); }});
        }
        vs.push_back({"w8_via16_nt", [=]() { hipLaunchKernelGGL(k_wv16nt, g, dim3(256), 0, 0, data, n16, o8); }});
        vs.push_back({"rec64_plain", [=]() { hipLaunchKernelGGL(k_rec<false>, g, dim3(256), 0, 0, data, n16, reinterpret_cast<uint8_t*>(rec)); }});
        vs.push_back({"rec64_nt", [=]() { hipLaunchKernelGGL(k_rec<true>, g, dim3(256), 0, 0, data, n16, reinterpret_cast<uint8_t*>(rec)); }});
        vs.push_back({"w8_via16", [=]() { hipLaunchKernelGGL(k_wv16, g, dim3(256), 0, 0, data, n16, o8); }});
        vs.push_back({"w8_nt", [=]() { hipLaunchKernelGGL((k_wv<8, 1>), g, dim3(256), 0, 0, data, n16, o8); }});
        vs.push_back({"w8_sc01nt", [=]() { hipLaunchKernelGGL((k_wv<8, 2>), g, dim3(256), 0, 0, data, n16, o8); }});
        vs.push_back({"w4_plain", [=]() { hipLaunchKernelGGL((k_wv<4, 0>), g, dim3(256), 0, 0, data, n16, o8); }});
        vs.push_back({"w4_nt", [=]() { hipLaunchKernelGGL((k_wv<4, 1>), g, dim3(256), 0, 0, data, n16, o8); }});
        vs.push_back({"w1_plain", [=]() { hipLaunchKernelGGL((k_wv<1, 0>), g, dim3(256), 0, 0, data, n16, o8); }});
        vs.push_back({"w1_nt", [=]() { hipLaunchKernelGGL((k_wv<1, 1>), g, dim3(256), 0, 0, data, n16, o8); }});
        vs.push_back({"wbatch4", [=]() { hipLaunchKernelGGL(k_wbatch<4>, dim3(n16 / 4096), dim3(256), 0, 0, data, n16, out); }});
        vs.push_back({"wbatch8", [=]() { hipLaunchKernelGGL(k_wbatch<8>, dim3(n16 / 8192), dim3(256), 0, 0, data, n16, out); }});
    }
    vs.push_back({"ldsdma", [=]() { hipLaunchKernelGGL(k_rp_ldsdma, dim3(n16 / 1024), dim3(256), 0, 0, data, n16, out); }});
    // rotation over ROT separate buffers of the same size: re-use distance
    // ROT x bytes (what a fresh batch per step sees from the memory-side cache)
    const int ROT = 6;
    std::vector<uint8_t*> rot(ROT, nullptr);
    int rot_ok = 1;
    for (int r = 0; r < ROT; r++) {
        if (hipMalloc(&rot[r], bytes) != hipSuccess) { rot_ok = 0; break; }
        CK(hipMemset(rot[r], 1, bytes));
    }
    if (rot_ok) {
        auto cnt = std::make_shared<int>(0);
        vs.push_back({"rot6_L4_nt", [=]() { int r = (*cnt)++ % ROT; hipLaunchKernelGGL((k_rp<4, true>), dim3(n16 / 1024), dim3(256), 0, 0, rot[r], n16, out); }});
        auto cnt2 = std::make_shared<int>(0);
        vs.push_back({"rot6_asm_nt_xcd", [=]() { int r = (*cnt2)++ % ROT; hipLaunchKernelGGL(k_rp_nt, dim3(n16 / 1024), dim3(256), 0, 0, rot[r], n16, out, 1); }});
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < 7; r++)
        for (auto& v : vs) {
            v.f();
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < 20; i++) v.f();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            v.ms.push_back(ms / 20);
        }
    CK(hipGetLastError());
    printf("CUs %d\n%-16s %9s %9s %8s\n", cus, "variant", "med_us", "GB/s", "frac8T");
    for (auto& v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        double med = v.ms[3];
        printf("%-16s %9.1f %9.1f %8.3f\n", v.name.c_str(), med * 1e3, bytes / (med * 1e-3) / 1e9, bytes / (med * 1e-3) / 8e12);
    }
}
