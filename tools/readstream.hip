// readstream.hip — a bare read stream over a caller's device buffer, loaded
// by tools/contig_ab.py to time the memory under each allocation with the
// parse (measurement tool; not part of libnexg).
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {
constexpr int kL = 16;                       // 16-B loads per thread
constexpr uint64_t kBlockBytes = 256ull * kL * 16;  // 64 KiB per workgroup

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_readstream(const u32x4* data, uint32_t* out) {
    const uint64_t base = (uint64_t)blockIdx.x * 256 * kL;
    uint32_t x = 0;
    u32x4 v[kL];
#pragma unroll
    for (int k = 0; k < kL; k++) v[k] = __builtin_nontemporal_load(data + base + threadIdx.x + 256 * k);
#pragma unroll
    for (int k = 0; k < kL; k++) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    if (x == 0x9e3779b9u) out[threadIdx.x] = x;  // never taken on the tool's data; keeps the loads
}
// The span kernel's read structure without its parse: each workgroup reads
// `per_wg` bytes (from a 16-B offset `skew` past a 64-KiB boundary) as 20-KiB
// sub-tiles, the next in flight while the current one is staged into LDS and
// summed across the workgroup (two barriers per sub-tile).
constexpr uint32_t kSub = 20480, kCpt = kSub / 4096;
__global__ __launch_bounds__(256) void k_readspan(const uint8_t* data, uint32_t per_wg, uint32_t skew, uint32_t* out) {
    __shared__ u32x4 s_tile[kSub / 16];
    const uint32_t t = threadIdx.x;
    const uint8_t* p = data + (uint64_t)blockIdx.x * per_wg + skew;
    u32x4 cur[kCpt];
    auto fetch = [&](uint32_t S) {
#pragma unroll
        for (int i = 0; i < (int)kCpt; i++) {
            const uint32_t c = S + 16u * (t + 256u * i);
            cur[i] = c < per_wg ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + c)) : u32x4{0, 0, 0, 0};
        }
    };
    fetch(0);
    uint32_t x = 0;
    for (uint32_t S = 0; S < per_wg; S += kSub) {
#pragma unroll
        for (int i = 0; i < (int)kCpt; i++) s_tile[t + 256u * i] = cur[i];
        if (S + kSub < per_wg) fetch(S + kSub);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < (int)kCpt; i++) {
            const u32x4 v = s_tile[(t * 5u + (uint32_t)i * 37u) % (kSub / 16)];
            x ^= v.x ^ v.y ^ v.z ^ v.w;
        }
        __syncthreads();
    }
    if (x == 0x9e3779b9u) out[t] = x;
}
}  // namespace

// Span-structured read of buf (k_readspan); returns the bytes read (0 on a bad argument).
extern "C" uint64_t readspan_launch(const void* buf, uint64_t bytes, uint32_t per_wg, uint32_t skew, void* out,
                                    hipStream_t s) {
    if (!buf || !out || per_wg == 0 || (per_wg & 15) || (skew & 15) || skew >= 65536 ||
        (reinterpret_cast<uintptr_t>(buf) & 15))
        return 0;
    const uint64_t usable = bytes > 65536 ? bytes - 65536 : 0;
    const uint64_t blocks = usable / per_wg;
    if (blocks == 0 || blocks > 0x7fffffffull) return 0;
    hipLaunchKernelGGL(k_readspan, dim3((uint32_t)blocks), dim3(256), 0, s, static_cast<const uint8_t*>(buf), per_wg,
                       skew, static_cast<uint32_t*>(out));
    return hipGetLastError() == hipSuccess ? blocks * per_wg : 0;
}

// Reads the first floor(bytes / 64 KiB) * 64 KiB bytes of buf once; returns
// the bytes read (0 on a bad argument or launch error). out: >= 1 KiB scratch.
extern "C" uint64_t readstream_launch(const void* buf, uint64_t bytes, void* out, hipStream_t s) {
    const uint64_t blocks = bytes / kBlockBytes;
    if (!buf || !out || blocks == 0 || blocks > 0x7fffffffull || (reinterpret_cast<uintptr_t>(buf) & 15)) return 0;
    hipLaunchKernelGGL(k_readstream, dim3((uint32_t)blocks), dim3(256), 0, s,
                       static_cast<const u32x4*>(buf), static_cast<uint32_t*>(out));
    return hipGetLastError() == hipSuccess ? blocks * kBlockBytes : 0;
}
