// orderbench.hip — read / write stream rates by workgroup -> tile order
// (tile_of, nex_amd/csrc/nexg_internal.hpp): is the fixed-stride parse kernel's
// 0.92 of 8 TB/s the stream's own ceiling in its best order, and which run
// length K wins for plain streams of 16-KiB and 32-KiB tiles.
// usage: ./tools/orderbench [frames of 64 B, default 16M]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>
#include "../nex_amd/csrc/frame_core.hpp"
#include "../nex_amd/csrc/nexg_internal.hpp"
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
using namespace nexg;

// read L 16-B non-temporal loads per lane (tile = 4 KiB * L), xor, one dword out per tile
template <int L>
__global__ __launch_bounds__(256) void k_read(const uint8_t* data, uint32_t* out, uint32_t order) {
    extern __shared__ uint32_t s_cap[];  // dynamic LDS only caps workgroups per CU
    const uint64_t tile = tile_index(order);
    if (order == 0xFFFFFFFFu) s_cap[threadIdx.x] = 0;
    const uint8_t* T = data + tile * (4096u * L);
    uint4 v[L];
#pragma unroll
    for (int k = 0; k < L; k++) v[k] = load16<true>(T + 16u * (threadIdx.x + 256u * k));
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < L; k++) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    if (x == 0x9e3779b9u) out[tile] = x;  // never true on the memset data: a pure read stream
}

// 16-B non-temporal stores, 16 KiB per workgroup (the builders' copy-out shape)
__global__ __launch_bounds__(256) void k_write(uint8_t* out, uint32_t order) {
    extern __shared__ uint32_t s_cap[];
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const uint64_t tile = tile_index(order);
    if (order == 0xFFFFFFFFu) s_cap[threadIdx.x] = 0;
    v4u* T = reinterpret_cast<v4u*>(out + tile * 16384u);
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
        const uint32_t c = threadIdx.x + 256u * k;
        __builtin_nontemporal_store(v4u{(uint32_t)tile, c, 0u, 0u}, T + c);
    }
}

int main(int argc, char** argv) {
    const uint64_t count = argc > 1 ? strtoull(argv[1], 0, 0) : (16ull << 20), bytes = count * 64;
    uint8_t* data;
    uint32_t* out;
    CK(hipMalloc(&data, bytes));
    CK(hipMalloc(&out, bytes / 4096 * 4 + 64));
    CK(hipMemset(data, 1, bytes));
    struct V { std::string name; std::function<void()> f; std::vector<float> ms; };
    std::vector<V> vs;
    const uint32_t orders[] = {0, 1, 4, 8, 16, 32, 64, 128};
    for (uint32_t o : orders) {
        const std::string on = o == 0 ? "grid" : (o == 1 ? "eighths" : "K" + std::to_string(o));
        vs.push_back({"read16K_" + on, [=]() { hipLaunchKernelGGL(k_read<4>, dim3((uint32_t)(bytes / 16384)), dim3(256), 0, 0, data, out, o); }});
        vs.push_back({"read32K_" + on, [=]() { hipLaunchKernelGGL(k_read<8>, dim3((uint32_t)(bytes / 32768)), dim3(256), 0, 0, data, out, o); }});
        vs.push_back({"write16K_" + on, [=]() { hipLaunchKernelGGL(k_write, dim3((uint32_t)(bytes / 16384)), dim3(256), 0, 0, data, o); }});
    }
    // workgroups per CU capped by dynamic LDS (160 KiB per CU): the parse
    // kernel runs 6 per CU (77 VGPRs), a bare stream 8
    for (int cap : {3, 4, 5, 6, 7}) {
        const uint32_t lds = 160u * 1024u / cap - 1024u;
        for (uint32_t o : {0u, 16u}) {
            const std::string on = o == 0 ? "grid" : "K16";
            vs.push_back({"read16K_" + on + "_cap" + std::to_string(cap), [=]() {
                hipLaunchKernelGGL(k_read<4>, dim3((uint32_t)(bytes / 16384)), dim3(256), lds, 0, data, out, o); }});
            vs.push_back({"write16K_" + on + "_cap" + std::to_string(cap), [=]() {
                hipLaunchKernelGGL(k_write, dim3((uint32_t)(bytes / 16384)), dim3(256), lds, 0, data, o); }});
        }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < 7; r++)
        for (auto& v : vs) {
            for (int i = 0; i < 5; i++) v.f();
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < 20; i++) v.f();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            v.ms.push_back(ms / 20);
        }
    CK(hipGetLastError());
    printf("bytes %llu\n%-20s %9s %9s %8s\n", (unsigned long long)bytes, "variant", "med_us", "GB/s", "frac8T");
    for (auto& v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        const double med = v.ms[3];
        printf("%-20s %9.1f %9.1f %8.3f\n", v.name.c_str(), med * 1e3, bytes / (med * 1e-3) / 1e9,
               bytes / (med * 1e-3) / 8e12);
    }
    CK(hipFree(data));
    CK(hipFree(out));
    return 0;
}
