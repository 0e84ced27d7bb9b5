// writebench.hip — the write-stream ceiling the builders' copy-out runs into:
// each workgroup writes one 256-frame tile (256 x P bytes, P = the probe
// batches' frame lengths) with 16-B non-temporal stores, 16M frames in all,
// by workgroups per CU (dynamic LDS cap), tile order (tile_of) and grid
// shape (one tile per workgroup, or a persistent sweep of 256 x cap
// workgroups over virtual tiles b, b + G, ...).
// usage: ./tools/writebench [frames, default 16M]
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

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void write_tile(uint8_t* out, uint64_t tile, uint32_t P) {
    v4u* T = reinterpret_cast<v4u*>(out + tile * 256u * P);
    for (uint32_t c = threadIdx.x; c < 16u * P; c += 256u)
        __builtin_nontemporal_store(v4u{(uint32_t)tile, c, P, 0u}, T + c);
}

__global__ __launch_bounds__(256) void k_wtile(uint8_t* out, uint32_t P, uint32_t order) {
    extern __shared__ uint32_t s_cap[];  // dynamic LDS only caps workgroups per CU
    if (order == 0xFFFFFFFFu) s_cap[threadIdx.x] = 0;
    write_tile(out, tile_index(order), P);
}

__global__ __launch_bounds__(256) void k_wsweep(uint8_t* out, uint32_t P, uint32_t order, uint32_t nt) {
    extern __shared__ uint32_t s_cap[];
    if (order == 0xFFFFFFFFu) s_cap[threadIdx.x] = 0;
    for (uint32_t v = blockIdx.x; v < nt; v += gridDim.x) {
        write_tile(out, tile_of(v, nt, order), P);
        __syncthreads();
    }
}

int main(int argc, char** argv) {
    const uint64_t count = argc > 1 ? strtoull(argv[1], 0, 0) : (16ull << 20);
    const uint32_t nt = (uint32_t)(count / 256);
    uint8_t* out;
    CK(hipMalloc(&out, count * 128));
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    struct V { std::string name; uint64_t bytes; std::function<void()> f; std::vector<float> ms; };
    std::vector<V> vs;
    for (uint32_t P : {42u, 47u, 62u, 66u, 67u, 86u})
        for (int cap : {2, 3, 4, 5, 6, 8})
            for (uint32_t o : {0u, 1u, 16u}) {
                const uint32_t lds = 160u * 1024u / cap - 1024u;
                const std::string on = o == 0 ? "grid" : (o == 1 ? "eighths" : "K16");
                const std::string base = "P" + std::to_string(P) + "_cap" + std::to_string(cap) + "_" + on;
                vs.push_back({"tile_" + base, count * P, [=]() {
                    hipLaunchKernelGGL(k_wtile, dim3(nt), dim3(256), lds, 0, out, P, o); }});
                const uint32_t g = std::min<uint32_t>(nt, (uint32_t)cus * cap);
                vs.push_back({"sweep_" + base, count * P, [=]() {
                    hipLaunchKernelGGL(k_wsweep, dim3(g), dim3(256), lds, 0, out, P, o, nt); }});
            }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < 5; r++) {
        for (auto& v : vs) {
            for (int i = 0; i < 3; i++) v.f();
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < 10; i++) v.f();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            v.ms.push_back(ms / 10);
        }
        printf("round %d done\n", r);
        fflush(stdout);
    }
    CK(hipGetLastError());
    printf("%-28s %9s %9s %8s\n", "variant", "med_us", "GB/s", "frac8T");
    for (auto& v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        const double med = v.ms[2];
        printf("%-28s %9.1f %9.1f %8.3f\n", v.name.c_str(), med * 1e3, v.bytes / (med * 1e-3) / 1e9,
               v.bytes / (med * 1e-3) / 8e12);
    }
    CK(hipFree(out));
    return 0;
}
