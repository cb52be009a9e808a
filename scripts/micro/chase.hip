// chase.hip -- dependent-load latency on gfx950 (pointer chase), the unit
// cost of a traversal step on a launch's critical path (one long path walks
// ~100-200 nodes one dependent fetch after another).
//
//   hipcc -O3 --offload-arch=gfx950 -o scripts/micro/chase scripts/micro/chase.hip
//
// One wave per launch (a lone long path at the end of a launch), 1 or 64
// lanes each following its own random cycle of 128-B lines through a table
// of S bytes; prints ns per dependent 16-B load for each S (L2 4 MB per XCD,
// MALL 256 MB, then HBM) and for the LDS.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>
#include <algorithm>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void chase(const u32x4* __restrict__ t, uint32_t lanes, uint32_t steps, uint32_t start_stride,
                     uint64_t* out)
{
    const uint32_t lane = threadIdx.x;
    uint32_t i = lane * start_stride;                     // line index (8 u32x4 per 128-B line)
    uint32_t acc = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    if (lane < lanes) {
#pragma unroll 1
        for (uint32_t s = 0; s < steps; ++s) {
            const u32x4 v = t[(size_t)i * 8u];
            i = v.x;
            acc += v.y;
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) { out[0] = t1 - t0; out[1] = acc + i; }
}

__global__ void chase_lds(uint32_t steps, uint64_t* out)
{
    __shared__ uint32_t s[4096];
    for (uint32_t k = threadIdx.x; k < 4096; k += blockDim.x) s[k] = (k * 2654435761u + 977u) & 4095u;
    __syncthreads();
    uint32_t i = threadIdx.x;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
    for (uint32_t k = 0; k < steps; ++k) i = s[i];
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = i; }
}

int main()
{
    const uint64_t maxb = 2048ull << 20;
    u32x4* tab = nullptr;
    uint64_t* out = nullptr;
    CHECK(hipMalloc(&tab, maxb));
    CHECK(hipMalloc(&out, 64));
    const uint64_t sizes[] = { 64ull << 10, 1ull << 20, 3ull << 20, 16ull << 20, 128ull << 20, 2048ull << 20 };
    std::mt19937 rng(1234);
    const uint32_t steps = 4000;
    for (uint64_t S : sizes) {
        const uint32_t n = (uint32_t)(S / 128);
        std::vector<uint32_t> perm(n);
        for (uint32_t k = 0; k < n; ++k) perm[k] = k;
        std::shuffle(perm.begin(), perm.end(), rng);
        std::vector<u32x4> h((size_t)n * 8);
        for (uint32_t k = 0; k < n; ++k) h[(size_t)perm[k] * 8] = u32x4{ perm[(k + 1) % n], 1u, 0u, 0u };
        CHECK(hipMemcpy(tab, h.data(), h.size() * sizeof(u32x4), hipMemcpyHostToDevice));
        for (uint32_t lanes : { 1u, 64u }) {
            double best = 1e30;
            for (int rep = 0; rep < 3; ++rep) {
                hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, tab, lanes, steps, n / 64u, out);
                uint64_t o[2];
                CHECK(hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost));
                best = std::min(best, o[0] * 10.0 / steps);      // s_memrealtime: 100 MHz
            }
            std::printf("table %8.1f MB  lanes %2u  %7.1f ns per dependent load\n", S / 1048576.0, lanes, best);
        }
    }
    hipLaunchKernelGGL(chase_lds, dim3(1), dim3(64), 0, 0, steps * 4, out);
    uint64_t o[2];
    CHECK(hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost));
    std::printf("LDS  lanes 64  %7.1f ns per dependent load\n", o[0] * 10.0 / (steps * 4));
    CHECK(hipFree(tab));
    CHECK(hipFree(out));
    return 0;
}
