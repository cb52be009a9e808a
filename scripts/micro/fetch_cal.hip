// fetch_cal.hip -- calibrates rocprofv3 FETCH_SIZE (and the TCC request
// counters behind it) for the access widths the path kernel uses, against
// known byte counts, on a table far larger than the 256 MiB Infinity Cache.
//
//   hipcc -O3 --offload-arch=gfx950 -o scripts/micro/fetch_cal scripts/micro/fetch_cal.hip
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- scripts/micro/fetch_cal
//   rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum -- scripts/micro/fetch_cal
//
// One dispatch per pattern, each over its own 512 MiB region of a 4 GiB
// table (no pattern reads lines another left in a cache).  Every pattern
// touches each of its 128-B lines at most once; lines are picked by an odd
// multiplicative permutation, so a wave's lanes read 64 different lines:
//   stream16   coalesced 16 B per lane, whole lines (the guide's calibrated case)
//   gather16   one 16-B load per line            (HDRI / texel / node-row fetch)
//   gather32   two 16-B loads, 32 contiguous B   (fp16 node visit, primary record)
//   gather72   4 x 16 B + 8 B, 72 contiguous B at a 36-B-aligned offset inside a
//              256-B pair of lines (triangle-pair fetch; straddles a line boundary
//              at some offsets)
// The program prints each pattern's loads and requested bytes (one line per
// dispatch, in dispatch order) so the counter passes can be divided by them.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr uint64_t kRegion = 512ull << 20;          // bytes per pattern
constexpr uint32_t kLines = (uint32_t)(kRegion / 256);   // 256-B slots per region (2 lines each)

__device__ __forceinline__ uint32_t perm(uint32_t i) { return (i * 2654435761u) & (kLines - 1u); }

__global__ void stream16(const u32x4* __restrict__ t, uint32_t n, uint32_t* out)
{
    uint32_t acc = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const u32x4 v = t[i];
        acc ^= v.x ^ v.w;
    }
    if (acc == 0x9e3779b9u) out[0] = acc;
}

// mode 16: one 16-B load; 32: two; 72: 4 x 16 + 8 at offset 36 * (i % 3) in the 256-B slot
template <int MODE>
__global__ void gather(const uint8_t* __restrict__ base, uint32_t n, uint32_t* out)
{
    uint32_t acc = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint64_t slot = (uint64_t)perm(i) * 256u;
        if (MODE == 16) {
            acc ^= reinterpret_cast<const u32x4*>(base + slot)[0].x;
        } else if (MODE == 32) {
            const u32x4* p = reinterpret_cast<const u32x4*>(base + slot);
            const u32x4 a = p[0], b = p[1];
            acc ^= a.x ^ b.w;
        } else {
            const uint32_t off = 36u * (i % 3u) + 36u;       // 36, 72 or 108: 72 B inside [36, 180)
            const uint8_t* q = base + slot + off;
            const u32x4 a = *reinterpret_cast<const u32x4*>(q + 0);
            const u32x4 b = *reinterpret_cast<const u32x4*>(q + 16);
            const u32x4 c = *reinterpret_cast<const u32x4*>(q + 32);
            const u32x4 d = *reinterpret_cast<const u32x4*>(q + 48);
            const u32x2 e = *reinterpret_cast<const u32x2*>(q + 64);
            acc ^= a.x ^ b.y ^ c.z ^ d.w ^ e.x;
        }
    }
    if (acc == 0x9e3779b9u) out[0] = acc;
}

int main()
{
    uint8_t* tab = nullptr;
    uint32_t* out = nullptr;
    const uint64_t total = 8 * kRegion;
    CHECK(hipMalloc(&tab, total));
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMemset(tab, 1, total));
    CHECK(hipDeviceSynchronize());
    const dim3 grid(256 * 16), block(256);
    // every pattern twice, in fresh regions: the second is the one to read (warm code, cold data)
    for (int rep = 0; rep < 2; ++rep) {
        uint8_t* r = tab + (uint64_t)rep * 4 * kRegion;
        const uint32_t ns = (uint32_t)(kRegion / 4 / 16);   // stream: a quarter of the region
        hipLaunchKernelGGL(stream16, grid, block, 0, 0, reinterpret_cast<const u32x4*>(r), ns, out);
        std::printf("rep %d stream16 loads %u bytes %llu lines128 %llu\n", rep, ns, (unsigned long long)ns * 16,
                    (unsigned long long)ns * 16 / 128);
        const uint32_t ng = kLines;                           // one access per 256-B slot
        hipLaunchKernelGGL(gather<16>, grid, block, 0, 0, r + kRegion, ng, out);
        std::printf("rep %d gather16 loads %u bytes %llu lines128 %u\n", rep, ng, (unsigned long long)ng * 16, ng);
        hipLaunchKernelGGL(gather<32>, grid, block, 0, 0, r + 2 * kRegion, ng, out);
        std::printf("rep %d gather32 loads %u bytes %llu lines128 %u\n", rep, 2 * ng, (unsigned long long)ng * 32, ng);
        hipLaunchKernelGGL(gather<72>, grid, block, 0, 0, r + 3 * kRegion, ng, out);
        // offsets 36/72/108 + 72 B end at 108/144/180: the 72- and 108-offset runs cross the 128-B boundary
        std::printf("rep %d gather72 loads %u bytes %llu lines128 %llu\n", rep, 5 * ng, (unsigned long long)ng * 72,
                    (unsigned long long)ng + 2ull * ng / 3ull);
        CHECK(hipDeviceSynchronize());
    }
    CHECK(hipFree(tab));
    CHECK(hipFree(out));
    return 0;
}
