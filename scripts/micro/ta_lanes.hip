// Micro-benchmark: cost of a divergent vector-memory instruction on gfx950.
// Each wave issues ITERS buffer_load_dwordx4 (L2-resident, gathered
// addresses) with only `active` lanes enabled; if the texture-address path
// charges per instruction, the time is independent of `active`.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) probe(const float4* buf, unsigned n, int active, int iters, float* out)
{
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)buf, 0, (int)(n * 16), 0x00020000);
    const unsigned lane = threadIdx.x & 63;
    unsigned idx = (blockIdx.x * 2654435761u + threadIdx.x * 40503u) % n;
    float acc = 0.f;
    if ((int)lane < active) {
        for (int i = 0; i < iters; ++i) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(idx * 16), 0, 0);
            acc += __uint_as_float(v.x);
            idx = (idx * 1103515245u + 12345u + v.y) % n;     // dependent: latency-bound per wave
        }
    }
    if (acc == 1234.5f) out[0] = acc;
}

__global__ void __launch_bounds__(256) probe_ind(const float4* buf, unsigned n, int active, int iters, float* out)
{
    // 4 independent chains per lane: throughput-bound
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)buf, 0, (int)(n * 16), 0x00020000);
    const unsigned lane = threadIdx.x & 63;
    unsigned i0 = (blockIdx.x * 2654435761u + threadIdx.x * 40503u) % n, i1 = (i0 + 977) % n, i2 = (i0 + 5003) % n,
             i3 = (i0 + 31337) % n;
    float acc = 0.f;
    if ((int)lane < active) {
        for (int i = 0; i < iters; ++i) {
            const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i0 * 16), 0, 0);
            const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i1 * 16), 0, 0);
            const u32x4 c = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i2 * 16), 0, 0);
            const u32x4 d = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i3 * 16), 0, 0);
            acc += __uint_as_float(a.x) + __uint_as_float(b.x) + __uint_as_float(c.x) + __uint_as_float(d.x);
            i0 = (i0 + 7919u + a.y) % n; i1 = (i1 + 104729u + b.y) % n;
            i2 = (i2 + 1299709u + c.y) % n; i3 = (i3 + 15485863u + d.y) % n;
        }
    }
    if (acc == 1234.5f) out[0] = acc;
}

int main()
{
    const unsigned n = 1u << 16;                 // 1 MiB of float4: L2-resident
    std::vector<float4> h(n);
    for (unsigned i = 0; i < n; ++i) h[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    float4* d; float* o;
    hipMalloc(&d, n * 16); hipMalloc(&o, 4);
    hipMemcpy(d, h.data(), n * 16, hipMemcpyHostToDevice);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const int blocks = 256 * 16, iters = 256;
    for (int kind = 0; kind < 2; ++kind) {
        for (int active : { 64, 32, 16, 8, 4, 1 }) {
            float best = 1e30f;
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(a);
                if (kind == 0) probe<<<blocks, 256>>>(d, n, active, iters, o);
                else probe_ind<<<blocks, 256>>>(d, n, active, iters, o);
                hipEventRecord(b); hipEventSynchronize(b);
                float ms; hipEventElapsedTime(&ms, a, b);
                if (ms < best) best = ms;
            }
            const double wave_insts = (double)blocks * 4 * iters * (kind ? 4 : 1);
            printf("%s active=%2d: %.3f ms  %.2f ns per wave-instruction (chip)  %.1f GB/s useful\n",
                   kind ? "independent" : "dependent  ", active, best, best * 1e6 / wave_insts,
                   wave_insts * active * 16 / (best * 1e-3) / 1e9);
        }
    }
    return 0;
}
