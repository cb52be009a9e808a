// Micro-benchmark for the wide-node question: what does
// the texture path charge a lane that reads a 32-B binary node record (2 x
// 16 B of one 128-B line) against a 64-B 4-wide record (4 x 16 B of one line),
// a whole 128-B line (8 x 16 B), or two 16-B records on two different lines?
// Every lane walks 4 independent chains of random 128-B lines of an
// L2-resident table; `active` lanes of each wave (scattered) take part, as in
// a diverged traversal.  Prints ns per wave-step (all 4 chains).
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/node_wide scripts/micro/node_wide.hip && /tmp/node_wide
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// MODE: 1, 2, 4, 8 loads of 16 B at offsets 0, 16, ... of one line; 20: two
// 16-B loads on two different lines (the second line = the next one)
template <int MODE>
__global__ void __launch_bounds__(256) walk(const unsigned* tab, unsigned lines, int active, int iters, unsigned* out)
{
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)tab, 0, (int)(lines * 128u), 0x00020000);
    const unsigned lane = threadIdx.x & 63u;
    const unsigned m = lines - 1u;
    unsigned i0 = (blockIdx.x * 2654435761u + threadIdx.x * 40503u) & m, i1 = (i0 + 977u) & m,
             i2 = (i0 + 5003u) & m, i3 = (i0 + 31337u) & m;
    unsigned acc = 0;
    auto ld = [&](unsigned line) -> unsigned {
        const int off = (int)(line * 128u);
        unsigned x = 0;
        if constexpr (MODE == 20) {
            const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
            const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(((line + 1u) & m) * 128u), 0, 0);
            return a.x ^ b.w;
        } else {
#pragma unroll
            for (int k = 0; k < MODE; ++k) {
                const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(r, off + 16 * k, 0, 0);
                x ^= a.x ^ a.w;
            }
        }
        return x;
    };
    if (((lane * 37u) & 63u) < (unsigned)active) {
        for (int i = 0; i < iters; ++i) {
            const unsigned a = ld(i0), b = ld(i1), c = ld(i2), d = ld(i3);
            acc += a + b + c + d;
            i0 = (i0 * 5u + 7919u + a) & m; i1 = (i1 * 5u + 104729u + b) & m;
            i2 = (i2 * 5u + 1299709u + c) & m; i3 = (i3 * 5u + 15485863u + d) & m;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main()
{
    const unsigned lines = 8192;                 // 1 MiB
    unsigned *tab, *out;
    hipMalloc(&tab, lines * 128);
    hipMemset(tab, 0, lines * 128);
    hipMalloc(&out, 64);
    const int blocks = 256 * 24, iters = 100;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int modes[] = { 1, 2, 4, 8, 20 };
    for (int active : { 64, 32, 18, 8 }) {
        for (int mode : modes) {
            float best = 1e30f;
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(e0);
                switch (mode) {
                case 1: hipLaunchKernelGGL(walk<1>, dim3(blocks), dim3(256), 0, 0, tab, lines, active, iters, out); break;
                case 2: hipLaunchKernelGGL(walk<2>, dim3(blocks), dim3(256), 0, 0, tab, lines, active, iters, out); break;
                case 4: hipLaunchKernelGGL(walk<4>, dim3(blocks), dim3(256), 0, 0, tab, lines, active, iters, out); break;
                case 8: hipLaunchKernelGGL(walk<8>, dim3(blocks), dim3(256), 0, 0, tab, lines, active, iters, out); break;
                default: hipLaunchKernelGGL(walk<20>, dim3(blocks), dim3(256), 0, 0, tab, lines, active, iters, out); break;
                }
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms; hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            const double wave_steps = (double)blocks * 4 * iters;
            printf("active %2d %-22s %.3f ms  %.3f ns per wave-step\n", active,
                   mode == 20 ? "2 x 16 B, two lines" : mode == 1 ? "1 x 16 B" : mode == 2 ? "2 x 16 B, one line" :
                   mode == 4 ? "4 x 16 B, one line" : "8 x 16 B, one line", best, best * 1e6 / wave_steps);
        }
    }
    return 0;
}
