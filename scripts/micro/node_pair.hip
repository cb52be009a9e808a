// Micro-benchmark: does the second 16-B load of a 32-B node record cost the
// texture path as much as the first?  Every lane walks 4 independent chains
// of random 128-B lines of an L2-resident table; per step and chain it loads
// mode 0: one 16-B record, mode 1: two 16-B halves of one 32-B record (same
// line), mode 2: 16 B + 8 B.  `active` lanes of each wave (scattered) take
// part, as in a diverged traversal.  Prints ns per wave-step (all 4 chains).
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/node_pair scripts/micro/node_pair.hip && /tmp/node_pair
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

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
        const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
        if constexpr (MODE == 1) {
            const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(r, off + 16, 0, 0);
            return a.x ^ b.w;
        } else if constexpr (MODE == 2) {
            const u32x2 b = __builtin_amdgcn_raw_buffer_load_b64(r, off + 16, 0, 0);
            return a.x ^ b.y;
        }
        return a.x ^ a.w;
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
    const int blocks = 256 * 24, iters = 200;   // 6 waves/SIMD-ish residency in waves of 256 threads
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int active : { 64, 32, 18, 8 }) {
        for (int mode = 0; mode < 3; ++mode) {
            float best = 1e30f;
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(e0);
                if (mode == 0) hipLaunchKernelGGL(walk<0>, dim3(blocks), dim3(256), 0, 0, tab, lines, active, iters, out);
                if (mode == 1) hipLaunchKernelGGL(walk<1>, dim3(blocks), dim3(256), 0, 0, tab, lines, active, iters, out);
                if (mode == 2) hipLaunchKernelGGL(walk<2>, dim3(blocks), dim3(256), 0, 0, tab, lines, active, iters, out);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms; hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            const double wave_steps = (double)blocks * 4 * iters;   // waves x steps (4 chains each)
            printf("active %2d mode %d (%s): %.3f ms  %.3f ns per wave-step  (%.1f CU-cycles at 2.4 GHz per load instr)\n",
                   active, mode, mode == 0 ? "16 B" : mode == 1 ? "2 x 16 B" : "16 + 8 B", best, best * 1e6 / wave_steps,
                   best * 1e-3 * 256 * 2.4e9 / (wave_steps * 4 * (mode ? 2 : 1)));
        }
    }
    return 0;
}
