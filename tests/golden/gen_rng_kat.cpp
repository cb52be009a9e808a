// Generates RNG known-answer vectors from rocThrust itself (the third-party
// dependency the reference kernel uses: cuda/src/PathTracer.cu:7-8,620-622),
// compiled for the host with hipcc.  Output: tests/golden/rng_kat.json.
//   hipcc -O2 -o /tmp/gen_rng_kat tests/golden/gen_rng_kat.cpp && /tmp/gen_rng_kat > tests/golden/rng_kat.json
#include <thrust/random.h>
#include <thrust/random/uniform_real_distribution.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

static uint32_t hash_seeds(uint32_t *s0, uint32_t *s1) {  // PathTracer.cu:574-580
    *s0 = 36969u * ((*s0) & 65535u) + ((*s0) >> 16);
    *s1 = 18000u * ((*s1) & 65535u) + ((*s1) >> 16);
    return *s0 * *s1;
}

int main() {
    const uint32_t seeds[] = {0u, 1u, 2u, 12345u, 2147483646u, 2147483647u, 2147483648u,
                              4294967295u, 0x88266ba4u, 0xcfc8cb90u, 0x19cbe700u, 0xdeadbeefu};
    std::printf("{\n  \"source\": \"rocThrust %d.%d.%d thrust::default_random_engine + uniform_real_distribution<float>(0,1)\",\n",
                THRUST_MAJOR_VERSION, THRUST_MINOR_VERSION, THRUST_SUBMINOR_VERSION);
    std::printf("  \"engine\": [\n");
    const int n = sizeof(seeds) / sizeof(seeds[0]);
    for (int i = 0; i < n; ++i) {
        thrust::default_random_engine rng(seeds[i]);
        thrust::uniform_real_distribution<float> u(0, 1);
        std::printf("    {\"seed\": %u, \"u_bits\": [", seeds[i]);
        for (int k = 0; k < 8; ++k) {
            float v = u(rng);
            uint32_t b; std::memcpy(&b, &v, 4);
            std::printf("%u%s", b, k < 7 ? ", " : "");
        }
        std::printf("]}%s\n", i < n - 1 ? "," : "");
    }
    std::printf("  ],\n  \"pixel\": [\n");
    const uint32_t px[][4] = {{100, 50, 1, 12345}, {640, 360, 2, 12345}, {0, 7, 3, 12345},
                              {1279, 719, 7, 1792098289u}, {511, 0, 4, 99}};
    const int np_ = sizeof(px) / sizeof(px[0]);
    for (int i = 0; i < np_; ++i) {
        uint32_t s0 = px[i][0] * px[i][2], s1 = px[i][1] * px[i][3];
        std::printf("    {\"x\": %u, \"y\": %u, \"frame\": %u, \"time\": %u, \"samples\": [", px[i][0], px[i][1], px[i][2], px[i][3]);
        for (int s = 0; s < 2; ++s) {
            uint32_t seed = hash_seeds(&s0, &s1);
            thrust::default_random_engine rng(seed);
            thrust::uniform_real_distribution<float> u(0, 1);
            std::printf("{\"seed\": %u, \"u_bits\": [", seed);
            for (int k = 0; k < 3; ++k) {
                float v = u(rng);
                uint32_t b; std::memcpy(&b, &v, 4);
                std::printf("%u%s", b, k < 2 ? ", " : "");
            }
            std::printf("]}%s", s == 0 ? ", " : "");
        }
        std::printf("]}%s\n", i < np_ - 1 ? "," : "");
    }
    std::printf("  ]\n}\n");
    return 0;
}
