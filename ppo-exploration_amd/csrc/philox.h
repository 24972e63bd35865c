// Philox4x32-10 counter-based RNG (Salmon et al., SC'11).  Stateless: every
// draw is a pure function of (counter, key), so the synthetic envs and the
// action sampler are reproducible, shard-invariant (keyed by GLOBAL env index)
// and graph-replay safe.  oracle/philox.py restates it for the parity tests.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace ppox {

struct u32x4 {
    uint32_t x, y, z, w;
};

__host__ __device__ inline u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)M0 * c.x;
        const uint64_t p1 = (uint64_t)M1 * c.z;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += W0;
        k1 += W1;
    }
    return c;
}

// uniform in [0, 1) with 24 random bits (exactly representable in f32)
__host__ __device__ inline float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

}  // namespace ppox
