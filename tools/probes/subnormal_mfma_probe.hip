// Does v_mfma_f32_32x32x16_f16 keep products whose f16 operands are subnormal? (dev probe, round 6)
// One wave; A = a and B = b in every lane, C = 0: each output = 16 a b exactly when every product is kept.
// Build: hipcc --offload-arch=gfx950 -O2 subnormal_mfma_probe.hip -o /tmp/snp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void probe(const unsigned short* ab, float* out, int ncase) {
    const int lane = threadIdx.x;
    for (int c = 0; c < ncase; ++c) {
        half8 a, b;
        for (int i = 0; i < 8; ++i) {
            a[i] = __builtin_bit_cast(_Float16, ab[2 * c]);
            b[i] = __builtin_bit_cast(_Float16, ab[2 * c + 1]);
        }
        f32x16 acc = {};
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
        if (lane == 0) out[c] = acc[0];
    }
}

int main() {
    // (a, b) f16 bit patterns: 2^-24 (0x0001), 2^-20 (0x0010), 2^-15 (0x0200), 255 * 2^-24 (0x00ff),
    // 2^-14 (0x0400, smallest normal), 1.0 (0x3c00), 2^-11 (0x1000)
    const unsigned short cases[][2] = {{0x0001, 0x3c00}, {0x0001, 0x0001}, {0x00ff, 0x0200}, {0x0010, 0x0010},
                                       {0x00ff, 0x0400}, {0x00ff, 0x1000}, {0x0200, 0x0200}, {0x03ff, 0x03ff}};
    const int n = sizeof(cases) / sizeof(cases[0]);
    unsigned short* d_ab;
    float* d_out;
    hipMalloc(&d_ab, sizeof(cases));
    hipMalloc(&d_out, n * sizeof(float));
    hipMemcpy(d_ab, cases, sizeof(cases), hipMemcpyHostToDevice);
    probe<<<1, 64>>>(d_ab, d_out, n);
    float out[16];
    hipMemcpy(out, d_out, n * sizeof(float), hipMemcpyDeviceToHost);
    for (int c = 0; c < n; ++c) {
        auto f = [](unsigned short h) {
            const int e = (h >> 10) & 31, m = h & 1023;
            return e ? std::ldexp(1.0 + m / 1024.0, e - 15) : std::ldexp((double)m, -24);
        };
        const double want = 16.0 * f(cases[c][0]) * f(cases[c][1]);
        printf("a=0x%04x b=0x%04x  mfma=%.9g  exact=%.9g  %s\n", cases[c][0], cases[c][1], out[c], want,
               out[c] == (float)want ? "kept" : (out[c] == 0.f ? "DROPPED" : "differs"));
    }
    hipFree(d_ab);
    hipFree(d_out);
    return 0;
}
