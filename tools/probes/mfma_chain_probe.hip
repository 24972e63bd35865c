// MFMA issue-rate probe (dev tool): v_mfma_f32_32x32x16_f16 throughput with one wave per SIMD as a
// function of how many independent accumulators the wave rotates through (1 = every MFMA reads the
// previous one's result as srcC).  Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_chain_probe.hip -o /tmp/mcp
#include <hip/hip_runtime.h>
#include <cstdio>

using f32x16 = __attribute__((ext_vector_type(16))) float;
using f16x8 = __attribute__((ext_vector_type(8))) _Float16;

template <int NACC>
__global__ void __launch_bounds__(256, 1) chain(float* out, int iters, float seed) {
    f16x8 a, b;
    for (int i = 0; i < 8; ++i) {
        a[i] = (_Float16)(seed * (threadIdx.x + i));
        b[i] = (_Float16)(seed * (i - (int)threadIdx.x));
    }
    f32x16 c[NACC];
    for (int k = 0; k < NACC; ++k) c[k] = (f32x16){};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 48 / NACC; ++j)
#pragma unroll
            for (int k = 0; k < NACC; ++k) c[k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c[k], 0, 0, 0);
    }
    float s = 0.f;
    for (int k = 0; k < NACC; ++k)
        for (int r = 0; r < 16; ++r) s += c[k][r];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int NACC>
void run(float* d, int cus) {
    const int iters = 2000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    chain<NACC><<<cus, 256>>>(d, 10, 1e-3f);
    hipEventRecord(e0);
    chain<NACC><<<cus, 256>>>(d, iters, 1e-3f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double per_simd = (double)iters * 48;  // MFMAs per wave (one wave per SIMD)
    const double flops = per_simd * cus * 4 * 32.0 * 32 * 16 * 2;
    printf("accumulators %2d: %.3f ms, %.2f ns per MFMA per SIMD, %.0f TF/s f16 dense\n", NACC, ms,
           ms * 1e6 / per_simd, flops / (ms * 1e-3) / 1e12);
}

int main() {
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    float* d;
    hipMalloc(&d, (size_t)cus * 256 * sizeof(float));
    run<1>(d, cus);
    run<2>(d, cus);
    run<3>(d, cus);
    run<4>(d, cus);
    run<6>(d, cus);
    run<1>(d, cus);
    hipFree(d);
    return 0;
}
