// ds_read_b64_tr_b16 semantics probe (dev tool): LDS image s[r*16 + c] = 100*r + c (16 rows x 16
// cols of int16); lane 4q+p of each 16-lane group supplies &s[q*16 + 4p]; prints what lanes 0..15 get.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short v4s __attribute__((ext_vector_type(4)));
__global__ void k(short* o) {
    __shared__ __attribute__((aligned(16))) short s[256];
    for (int i = threadIdx.x; i < 256; i += 64) s[i] = (short)(100 * (i / 16) + i % 16);
    __syncthreads();
    const int i = threadIdx.x & 15, q = i >> 2, p = i & 3;
    v4s r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(s + q * 16 + 4 * p));
    for (int e = 0; e < 4; ++e) o[threadIdx.x * 4 + e] = r[e];
}
int main() {
    short* d;
    hipMalloc(&d, 64 * 4 * 2);
    k<<<1, 64>>>(d);
    short h[256];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int l = 0; l < 16; ++l) printf("lane %2d: %4d %4d %4d %4d\n", l, h[4 * l], h[4 * l + 1], h[4 * l + 2], h[4 * l + 3]);
    return 0;
}
