// K5 — minibatch row gather.  Replaces swap_and_flatten + fancy indexing +
// to_torch (buffer.py:41-52, 256-267, 97-109): for each env-major flat index
// i = n*T + t of the minibatch, copy the step-major row (t, n) of the rollout
// into a contiguous minibatch buffer.  The rollout is never flattened.
// One workgroup per row batch; 16-byte lanes when rows are 16-byte aligned.
#include "common.h"

namespace {

template <typename V>
__global__ void __launch_bounds__(256) gather_rows(const uint8_t* __restrict__ src, long long T, long long N,
                                                   long long row_bytes, long long src_row_stride,
                                                   const long long* __restrict__ idx, long long nrows,
                                                   uint8_t* __restrict__ dst) {
    const long long vec_per_row = row_bytes / (long long)sizeof(V);
    for (long long r = blockIdx.x; r < nrows; r += gridDim.x) {
        const long long i = idx[r];
        const long long e = (i % T) * N + (i / T);
        const V* s = reinterpret_cast<const V*>(src + e * src_row_stride);
        V* d = reinterpret_cast<V*>(dst + r * row_bytes);
        for (long long k = threadIdx.x; k < vec_per_row; k += blockDim.x) d[k] = s[k];
    }
}

// u8 -> f32 widening (the ICM encoder's input, ppo.py:629-633 / 684-688 feed float
// observations): 16 bytes in, 64 out per lane, grid-stride; HBM-bound (5 B per element)
__global__ void __launch_bounds__(256) u8_to_f32(const uint4* __restrict__ src, long long n16, float4* __restrict__ dst) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n16; i += (long long)gridDim.x * 256) {
        const uint4 v = src[i];
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q)
            dst[i * 4 + q] = make_float4((float)(w[q] & 0xFFu), (float)((w[q] >> 8) & 0xFFu),
                                         (float)((w[q] >> 16) & 0xFFu), (float)(w[q] >> 24));
    }
}

}  // namespace

extern "C" int ppox_u8_to_f32(const void* src, int64_t n, float* dst, void* stream) {
    if (n == 0) return PPOX_OK;  // empty shard / minibatch: no pointers to check
    PPOX_REQUIRE(src && dst && n >= 0 && n % 16 == 0, "ppox_u8_to_f32: n must be a multiple of 16");
    PPOX_REQUIRE(ppox::aligned16(src) && ppox::aligned16(dst), "ppox_u8_to_f32: 16B alignment");
    const long long n16 = n / 16;
    const unsigned blocks = (unsigned)std::min<long long>((n16 + 255) / 256, 8192);
    u8_to_f32<<<blocks, 256, 0, ppox::as_stream(stream)>>>(reinterpret_cast<const uint4*>(src), n16,
                                                           reinterpret_cast<float4*>(dst));
    PPOX_LAUNCHED("ppox_u8_to_f32");
}

extern "C" int ppox_gather_rows(const void* src, int64_t T, int64_t N, int64_t row_bytes, int64_t src_row_stride,
                                const int64_t* idx, int64_t nrows, void* dst, void* stream) {
    if (nrows == 0) return PPOX_OK;  // empty shard / minibatch: no pointers to check
    PPOX_REQUIRE(src && idx && dst, "ppox_gather_rows: null pointer");
    PPOX_REQUIRE(T > 0 && N > 0 && row_bytes > 0 && src_row_stride >= row_bytes && nrows >= 0,
                 "ppox_gather_rows: bad sizes");
    const unsigned grid = (unsigned)std::min<long long>(nrows, 8192);
    hipStream_t s = ppox::as_stream(stream);
    const auto* sp = reinterpret_cast<const uint8_t*>(src);
    auto* dp = reinterpret_cast<uint8_t*>(dst);
    const auto* ip = reinterpret_cast<const long long*>(idx);
    if (row_bytes % 16 == 0 && src_row_stride % 16 == 0 && ppox::aligned16(src) && ppox::aligned16(dst))
        gather_rows<uint4><<<grid, 256, 0, s>>>(sp, T, N, row_bytes, src_row_stride, ip, nrows, dp);
    else if (row_bytes % 4 == 0 && src_row_stride % 4 == 0 && !(reinterpret_cast<uintptr_t>(src) & 3) &&
             !(reinterpret_cast<uintptr_t>(dst) & 3))
        gather_rows<uint32_t><<<grid, 256, 0, s>>>(sp, T, N, row_bytes, src_row_stride, ip, nrows, dp);
    else
        gather_rows<uint8_t><<<grid, 256, 0, s>>>(sp, T, N, row_bytes, src_row_stride, ip, nrows, dp);
    PPOX_LAUNCHED("ppox_gather_rows");
}
