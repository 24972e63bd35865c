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

}  // namespace

extern "C" int ppox_gather_rows(const void* src, int64_t T, int64_t N, int64_t row_bytes, int64_t src_row_stride,
                                const int64_t* idx, int64_t nrows, void* dst, void* stream) {
    PPOX_REQUIRE(src && idx && dst, "ppox_gather_rows: null pointer");
    PPOX_REQUIRE(T > 0 && N > 0 && row_bytes > 0 && src_row_stride >= row_bytes && nrows >= 0,
                 "ppox_gather_rows: bad sizes");
    if (nrows == 0) return PPOX_OK;
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
