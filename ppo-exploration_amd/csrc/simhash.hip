// K8 — SimHash count bonus (reference buffer.py:188-200, RolloutStorage(sim_hash=True)).
//   key_n    = sign bits of A @ obs_n  (A: 16 x D f64, obs promoted to f64, bit b <- row b)
//   envs in global index order: count[key] += 1; r_n += beta / sqrt(count[key])
// The sequential dictionary update is reproduced exactly: env n's count is the
// table value before the step plus its 1-based rank among the envs of this step
// (global index order) that share its key.  The table (65,536 u32, one per key)
// is replicated on every rank and advanced with ALL envs' keys, so sharded runs
// see the same counts as one process.
#include "common.h"

namespace {

constexpr int BITS = 16;
constexpr int TILE = 1024;

__global__ void __launch_bounds__(256) simhash_keys_kernel(const float* __restrict__ obs, long long N, long long D,
                                                           long long stride, const double* __restrict__ A,
                                                           int32_t* __restrict__ keys) {
    const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const float* x = obs + n * stride;
    int32_t key = 0;
    for (int b = 0; b < BITS; ++b) {
        double s = 0.0;
        for (long long d = 0; d < D; ++d) s += A[b * D + d] * (double)x[d];
        if (s > 0.0) key |= 1 << b;
    }
    keys[n] = key;
}

__global__ void __launch_bounds__(256) simhash_bonus_kernel(const int32_t* __restrict__ keys, long long offset,
                                                            long long n_local, const uint32_t* __restrict__ counts,
                                                            double beta, float* __restrict__ rewards) {
    __shared__ int32_t tile[TILE];
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = i < n_local;
    const long long g = offset + (valid ? i : 0);
    const int32_t k = valid ? keys[g] : -1;
    // envs before this block's last env, in global order
    const long long last = offset + min(n_local, (long long)(blockIdx.x + 1) * blockDim.x) - 1;
    unsigned rank = 1;
    for (long long base = 0; base < last; base += TILE) {
        __syncthreads();
        for (int j = threadIdx.x; j < TILE; j += blockDim.x) tile[j] = base + j < last ? keys[base + j] : -2;
        __syncthreads();
        const long long hi = g - base < TILE ? g - base : TILE;  // envs j < g of this tile
        for (long long j = 0; j < hi; ++j) rank += tile[j] == k;
    }
    if (valid) rewards[i] = (float)((double)rewards[i] + beta / sqrt((double)(counts[k] + rank)));
}

__global__ void __launch_bounds__(256) simhash_count_kernel(const int32_t* __restrict__ keys, long long n,
                                                            uint32_t* __restrict__ counts) {
    const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) atomicAdd(&counts[keys[j]], 1u);  // integer: order-free
}

}  // namespace

extern "C" int ppox_simhash_keys(const float* obs, int64_t N, int64_t D, int64_t obs_stride, const double* A,
                                 int32_t* keys, void* stream) {
    if (N == 0) return PPOX_OK;  // empty shard / minibatch: no pointers to check
    PPOX_REQUIRE(obs && A && keys, "ppox_simhash_keys: null pointer");
    PPOX_REQUIRE(N >= 0 && D >= 1 && obs_stride >= D, "ppox_simhash_keys: bad sizes");
    simhash_keys_kernel<<<ppox::ceil_div(N, 256), 256, 0, ppox::as_stream(stream)>>>(obs, N, D, obs_stride, A, keys);
    PPOX_LAUNCHED("ppox_simhash_keys");
}

extern "C" int ppox_simhash_apply(const int32_t* keys_all, int64_t n_total, int64_t offset, int64_t n_local,
                                  uint32_t* counts, double beta, float* rewards, void* stream) {
    if (n_total == 0) return PPOX_OK;  // empty shard / minibatch: no pointers to check
    PPOX_REQUIRE(keys_all && counts && (rewards || n_local == 0), "ppox_simhash_apply: null pointer");
    PPOX_REQUIRE(n_total >= 0 && offset >= 0 && n_local >= 0 && offset + n_local <= n_total,
                 "ppox_simhash_apply: bad sizes");
    hipStream_t s = ppox::as_stream(stream);
    if (n_local > 0) {
        simhash_bonus_kernel<<<ppox::ceil_div(n_local, 256), 256, 0, s>>>(keys_all, offset, n_local, counts, beta,
                                                                          rewards);
        PPOX_LAUNCHED_NORET("ppox_simhash_apply");
    }
    simhash_count_kernel<<<ppox::ceil_div(n_total, 256), 256, 0, s>>>(keys_all, n_total, counts);
    PPOX_LAUNCHED("ppox_simhash_apply");
}
