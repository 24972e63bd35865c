// K2/K3 — running moments (util.py:9-44) and observation normalisation
// (ppo.py:111-118), plus the intrinsic-reward scaling of ppo.py:394-398.
//
// u8 feature batches (Atari frames): per-column integer sums S = sum x and
// Q = sum x^2 are exact, so they are accumulated in parallel over row chunks
// in any order (chunk partials to a caller workspace, reduced in a fixed order;
// no atomics).  mean = S / n is then bit-identical to numpy's float64 mean;
// var = (Q - 2 m S + n m^2) / n is the exact sum of squared deviations about
// the rounded mean, within ~1e-15 relative of numpy's sequential float64 sum.
// f32 feature batches (MLP envs, D > 1): one lane per column, rows summed
// sequentially in f32 — numpy's own order for an axis-0 reduction, so the batch
// moments are bit-identical.  Scalar streams (int_rew_rms, (N,) f32): numpy's
// pairwise float32 summation reproduced exactly (leaves of <= 128 elements with
// 8 accumulators, combined in the recursion's order).
// The Chan merge into the float64 state follows util.py:30-44 op for op.
#include <algorithm>

#include "common.h"

namespace {

// m_b = batch_var * batch_count is passed in: numpy evaluates it in the batch
// variance's dtype (float32 for float32 batches: np.float32 * Python int stays
// f32 under NEP 50; float64 for uint8 batches), util.py:36.
__device__ inline void chan_merge(double& mean, double& var, double count, double bmean, double m_b, double bcount) {
    // util.py:31-44, same association as the Python expressions
    const double delta = bmean - mean;
    const double tot = count + bcount;
    const double new_mean = mean + delta * bcount / tot;
    const double m_a = var * count;
    const double m2 = m_a + m_b + delta * delta * count * bcount / (count + bcount);
    mean = new_mean;
    var = m2 / (count + bcount);
}

// ---- u8 columns -------------------------------------------------------------
constexpr int ROWS_PER_CHUNK = 64;

__global__ void __launch_bounds__(256) u8_chunk_sums(const uint8_t* __restrict__ x, long long rows, long long cols,
                                                     long long row_stride, unsigned long long* __restrict__ ws) {
    const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= cols) return;
    const long long r0 = (long long)blockIdx.y * ROWS_PER_CHUNK;
    const long long r1 = min(rows, r0 + ROWS_PER_CHUNK);
    unsigned s = 0, q = 0;  // <= 64*255 and 64*65025: fit in 32 bits
    for (long long r = r0; r < r1; ++r) {
        const unsigned v = x[r * row_stride + c];
        s += v;
        q += v * v;
    }
    ws[(blockIdx.y * cols + c) * 2 + 0] = s;
    ws[(blockIdx.y * cols + c) * 2 + 1] = q;
}

__global__ void __launch_bounds__(256) u8_finalize(const unsigned long long* __restrict__ ws, int nchunks,
                                                   long long rows, long long cols, double* __restrict__ mean,
                                                   double* __restrict__ var, double count,
                                                   double* __restrict__ bmean_out, double* __restrict__ bvar_out) {
    const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= cols) return;
    unsigned long long S = 0, Q = 0;
    for (int k = 0; k < nchunks; ++k) {
        S += ws[((long long)k * cols + c) * 2 + 0];
        Q += ws[((long long)k * cols + c) * 2 + 1];
    }
    const double n = (double)rows;
    const double m = (double)S / n;
    const double ssd = ((double)Q - 2.0 * m * (double)S) + n * m * m;
    const double bvar = (ssd > 0 ? ssd : 0.0) / n;
    if (bmean_out) bmean_out[c] = m;
    if (bvar_out) bvar_out[c] = bvar;
    if (mean && var) {
        double mu = mean[c], vv = var[c];
        chan_merge(mu, vv, count, m, bvar * n, n);
        mean[c] = mu;
        var[c] = vv;
    }
}

// ---- f32 columns (sequential rows, numpy axis-0 order) ----------------------
__global__ void __launch_bounds__(256) f32_columns(const float* __restrict__ x, long long rows, long long cols,
                                                   long long row_stride, double* __restrict__ mean,
                                                   double* __restrict__ var, double count) {
    const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= cols) return;
    float s = 0.f;
    for (long long r = 0; r < rows; ++r) s = s + x[r * row_stride + c];
    const float m = s / (float)rows;
    float q = 0.f;
    for (long long r = 0; r < rows; ++r) {
        const float d = x[r * row_stride + c] - m;
        q = q + d * d;
    }
    const float bv = q / (float)rows;
    double mu = mean[c], vv = var[c];
    chan_merge(mu, vv, count, (double)m, (double)(bv * (float)rows), (double)rows);
    mean[c] = mu;
    var[c] = vv;
}

// ---- numpy pairwise float32 sum (single block) ------------------------------
constexpr int PW_BLOCK = 128;
constexpr int MAX_LEAVES = 4096;

struct Frame {
    int off, n, state;
};

// leaf: numpy's 8-accumulator loop for 8 <= n <= 128, plain loop below 8
// (T = float for float32 arrays, double for float64 ones: numpy's pairwise_sum is
// the same algorithm for both)
template <typename T = float, typename F>
__device__ T pw_leaf(F get, int off, int n) {
    if (n < 8) {
        T res = 0;
        for (int i = 0; i < n; ++i) res = res + get(off + i);
        return res;
    }
    T r[8];
    for (int j = 0; j < 8; ++j) r[j] = get(off + j);
    int i = 8;
    for (; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; ++j) r[j] = r[j] + get(off + i + j);
    T res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res = res + get(off + i);
    return res;
}

// Enumerate leaves (thread 0), sum them in parallel, combine in recursion order (thread 0).
template <typename T = float, typename F>
__device__ T pairwise_sum_block(F get, int n, int* leaf_off, int* leaf_len, T* leaf_sum, int* nleaves_sh) {
    if (threadIdx.x == 0) {
        Frame st[40];
        int sp = 0, nl = 0;
        st[sp++] = Frame{0, n, 0};
        while (sp) {
            Frame f = st[--sp];
            if (f.n <= PW_BLOCK) {
                leaf_off[nl] = f.off;
                leaf_len[nl] = f.n;
                ++nl;
                continue;
            }
            int n2 = f.n / 2;
            n2 -= n2 % 8;
            st[sp++] = Frame{f.off + n2, f.n - n2, 0};  // right pushed first -> left visited first
            st[sp++] = Frame{f.off, n2, 0};
        }
        *nleaves_sh = nl;
    }
    __syncthreads();
    const int nl = *nleaves_sh;
    for (int k = threadIdx.x; k < nl; k += blockDim.x) leaf_sum[k] = pw_leaf<T>(get, leaf_off[k], leaf_len[k]);
    __syncthreads();
    T result = 0;
    if (threadIdx.x == 0) {
        // post-order combine with a value stack
        Frame st[40];
        T vs[40];
        int sp = 0, vp = 0, k = 0;
        st[sp++] = Frame{0, n, 0};
        while (sp) {
            Frame& f = st[sp - 1];
            if (f.n <= PW_BLOCK) {
                vs[vp++] = leaf_sum[k++];
                --sp;
                continue;
            }
            int n2 = f.n / 2;
            n2 -= n2 % 8;
            if (f.state == 0) {
                f.state = 1;
                st[sp++] = Frame{f.off, n2, 0};
            } else if (f.state == 1) {
                f.state = 2;
                st[sp++] = Frame{f.off + n2, f.n - n2, 0};
            } else {
                const T b = vs[--vp], a = vs[--vp];
                vs[vp++] = a + b;
                --sp;
            }
        }
        result = vs[0];
    }
    return result;  // valid in thread 0 only
}

__global__ void __launch_bounds__(256) scalar_rms_scale(float* __restrict__ x, int n, double* __restrict__ mean,
                                                        double* __restrict__ var, double count, int scale_inplace) {
    __shared__ int leaf_off[MAX_LEAVES], leaf_len[MAX_LEAVES];
    __shared__ float leaf_sum[MAX_LEAVES];
    __shared__ int nl;
    __shared__ float bm_sh;
    __shared__ double denom_sh;
    // batch mean (np.mean: pairwise f32 sum / n)
    float s = pairwise_sum_block([&](int i) { return x[i]; }, n, leaf_off, leaf_len, leaf_sum, &nl);
    if (threadIdx.x == 0) bm_sh = s / (float)n;
    __syncthreads();
    const float bm = bm_sh;
    // batch var (np.var: (x - mean)^2 in f32, pairwise sum / n)
    float q = pairwise_sum_block(
        [&](int i) {
            const float d = x[i] - bm;
            return d * d;
        },
        n, leaf_off, leaf_len, leaf_sum, &nl);
    if (threadIdx.x == 0) {
        const float bv = q / (float)n;
        double mu = *mean, vv = *var;
        chan_merge(mu, vv, count, (double)bm, (double)(bv * (float)n), (double)n);
        *mean = mu;
        *var = vv;
        denom_sh = sqrt(vv) + 1e-08;  // ppo.py:398
    }
    __syncthreads();
    if (scale_inplace) {
        const double d = denom_sh;
        for (int i = threadIdx.x; i < n; i += blockDim.x) x[i] = (float)((double)x[i] / d);
    }
}

// ---- normalize_obs (ppo.py:117): f32(clip((x - mean) / sqrt(var + 1e-10), -5, 5)) in f64;
// SB3 VecNormalize.normalize_obs: eps 1e-8, clip 10
template <typename T>
__global__ void __launch_bounds__(256) normalize_kernel(const T* __restrict__ x, long long rows, long long cols,
                                                        long long row_stride, const double* __restrict__ mean,
                                                        const double* __restrict__ var, float* __restrict__ out,
                                                        double eps = 1e-10, double clip = 5.0) {
    const long long total = rows * cols;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const long long r = i / cols, c = i - r * cols;
        const double y = ((double)x[r * row_stride + c] - mean[c]) / sqrt(var[c] + eps);
        out[i] = (float)fmin(fmax(y, -clip), clip);
    }
}

// ---- SB3 VecNormalize reward path (VecNormalize.step_wait, 0.x series):
//   ret = ret * gamma + reward                 (float64 returns, float32 rewards)
//   ret_rms.update(ret)                        (np.mean / np.var of a float64 array:
//                                               pairwise float64 sums; Chan merge)
//   reward = clip(reward / sqrt(ret_rms.var + eps), -clip, clip)   (float64 -> the f32 buffer)
//   ret[dones] = 0
// One block (the env count per rank is a few thousand at most).
__global__ void __launch_bounds__(256) vecnorm_reward_kernel(float* __restrict__ rew, const uint8_t* __restrict__ dones,
                                                             double* __restrict__ ret, int n, double gamma,
                                                             double* __restrict__ mean, double* __restrict__ var,
                                                             double count, double eps, double clip, int update) {
    __shared__ int leaf_off[MAX_LEAVES], leaf_len[MAX_LEAVES];
    __shared__ double leaf_sum[MAX_LEAVES];
    __shared__ int nl;
    __shared__ double bm_sh, denom_sh;
    if (update) {
        for (int i = threadIdx.x; i < n; i += blockDim.x) ret[i] = ret[i] * gamma + (double)rew[i];
        __syncthreads();
        const double s = pairwise_sum_block<double>([&](int i) { return ret[i]; }, n, leaf_off, leaf_len, leaf_sum, &nl);
        if (threadIdx.x == 0) bm_sh = s / (double)n;
        __syncthreads();
        const double bm = bm_sh;
        const double q = pairwise_sum_block<double>(
            [&](int i) {
                const double d = ret[i] - bm;
                return d * d;
            },
            n, leaf_off, leaf_len, leaf_sum, &nl);
        if (threadIdx.x == 0) {
            const double bv = q / (double)n;
            double mu = *mean, vv = *var;
            chan_merge(mu, vv, count, bm, bv * (double)n, (double)n);
            *mean = mu;
            *var = vv;
        }
    }
    if (threadIdx.x == 0) denom_sh = sqrt(*var + eps);
    __syncthreads();
    const double d = denom_sh;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const double r = (double)rew[i] / d;
        rew[i] = (float)fmin(fmax(r, -clip), clip);
        if (dones && dones[i]) ret[i] = 0.0;
    }
}

}  // namespace

extern "C" int64_t ppox_rms_u8_workspace_bytes(int64_t rows, int64_t cols) {
    const int64_t nchunks = (rows + ROWS_PER_CHUNK - 1) / ROWS_PER_CHUNK;
    return nchunks * cols * 2 * (int64_t)sizeof(unsigned long long);
}

extern "C" int ppox_rms_update_u8(const uint8_t* x, int64_t rows, int64_t cols, int64_t row_stride, double* mean,
                                  double* var, double count, void* workspace, int64_t workspace_bytes,
                                  double* batch_mean, double* batch_var, void* stream) {
    PPOX_REQUIRE(x && workspace, "ppox_rms_update_u8: null pointer");
    PPOX_REQUIRE(rows > 0 && cols > 0 && row_stride >= cols, "ppox_rms_update_u8: bad sizes");
    PPOX_REQUIRE(workspace_bytes >= ppox_rms_u8_workspace_bytes(rows, cols), "ppox_rms_update_u8: workspace too small");
    PPOX_REQUIRE((mean == nullptr) == (var == nullptr), "ppox_rms_update_u8: mean/var must both be given");
    const int nchunks = (int)((rows + ROWS_PER_CHUNK - 1) / ROWS_PER_CHUNK);
    PPOX_REQUIRE(nchunks < 65536, "ppox_rms_update_u8: too many rows");
    hipStream_t s = ppox::as_stream(stream);
    auto* ws = reinterpret_cast<unsigned long long*>(workspace);
    u8_chunk_sums<<<dim3(ppox::ceil_div(cols, 256), nchunks), 256, 0, s>>>(x, rows, cols, row_stride, ws);
    u8_finalize<<<ppox::ceil_div(cols, 256), 256, 0, s>>>(ws, nchunks, rows, cols, mean, var, count, batch_mean,
                                                          batch_var);
    PPOX_LAUNCHED("ppox_rms_update_u8");
}

extern "C" int ppox_rms_update_f32(const float* x, int64_t rows, int64_t cols, int64_t row_stride, double* mean,
                                   double* var, double count, void* stream) {
    PPOX_REQUIRE(x && mean && var, "ppox_rms_update_f32: null pointer");
    PPOX_REQUIRE(rows > 0 && cols > 0 && row_stride >= cols, "ppox_rms_update_f32: bad sizes");
    hipStream_t s = ppox::as_stream(stream);
    if (cols == 1) {
        // a single column is reduced by numpy along a contiguous axis: pairwise
        PPOX_REQUIRE(row_stride == 1 && rows <= (int64_t)MAX_LEAVES * 64, "ppox_rms_update_f32: unsupported 1-col");
        scalar_rms_scale<<<1, 256, 0, s>>>(const_cast<float*>(x), (int)rows, mean, var, count, 0);
    } else {
        f32_columns<<<ppox::ceil_div(cols, 256), 256, 0, s>>>(x, rows, cols, row_stride, mean, var, count);
    }
    PPOX_LAUNCHED("ppox_rms_update_f32");
}

extern "C" int ppox_rms_scale_int_rewards(float* int_rewards, int64_t n, double* mean, double* var, double count,
                                          void* stream) {
    PPOX_REQUIRE(int_rewards && mean && var, "ppox_rms_scale_int_rewards: null pointer");
    PPOX_REQUIRE(n > 0 && n <= (int64_t)MAX_LEAVES * 64, "ppox_rms_scale_int_rewards: n=%lld unsupported",
                 (long long)n);
    scalar_rms_scale<<<1, 256, 0, ppox::as_stream(stream)>>>(int_rewards, (int)n, mean, var, count, 1);
    PPOX_LAUNCHED("ppox_rms_scale_int_rewards");
}

extern "C" int ppox_normalize_obs_u8(const uint8_t* x, int64_t rows, int64_t cols, int64_t row_stride,
                                     const double* mean, const double* var, float* out, void* stream) {
    if (rows == 0) return PPOX_OK;  // empty shard / minibatch: no pointers to check
    PPOX_REQUIRE(x && mean && var && out, "ppox_normalize_obs_u8: null pointer");
    PPOX_REQUIRE(rows >= 0 && cols > 0 && row_stride >= cols, "ppox_normalize_obs_u8: bad sizes");
    const long long total = rows * cols;
    const unsigned grid = (unsigned)std::min<long long>(ppox::ceil_div(total, 256), 4096);
    normalize_kernel<uint8_t><<<grid, 256, 0, ppox::as_stream(stream)>>>(x, rows, cols, row_stride, mean, var, out);
    PPOX_LAUNCHED("ppox_normalize_obs_u8");
}

extern "C" int ppox_normalize_obs_f32(const float* x, int64_t rows, int64_t cols, int64_t row_stride,
                                      const double* mean, const double* var, float* out, void* stream) {
    if (rows == 0) return PPOX_OK;  // empty shard / minibatch: no pointers to check
    PPOX_REQUIRE(x && mean && var && out, "ppox_normalize_obs_f32: null pointer");
    PPOX_REQUIRE(rows >= 0 && cols > 0 && row_stride >= cols, "ppox_normalize_obs_f32: bad sizes");
    const long long total = rows * cols;
    const unsigned grid = (unsigned)std::min<long long>(ppox::ceil_div(total, 256), 4096);
    normalize_kernel<float><<<grid, 256, 0, ppox::as_stream(stream)>>>(x, rows, cols, row_stride, mean, var, out);
    PPOX_LAUNCHED("ppox_normalize_obs_f32");
}

extern "C" int ppox_normalize_obs_f32_ex(const float* x, int64_t rows, int64_t cols, int64_t row_stride,
                                         const double* mean, const double* var, double eps, double clip, float* out,
                                         void* stream) {
    if (rows == 0) return PPOX_OK;  // empty shard / minibatch: no pointers to check
    PPOX_REQUIRE(x && mean && var && out && rows >= 0 && cols > 0 && row_stride >= cols,
                 "ppox_normalize_obs_f32_ex: bad arguments");
    const long long total = rows * cols;
    const unsigned blocks = (unsigned)std::min<long long>((total + 255) / 256, 8192);
    normalize_kernel<float><<<blocks, 256, 0, ppox::as_stream(stream)>>>(x, rows, cols, row_stride, mean, var, out, eps,
                                                                         clip);
    PPOX_LAUNCHED("ppox_normalize_obs_f32_ex");
}

extern "C" int ppox_vecnorm_reward(float* rewards, const uint8_t* dones, double* ret, int64_t n, double gamma,
                                   double* mean, double* var, double count, double eps, double clip, int32_t update,
                                   void* stream) {
    PPOX_REQUIRE(rewards && ret && mean && var && n > 0, "ppox_vecnorm_reward: bad arguments");
    PPOX_REQUIRE(n <= (int64_t)MAX_LEAVES * PW_BLOCK, "ppox_vecnorm_reward: too many envs for one block");
    vecnorm_reward_kernel<<<1, 256, 0, ppox::as_stream(stream)>>>(rewards, dones, ret, (int)n, gamma, mean, var, count,
                                                                  eps, clip, update);
    PPOX_LAUNCHED("ppox_vecnorm_reward");
}
