// Optimiser step over the FLAT parameter/gradient buffers:
//   clip_grad_norm_(params, max_norm)   ppo.py:243 (torch.nn.utils.clip_grad_norm_)
//   Adam(lr, betas=(0.9, 0.999), eps=1e-8).step()   ppo.py:244 (torch.optim.Adam)
// All parameters of a network live in one contiguous f32 buffer (and their
// gradients in another), so the data-parallel all-reduce is one bucket and the
// update is one streaming pass: read p, g, m, v; write p, m, v (28 B/param).
//
// torch semantics kept: total_norm = ||g||_2 over all parameters;
// coef = max_norm / (total_norm + 1e-6) clamped to <= 1 and ALWAYS multiplied
// in; m.lerp_(g, 1-beta1); v = v*beta2 + (1-beta2)*g*g;
// p += -step_size * m / (sqrt(v)/sqrt(bc2) + eps),  step_size = lr / bc1.
// The bias corrections depend only on the step count and are computed on the
// host in float64 exactly like torch's Python code and passed in.
#include "common.h"

namespace {

constexpr int P = PPOX_NORM_PARTIALS;

constexpr int SUMSQ_T = 1024;  // threads per partial: more loads in flight (the buffer is only ~8 MB)

__global__ void __launch_bounds__(SUMSQ_T) sumsq_kernel(const float* __restrict__ g, long long n,
                                                        double* __restrict__ partials) {
    __shared__ double red[SUMSQ_T / 64];
    double acc = 0.0;
    const long long n4 = n / 4;
    const float4* g4 = reinterpret_cast<const float4*>(g);
    // unrolled: the loads of several strides issue before the first add (same summation order)
#pragma unroll 4
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
        const float4 v = g4[i];
        acc += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
    }
    if (blockIdx.x == 0)
        for (long long i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) acc += (double)g[i] * g[i];
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < SUMSQ_T / 64; ++w) t += red[w];
        partials[blockIdx.x] = t;
    }
}

__device__ inline float adam_one(float& p, float g, float& m, float& v, float coef, float w1, float b2, float w2,
                                 float neg_step, float bc2s, float eps) {
    g = g * coef;
    m = m + w1 * (g - m);  // lerp with weight < 0.5
    v = v * b2 + w2 * g * g;
    const float denom = sqrtf(v) / bc2s + eps;
    p = p + neg_step * (m / denom);
    return g;
}

// the weight tensors whose new maxima the Adam step records (ppox_adam_step_wmax): element ranges [lo, hi) of the
// flat buffer, and their [tensor][slot] amax partials (zeroed beforehand)
constexpr int WT = PPOX_WMAX_TENSORS, WSLOTS = PPOX_WMAX_SLOTS;
struct Wmax {
    long long lo[WT], hi[WT];
    uint32_t* out;
};
// |x| into tensor t's running maximum if element e lies in its range (any tensor may be empty: lo == hi)
__device__ inline void wmax_note(const Wmax& w, float (&mx)[WT], long long e, float x) {
#pragma unroll
    for (int t = 0; t < WT; ++t)
        if (e >= w.lo[t] && e < w.hi[t]) mx[t] = fmaxf(mx[t], fabsf(x));
}

template <bool WMAX>
__global__ void __launch_bounds__(256) adam_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                                   float* __restrict__ v, long long n,
                                                   const double* __restrict__ partials, float max_norm, float w1,
                                                   float b2, float w2, float neg_step, float bc2s, float eps,
                                                   float* __restrict__ norm_out, Wmax wm) {
    // clip coefficient: every block sums the P partials in the same fixed tree order
    // (thread t loads partial t; 64-lane butterflies, then the 4 wave sums in order)
    static_assert(P == 256, "one partial per thread");
    __shared__ double red[4];
    __shared__ float coef_sh;
    float coef = 1.0f;
    if (max_norm > 0.f) {
        double s = partials[threadIdx.x];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
        __syncthreads();
        if (threadIdx.x == 0) {
            const float total = (float)sqrt((red[0] + red[1]) + (red[2] + red[3]));
            coef_sh = fminf(max_norm / (total + 1e-6f), 1.0f);
            if (blockIdx.x == 0 && norm_out) *norm_out = total;
        }
        __syncthreads();
        coef = coef_sh;
    }
    const long long n4 = n / 4;
    float4* p4 = reinterpret_cast<float4*>(p);
    float4* g4 = reinterpret_cast<float4*>(g);
    float4* m4 = reinterpret_cast<float4*>(m);
    float4* v4 = reinterpret_cast<float4*>(v);
    float mx[WT] = {};
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
        float4 pp = p4[i], gg = g4[i], mm = m4[i], vv = v4[i];
        gg.x = adam_one(pp.x, gg.x, mm.x, vv.x, coef, w1, b2, w2, neg_step, bc2s, eps);
        gg.y = adam_one(pp.y, gg.y, mm.y, vv.y, coef, w1, b2, w2, neg_step, bc2s, eps);
        gg.z = adam_one(pp.z, gg.z, mm.z, vv.z, coef, w1, b2, w2, neg_step, bc2s, eps);
        gg.w = adam_one(pp.w, gg.w, mm.w, vv.w, coef, w1, b2, w2, neg_step, bc2s, eps);
        p4[i] = pp;
        m4[i] = mm;
        v4[i] = vv;
        if (WMAX) {
            wmax_note(wm, mx, 4 * i, pp.x);
            wmax_note(wm, mx, 4 * i + 1, pp.y);
            wmax_note(wm, mx, 4 * i + 2, pp.z);
            wmax_note(wm, mx, 4 * i + 3, pp.w);
        }
    }
    if (blockIdx.x == 0)
        for (long long i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) {
            float pp = p[i], mm = m[i], vv = v[i];
            adam_one(pp, g[i], mm, vv, coef, w1, b2, w2, neg_step, bc2s, eps);
            p[i] = pp;
            m[i] = mm;
            v[i] = vv;
            if (WMAX) wmax_note(wm, mx, i, pp);
        }
    if (WMAX) {  // the workgroup's maxima into slot blockIdx mod WSLOTS of each tensor it touched
        __shared__ uint32_t wred[4][WT];
#pragma unroll
        for (int t = 0; t < WT; ++t) {
            uint32_t x = __float_as_uint(mx[t]);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o, 64));
            if ((threadIdx.x & 63) == 0) wred[threadIdx.x >> 6][t] = x;
        }
        __syncthreads();
        if (threadIdx.x < WT) {
            const int t = threadIdx.x;
            const uint32_t x = max(max(wred[0][t], wred[1][t]), max(wred[2][t], wred[3][t]));
            if (x) atomicMax(wm.out + t * WSLOTS + (blockIdx.x & (WSLOTS - 1)), x);
        }
    }
}

}  // namespace

extern "C" int ppox_grad_sumsq(const float* grads, int64_t n, double* partials, void* stream) {
    PPOX_REQUIRE(grads && partials && n > 0, "ppox_grad_sumsq: bad arguments");
    PPOX_REQUIRE(ppox::aligned16(grads), "ppox_grad_sumsq: grads must be 16-byte aligned");
    sumsq_kernel<<<P, SUMSQ_T, 0, ppox::as_stream(stream)>>>(grads, n, partials);
    PPOX_LAUNCHED("ppox_grad_sumsq");
}

namespace {
int adam_launch(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n, const double* norm_partials,
                float max_norm, double lr, double beta1, double beta2, double eps, int64_t step, float* total_norm_out,
                const Wmax* wm, void* stream, const char* name) {
    PPOX_REQUIRE(params && grads && exp_avg && exp_avg_sq && n > 0 && step >= 1, "ppox_adam_step: bad arguments");
    PPOX_REQUIRE(max_norm <= 0.f || norm_partials, "ppox_adam_step: clipping needs norm partials");
    PPOX_REQUIRE(ppox::aligned16(params) && ppox::aligned16(grads) && ppox::aligned16(exp_avg) &&
                     ppox::aligned16(exp_avg_sq),
                 "ppox_adam_step: buffers must be 16-byte aligned");
    // torch/optim/adam.py _single_tensor_adam scalar math, in Python-float (f64) precision
    const double bc1 = 1.0 - std::pow(beta1, (double)step);
    const double bc2 = 1.0 - std::pow(beta2, (double)step);
    const double step_size = lr / bc1;
    const double bc2s = std::sqrt(bc2);
    const long long n4 = n / 4;
    // one float4 per thread up to 2M params: a single round trip of loads per thread (the
    // grid-stride form with 1024 blocks took two, serialised by the loop's wait)
    const unsigned grid = (unsigned)std::max<long long>(1, std::min<long long>(ppox::ceil_div(n4, 256), 2048));
    if (wm)
        adam_kernel<true><<<grid, 256, 0, ppox::as_stream(stream)>>>(
            params, grads, exp_avg, exp_avg_sq, n, norm_partials, max_norm, (float)(1.0 - beta1), (float)beta2,
            (float)(1.0 - beta2), (float)(-step_size), (float)bc2s, (float)eps, total_norm_out, *wm);
    else
        adam_kernel<false><<<grid, 256, 0, ppox::as_stream(stream)>>>(
            params, grads, exp_avg, exp_avg_sq, n, norm_partials, max_norm, (float)(1.0 - beta1), (float)beta2,
            (float)(1.0 - beta2), (float)(-step_size), (float)bc2s, (float)eps, total_norm_out, Wmax{});
    PPOX_LAUNCHED(name);
}
}  // namespace

extern "C" int ppox_adam_step(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                              const double* norm_partials, float max_norm, double lr, double beta1, double beta2,
                              double eps, int64_t step, float* total_norm_out, void* stream) {
    return adam_launch(params, grads, exp_avg, exp_avg_sq, n, norm_partials, max_norm, lr, beta1, beta2, eps, step,
                       total_norm_out, nullptr, stream, "ppox_adam_step");
}

extern "C" int ppox_adam_step_wmax(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                                   const double* norm_partials, float max_norm, double lr, double beta1, double beta2,
                                   double eps, int64_t step, float* total_norm_out, const int64_t* ranges,
                                   uint32_t* amax_out, void* stream) {
    PPOX_REQUIRE(ranges && amax_out && ppox::aligned16(amax_out), "ppox_adam_step_wmax: bad arguments");
    Wmax wm{};
    for (int t = 0; t < WT; ++t) {
        PPOX_REQUIRE(ranges[t] >= 0 && ranges[WT + t] >= 0 && ranges[t] + ranges[WT + t] <= n,
                     "ppox_adam_step_wmax: a tensor range outside the buffer");
        wm.lo[t] = ranges[t];
        wm.hi[t] = ranges[t] + ranges[WT + t];
    }
    wm.out = amax_out;
    return adam_launch(params, grads, exp_avg, exp_avg_sq, n, norm_partials, max_norm, lr, beta1, beta2, eps, step,
                       total_norm_out, &wm, stream, "ppox_adam_step_wmax");
}
