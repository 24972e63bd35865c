// K1 — GAE(lambda) backward scan, bit-identical to the reference's numpy loop
// (buffer.py:203-230 one stream; buffer.py:321-362 two streams).
//
// Layout: step-major (T, N) rows, so at every step the lanes of a wave read
// consecutive envs: coalesced.  Each lane owns EPL consecutive envs (EPL = 4:
// 16-byte loads/stores and four independent recurrences for ILP; EPL = 1 for
// ragged/unaligned N or when N is too small to fill the chip).  The recurrence
// is sequential in t per env — the only order that reproduces the reference's
// rounding bit-for-bit — and independent across envs, so the chip-wide
// parallelism is N / EPL lanes.
//
// Exact arithmetic (see oracle/gae.py):
//   gv    = f32(gamma) * next_value                      (f32 multiply)
//   delta = (f64(r) + f64(gv) * nnt) - f64(v)            (f64, nnt = 1 - done)
//   carry = delta + (gl * nnt) * carry                   (f64, gl = gamma*lam in f64)
//   adv   = f32(carry);  ret = adv + v                   (f32)
// intrinsic stream (f32 only, no done mask):
//   d = (ir + f32(int_gamma) * niv) - iv ; carry = d + f32(int_gamma*lam) * carry
// FP contraction is disabled for this file (Makefile: -ffp-contract=off) — an
// fma would change the rounding.
#include "common.h"

namespace {

template <int EPL>
struct Vec;
template <>
struct Vec<1> {
    using f = float;
    using u8 = uint8_t;
};
template <>
struct Vec<4> {
    using f = float4;
    using u8 = uchar4;
};

__device__ inline float get(const float& v, int) { return v; }
__device__ inline float get(const float4& v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }
__device__ inline uint8_t get(const uint8_t& v, int) { return v; }
__device__ inline uint8_t get(const uchar4& v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }
__device__ inline void put(float& v, int, float x) { v = x; }
__device__ inline void put(float4& v, int k, float x) {
    if (k == 0) v.x = x; else if (k == 1) v.y = x; else if (k == 2) v.z = x; else v.w = x;
}

template <int EPL, bool DUAL>
__global__ void __launch_bounds__(256) gae_kernel(
    const float* __restrict__ rew, const float* __restrict__ val, const uint8_t* __restrict__ done,
    const float* __restrict__ last_v, const uint8_t* __restrict__ last_done,
    const float* __restrict__ irew, const float* __restrict__ ival, const float* __restrict__ last_iv,
    int T, long long N, float g32, double gl, float ig32, float igl32,
    float* __restrict__ adv, float* __restrict__ ret, float* __restrict__ iadv, float* __restrict__ iret) {
    using VF = typename Vec<EPL>::f;
    using VU = typename Vec<EPL>::u8;
    const long long lane = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (lane * EPL >= N) return;
    const long long L = N / EPL;  // row length in vector units
    const VF* R = reinterpret_cast<const VF*>(rew) + lane;
    const VF* V = reinterpret_cast<const VF*>(val) + lane;
    const VU* Dn = reinterpret_cast<const VU*>(done) + lane;
    VF* A = reinterpret_cast<VF*>(adv) + lane;
    VF* RT = reinterpret_cast<VF*>(ret) + lane;

    double carry[EPL], nnt[EPL];
    float nv[EPL];
    {
        const VF lv = reinterpret_cast<const VF*>(last_v)[lane];
        const VU ld = reinterpret_cast<const VU*>(last_done)[lane];
#pragma unroll
        for (int k = 0; k < EPL; ++k) {
            carry[k] = 0.0;
            nv[k] = get(lv, k);
            nnt[k] = 1.0 - (double)get(ld, k);
        }
    }
    // intrinsic stream state
    float icarry[EPL], niv[EPL];
    if constexpr (DUAL) {
        const VF liv = reinterpret_cast<const VF*>(last_iv)[lane];
#pragma unroll
        for (int k = 0; k < EPL; ++k) niv[k] = get(liv, k);
    }

#pragma unroll 4
    for (int t = T - 1; t >= 0; --t) {
        const long long o = (long long)t * L;
        const VF r = R[o];
        const VF v = V[o];
        const VU d = Dn[o];
        VF a_out, r_out;
#pragma unroll
        for (int k = 0; k < EPL; ++k) {
            const float vk = get(v, k);
            const float gv = g32 * nv[k];
            const double delta = ((double)get(r, k) + (double)gv * nnt[k]) - (double)vk;
            carry[k] = delta + (gl * nnt[k]) * carry[k];
            const float a = (float)carry[k];
            put(a_out, k, a);
            put(r_out, k, a + vk);
            nv[k] = vk;
            nnt[k] = 1.0 - (double)get(d, k);
        }
        A[o] = a_out;
        RT[o] = r_out;
        if constexpr (DUAL) {
            const VF ir = reinterpret_cast<const VF*>(irew)[lane + o];
            const VF iv = reinterpret_cast<const VF*>(ival)[lane + o];
            VF ia_out, ir_out;
#pragma unroll
            for (int k = 0; k < EPL; ++k) {
                const float ivk = get(iv, k);
                const float dlt = (get(ir, k) + ig32 * niv[k]) - ivk;
                icarry[k] = (t == T - 1) ? (dlt + 0.0f) : (dlt + igl32 * icarry[k]);
                put(ia_out, k, icarry[k]);
                put(ir_out, k, icarry[k] + ivk);
                niv[k] = ivk;
            }
            reinterpret_cast<VF*>(iadv)[lane + o] = ia_out;
            reinterpret_cast<VF*>(iret)[lane + o] = ir_out;
        }
    }
}

template <bool DUAL>
int launch_gae(const float* rew, const float* val, const uint8_t* done, const float* last_v,
               const uint8_t* last_done, const float* irew, const float* ival, const float* last_iv,
               int64_t T, int64_t N, double gamma, double int_gamma, double lam, float* adv, float* ret,
               float* iadv, float* iret, void* stream, const char* name) {
    PPOX_REQUIRE(T > 0 && N > 0, "%s: T=%lld N=%lld must be positive", name, (long long)T, (long long)N);
    PPOX_REQUIRE(T < (1LL << 31), "%s: T too large", name);
    PPOX_REQUIRE(rew && val && done && last_v && last_done && adv && ret, "%s: null pointer", name);
    if (DUAL) PPOX_REQUIRE(irew && ival && last_iv && iadv && iret, "%s: null intrinsic pointer", name);
    const float g32 = (float)gamma;
    const double gl = gamma * lam;
    const float ig32 = (float)int_gamma;
    const float igl32 = (float)(int_gamma * lam);
    hipStream_t s = ppox::as_stream(stream);
    // EPL=4 needs 16-byte alignment of every row; only worth it when it still
    // leaves >= 2 waves per CU worth of lanes (N/4 >= 32768).
    bool vec4 = (N % 4 == 0) && (N / 4 >= 32768);
    const void* ptrs[] = {rew, val, last_v, adv, ret, irew, ival, last_iv, iadv, iret};
    for (const void* p : ptrs)
        if (p && !ppox::aligned16(p)) vec4 = false;
    if (reinterpret_cast<uintptr_t>(done) % 4 || reinterpret_cast<uintptr_t>(last_done) % 4) vec4 = false;
    if (vec4) {
        const long long lanes = N / 4;
        const int bs = 256;
        gae_kernel<4, DUAL><<<ppox::ceil_div(lanes, bs), bs, 0, s>>>(
            rew, val, done, last_v, last_done, irew, ival, last_iv, (int)T, N, g32, gl, ig32, igl32, adv,
            ret, iadv, iret);
    } else {
        // small N: 64-thread blocks spread the few waves over as many CUs as possible
        const int bs = N >= 65536 ? 256 : 64;
        gae_kernel<1, DUAL><<<ppox::ceil_div(N, bs), bs, 0, s>>>(
            rew, val, done, last_v, last_done, irew, ival, last_iv, (int)T, N, g32, gl, ig32, igl32, adv,
            ret, iadv, iret);
    }
    PPOX_LAUNCHED(name);
}

}  // namespace

extern "C" int ppox_gae(const float* rewards, const float* values, const uint8_t* dones,
                        const float* last_value, const uint8_t* last_done, int64_t T, int64_t N,
                        double gamma, double lam, float* advantages, float* returns, void* stream) {
    return launch_gae<false>(rewards, values, dones, last_value, last_done, nullptr, nullptr, nullptr, T, N,
                             gamma, 0.0, lam, advantages, returns, nullptr, nullptr, stream, "ppox_gae");
}

extern "C" int ppox_gae_dual(const float* rewards, const float* values, const uint8_t* dones,
                             const float* last_value, const uint8_t* last_done, const float* int_rewards,
                             const float* int_values, const float* last_int_value, int64_t T, int64_t N,
                             double gamma, double int_gamma, double lam, float* advantages, float* returns,
                             float* int_advantages, float* int_returns, void* stream) {
    return launch_gae<true>(rewards, values, dones, last_value, last_done, int_rewards, int_values,
                            last_int_value, T, N, gamma, int_gamma, lam, advantages, returns, int_advantages,
                            int_returns, stream, "ppox_gae_dual");
}
