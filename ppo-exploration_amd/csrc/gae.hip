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
struct Vec<2> {
    using f = float2;
    using u8 = uchar2;
};
template <>
struct Vec<4> {
    using f = float4;
    using u8 = uchar4;
};

__device__ inline float get(const float& v, int) { return v; }
__device__ inline float get(const float2& v, int k) { return k == 0 ? v.x : v.y; }
__device__ inline float get(const float4& v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }
__device__ inline uint8_t get(const uint8_t& v, int) { return v; }
__device__ inline uint8_t get(const uchar2& v, int k) { return k == 0 ? v.x : v.y; }
__device__ inline uint8_t get(const uchar4& v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }
__device__ inline void put(float& v, int, float x) { v = x; }
__device__ inline void put(float2& v, int k, float x) {
    if (k == 0) v.x = x; else v.y = x;
}
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

// Small-N form (N up to a few 10k envs, T <= STAGED_TMAX): a 256-thread block owns
// EB = 16 envs (8 for two streams) x all T steps.  Phase 1 (all threads): coalesced loads of the
// block's (t, env) tile, delta and the f64 decay factor (gl * nnt) per element
// into LDS.  Phase 2 (16 lanes, +16 for the intrinsic stream): the sequential
// carry chain per env reading LDS — the same operations in the same order as
// the lane-per-env form, so the result is bit-identical.  Phase 3 (all
// threads): adv / ret stores.  N / 16 blocks instead of N / 64 waves: the
// latency of the loads is paid once per block, not once per step.
template <bool DUAL>
constexpr int staged_eb() { return DUAL ? 8 : 16; }  // envs per block (LDS <= 64 KB at T = 128)
constexpr int STAGED_TMAX = 256;
constexpr int CH = 16;  // chain steps per register chunk
constexpr int STAGED_NMAX = 8192;  // measured crossover (tools/gae_sweep.py): above it the lane-per-env form wins

template <bool DUAL>
__global__ void __launch_bounds__(256) gae_staged_kernel(
    const float* __restrict__ rew, const float* __restrict__ val, const uint8_t* __restrict__ done,
    const float* __restrict__ last_v, const uint8_t* __restrict__ last_done,
    const float* __restrict__ irew, const float* __restrict__ ival, const float* __restrict__ last_iv,
    int T, long long N, float g32, double gl, float ig32, float igl32,
    float* __restrict__ adv, float* __restrict__ ret, float* __restrict__ iadv, float* __restrict__ iret) {
    constexpr int EB = staged_eb<DUAL>();
    constexpr int PER = STAGED_TMAX / (256 / EB);  // steps per thread
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double* sdelta = reinterpret_cast<double*>(smem);        // [T][EB]
    double* sdecay = sdelta + T * EB;                         // [T][EB] gl * nnt
    float* sadv = reinterpret_cast<float*>(sdecay + T * EB);  // [T][EB] adv, then ret
    float* sv = sadv + T * EB;                                // [T][EB] values
    float* sid = sv + T * EB;                                 // [T][EB] intrinsic delta (DUAL)
    float* siadv = sid + (DUAL ? T * EB : 0);                 // [T][EB] (DUAL)
    float* siv = siadv + (DUAL ? T * EB : 0);                 // [T][EB] (DUAL)
    const long long n0 = (long long)blockIdx.x * EB;
    const int e = threadIdx.x % EB, t0 = threadIdx.x / EB;
    const long long n = n0 + e;
    const bool ok = n < N;
    const long long nc = ok ? n : n0;  // clamped: loads stay in bounds, results unused
    // phase 1: every load of this thread's (t, e) elements in flight at once
    float r[PER], v[PER], nv[PER], ir[PER], iv[PER], niv[PER];
    uint8_t dn[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int t = t0 + k * (256 / EB);
        if (t < T) {
            const long long o = (long long)t * N + nc;
            const bool last = t == T - 1;
            r[k] = rew[o];
            v[k] = val[o];
            nv[k] = last ? last_v[nc] : val[o + N];
            dn[k] = last ? last_done[nc] : done[o + N];
            if constexpr (DUAL) {
                ir[k] = irew[o];
                iv[k] = ival[o];
                niv[k] = last ? last_iv[nc] : ival[o + N];
            }
        }
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int t = t0 + k * (256 / EB);
        if (t < T) {
            const double nnt = 1.0 - (double)dn[k];
            const float gv = g32 * nv[k];
            sdelta[t * EB + e] = ((double)r[k] + (double)gv * nnt) - (double)v[k];
            sdecay[t * EB + e] = gl * nnt;
            sv[t * EB + e] = v[k];
            if constexpr (DUAL) {
                sid[t * EB + e] = (ir[k] + ig32 * niv[k]) - iv[k];
                siv[t * EB + e] = iv[k];
            }
        }
    }
    __syncthreads();
    // phase 2: the carry chains (extrinsic on wave 0, intrinsic on wave 1, concurrently).
    // Each chunk of CH steps is read into registers first, so the LDS latency is paid
    // once per chunk, not once per step (a store in the loop would otherwise order
    // every next load behind it).
    if (threadIdx.x < EB) {
        double carry = 0.0;
        for (int hi = T - 1; hi >= 0; hi -= CH) {
            double dl[CH], dc[CH];
            float out[CH];
#pragma unroll
            for (int j = 0; j < CH; ++j)
                if (hi - j >= 0) {
                    dl[j] = sdelta[(hi - j) * EB + e];
                    dc[j] = sdecay[(hi - j) * EB + e];
                }
#pragma unroll
            for (int j = 0; j < CH; ++j)
                if (hi - j >= 0) {
                    carry = dl[j] + dc[j] * carry;
                    out[j] = (float)carry;
                }
#pragma unroll
            for (int j = 0; j < CH; ++j)
                if (hi - j >= 0) sadv[(hi - j) * EB + e] = out[j];
        }
    } else if (DUAL && threadIdx.x >= 64 && threadIdx.x < 64 + EB) {
        float icarry = 0.f;
        for (int hi = T - 1; hi >= 0; hi -= CH) {
            float d[CH];
#pragma unroll
            for (int j = 0; j < CH; ++j)
                if (hi - j >= 0) d[j] = sid[(hi - j) * EB + e];
#pragma unroll
            for (int j = 0; j < CH; ++j)
                if (hi - j >= 0) {
                    icarry = (hi - j == T - 1) ? (d[j] + 0.0f) : (d[j] + igl32 * icarry);
                    d[j] = icarry;
                }
#pragma unroll
            for (int j = 0; j < CH; ++j)
                if (hi - j >= 0) siadv[(hi - j) * EB + e] = d[j];
        }
    }
    __syncthreads();
    // phase 3: stores
    if (!ok) return;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int t = t0 + k * (256 / EB);
        if (t < T) {
            const long long o = (long long)t * N + n;
            const float a = sadv[t * EB + e];
            adv[o] = a;
            ret[o] = a + sv[t * EB + e];
            if constexpr (DUAL) {
                const float ia = siadv[t * EB + e];
                iadv[o] = ia;
                iret[o] = ia + siv[t * EB + e];
            }
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
    // EPL envs per lane (float4 / float2 rows): the widest that still leaves >= 65,536 lanes
    // (4 waves per CU; the sweep dipped to 0.35 of HBM at N = 131,072 with float4 lanes on 2),
    // given N % EPL == 0 and rows aligned to EPL floats
    const void* ptrs[] = {rew, val, last_v, adv, ret, irew, ival, last_iv, iadv, iret};
    auto fits = [&](int epl) {
        if (N % epl || N / epl < 65536) return false;
        for (const void* p : ptrs)
            if (p && (reinterpret_cast<uintptr_t>(p) % (4 * epl))) return false;
        return reinterpret_cast<uintptr_t>(done) % epl == 0 && reinterpret_cast<uintptr_t>(last_done) % epl == 0;
    };
    const int epl = fits(4) ? 4 : fits(2) ? 2 : 1;
    constexpr int EB = staged_eb<DUAL>();
    const size_t lds = (size_t)T * EB * (16 + 8 + (DUAL ? 12 : 0));
    if (N <= STAGED_NMAX && T <= STAGED_TMAX && lds <= 65536) {
        gae_staged_kernel<DUAL><<<ppox::ceil_div(N, EB), 256, lds, s>>>(
            rew, val, done, last_v, last_done, irew, ival, last_iv, (int)T, N, g32, gl, ig32, igl32, adv, ret,
            iadv, iret);
    } else if (epl == 4) {
        gae_kernel<4, DUAL><<<ppox::ceil_div(N / 4, 256), 256, 0, s>>>(
            rew, val, done, last_v, last_done, irew, ival, last_iv, (int)T, N, g32, gl, ig32, igl32, adv,
            ret, iadv, iret);
    } else if (epl == 2) {
        gae_kernel<2, DUAL><<<ppox::ceil_div(N / 2, 256), 256, 0, s>>>(
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
