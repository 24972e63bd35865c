// K4 — fused PPO minibatch loss (forward statistics + backward to the network
// outputs) and the collect-time categorical action head.
//
// Replaces (reference, per minibatch):
//   advantage normalisation       ppo.py:219 (/ :431-434 RND: both streams)
//   Categorical(probs=softmax)    models.py:52-73 (evaluate) -> log_prob, entropy
//   clipped surrogate             ppo.py:222-226
//   clipped value loss (max of means)  ppo.py:229-232 (+ :451-454 int value)
//   entropy loss + total          ppo.py:235-238 / :457-460 / :692
// and the autograd of all of that down to dL/dlogits, dL/dvalue(s).
//
// Two launches per minibatch so that data-parallel ranks can all-reduce the
// tiny partial-sum table between them:
//   ppox_ppo_loss_partials  -> f64 partials[P][8] (P = PPOX_LOSS_PARTIALS)
//   ppox_ppo_loss_backward  -> every block re-reduces the (all-reduced) table
//                              in a fixed order (deterministic), picks the
//                              max-of-means branch, writes the gradients.
// Per-element arithmetic follows torch's CPU kernels op by op in f32 (the
// reference runs torch-CPU fp32): softmax as e*(1/S), probs renormalised,
// log(clamp(p, eps, 1-eps)), min/max ties split the gradient in half, clamp
// masks inclusive.
#include "common.h"
#include "philox.h"

namespace {

constexpr int P = PPOX_LOSS_PARTIALS;
constexpr int NS = 8;  // partial columns
constexpr float F32_EPS = 1.1920928955078125e-07f;

// index map: env-major flat i -> step-major element (t*N + n)
__device__ inline long long elem(long long i, long long T, long long N) { return (i % T) * N + (i / T); }

struct Minibatch {
    const float* logits;
    const float* values;
    const float* int_values;  // nullable
    long long B;               // local rows
    int A;
    const long long* idx;
    long long T, N;
    const int32_t* actions;
    const float* old_logp;
    const float* old_values;
    const float* adv;
    const float* ret;
    const float* old_int_values;  // nullable (dual)
    const float* int_adv;
    const float* int_ret;
    const double* adv_stats;  // [4] mean, std, int mean, int std
    float clip;
};

// ---- categorical head (models.py:62-64 via torch.distributions.Categorical) ----
template <int MAXA>
struct CatRow {
    float p[MAXA], q[MAXA], c[MAXA], lp[MAXA];
    float s;  // sum of p (renormaliser)
    float ent;
};

template <int MAXA>
__device__ inline void categorical_forward(const float* zp, int A, CatRow<MAXA>& r) {
    // the row's logits loaded unconditionally first (j >= A re-reads logit A - 1, never used):
    // a load under the j < A branches below would cost a memory round trip per logit
    float z[MAXA];
#pragma unroll
    for (int j = 0; j < MAXA; ++j) z[j] = zp[j < A ? j : A - 1];
    float m = z[0];
#pragma unroll
    for (int j = 1; j < MAXA; ++j)
        if (j < A) m = fmaxf(m, z[j]);
    float S = 0.f;
#pragma unroll
    for (int j = 0; j < MAXA; ++j)
        if (j < A) {
            r.p[j] = expf(z[j] - m);
            S += r.p[j];
        }
    const float inv = 1.0f / S;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < MAXA; ++j)
        if (j < A) {
            r.p[j] = r.p[j] * inv;
            s += r.p[j];
        }
    r.s = s;
    float ent = 0.f;
#pragma unroll
    for (int j = 0; j < MAXA; ++j)
        if (j < A) {
            r.q[j] = r.p[j] / s;
            r.c[j] = fminf(fmaxf(r.q[j], F32_EPS), 1.0f - F32_EPS);
            r.lp[j] = logf(r.c[j]);
            ent += r.lp[j] * r.q[j];
        }
    r.ent = -ent;
}

struct Scalars {
    float mean, std, imean, istd;
};

__device__ inline Scalars load_stats(const double* st, bool dual) {
    Scalars s;
    s.mean = (float)st[0];
    s.std = (float)st[1];
    s.imean = dual ? (float)st[2] : 0.f;
    s.istd = dual ? (float)st[3] : 0.f;
    return s;
}

__device__ inline float norm_adv(float a, float mean, float std) { return (a - mean) / (std + 1e-8f); }

__device__ inline float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

// ---------------------------------------------------------------------------
template <int MAXA, bool DUAL>
__global__ void __launch_bounds__(256) loss_partials_kernel(Minibatch mb, double* __restrict__ partials) {
    __shared__ double red[NS][256 / 64];
    const Scalars st = load_stats(mb.adv_stats, DUAL);
    double acc[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) acc[k] = 0.0;
    for (long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x; b < mb.B; b += (long long)gridDim.x * blockDim.x) {
        const long long e = elem(mb.idx[b], mb.T, mb.N);
        CatRow<MAXA> r;
        categorical_forward<MAXA>(mb.logits + b * mb.A, mb.A, r);
        const int a = mb.actions[e];
        float lpa = 0.f;
#pragma unroll
        for (int j = 0; j < MAXA; ++j)
            if (j == a) lpa = r.lp[j];
        float advn = norm_adv(mb.adv[e], st.mean, st.std);
        if (DUAL) advn = advn + norm_adv(mb.int_adv[e], st.imean, st.istd);
        const float ratio = expf(lpa - mb.old_logp[e]);
        const float s1 = advn * ratio;
        const float s2 = advn * clampf(ratio, 1.f - mb.clip, 1.f + mb.clip);
        const float v = mb.values[b], ov = mb.old_values[e], rt = mb.ret[e];
        const float vc = ov + clampf(v - ov, -mb.clip, mb.clip);
        const float e1 = (rt - v) * (rt - v), e2 = (rt - vc) * (rt - vc);
        acc[0] += (double)fminf(s1, s2);
        acc[1] += (double)e1;
        acc[2] += (double)e2;
        acc[3] += (double)r.ent;
        if (DUAL) {
            const float iv = mb.int_values[b], oiv = mb.old_int_values[e], irt = mb.int_ret[e];
            const float ivc = oiv + clampf(iv - oiv, -mb.clip, mb.clip);
            acc[4] += (double)((irt - iv) * (irt - iv));
            acc[5] += (double)((irt - ivc) * (irt - ivc));
        }
        acc[6] += 1.0;
    }
    // wave reduce then block reduce (fixed order => deterministic)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        double x = acc[k];
        for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o, 64);
        if (lane == 0) red[k][wv] = x;
    }
    __syncthreads();
    if (threadIdx.x < NS) {
        double x = 0.0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) x += red[threadIdx.x][w];
        partials[blockIdx.x * NS + threadIdx.x] = x;
    }
}

template <int MAXA, bool DUAL>
__global__ void __launch_bounds__(256) loss_backward_kernel(Minibatch mb, const double* __restrict__ partials,
                                                            double Bglob, float ent_coef, float vf_coef,
                                                            float int_vf_coef, float scale,
                                                            float* __restrict__ dlogits, float* __restrict__ dvalues,
                                                            float* __restrict__ dint_values,
                                                            double* __restrict__ loss_accum) {
    __shared__ double tot[NS];
    if (threadIdx.x < NS) {
        double x = 0.0;
        for (int p = 0; p < P; ++p) x += partials[p * NS + threadIdx.x];
        tot[threadIdx.x] = x;
    }
    __syncthreads();
    // per-minibatch scalar losses as torch would hold them (f32 means)
    const float vl1 = (float)(tot[1] / Bglob), vl2 = (float)(tot[2] / Bglob);
    const float wA = vl1 == vl2 ? 0.5f : (vl1 > vl2 ? 1.f : 0.f);
    const float wB = vl1 == vl2 ? 0.5f : (vl2 > vl1 ? 1.f : 0.f);
    float iwA = 0.f, iwB = 0.f;
    const float ivl1 = (float)(tot[4] / Bglob), ivl2 = (float)(tot[5] / Bglob);
    if (DUAL) {
        iwA = ivl1 == ivl2 ? 0.5f : (ivl1 > ivl2 ? 1.f : 0.f);
        iwB = ivl1 == ivl2 ? 0.5f : (ivl2 > ivl1 ? 1.f : 0.f);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && loss_accum) {
        const double pl = -(double)(float)(tot[0] / Bglob);
        const double vl = (double)fmaxf(vl1, vl2);
        const double el = -(double)(float)(tot[3] / Bglob);
        const double ivl = DUAL ? (double)fmaxf(ivl1, ivl2) : 0.0;
        loss_accum[0] += pl;
        loss_accum[1] += vl;
        loss_accum[2] += el;
        loss_accum[3] += pl + (double)ent_coef * el + (double)vf_coef * vl + (DUAL ? (double)int_vf_coef * ivl : 0.0);
        loss_accum[4] += ivl;
        loss_accum[5] += 1.0;
    }
    const float invB = (float)(1.0 / Bglob);
    const float two_invB = (float)(2.0 / Bglob);
    const Scalars st = load_stats(mb.adv_stats, DUAL);
    const float g_surr = -invB * scale;
    const float g_ent = -ent_coef * invB * scale;
    const float lo = 1.f - mb.clip, hi = 1.f + mb.clip;
    for (long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x; b < mb.B; b += (long long)gridDim.x * blockDim.x) {
        const long long e = elem(mb.idx[b], mb.T, mb.N);
        const float* z = mb.logits + b * mb.A;
        CatRow<MAXA> r;
        categorical_forward<MAXA>(z, mb.A, r);
        const int a = mb.actions[e];
        float lpa = 0.f;
#pragma unroll
        for (int j = 0; j < MAXA; ++j)
            if (j == a) lpa = r.lp[j];
        float advn = norm_adv(mb.adv[e], st.mean, st.std);
        if (DUAL) advn = advn + norm_adv(mb.int_adv[e], st.imean, st.istd);
        const float ratio = expf(lpa - mb.old_logp[e]);
        const float s1 = advn * ratio;
        const float s2 = advn * clampf(ratio, lo, hi);
        const float g1 = s1 < s2 ? g_surr : (s1 == s2 ? g_surr * 0.5f : 0.f);
        const float g2 = s2 < s1 ? g_surr : (s1 == s2 ? g_surr * 0.5f : 0.f);
        const float g_ratio = g1 * advn + ((ratio >= lo && ratio <= hi) ? g2 * advn : 0.f);
        const float g_lpa = g_ratio * ratio;
        // back through log(clamp(q)), q = p / s, p = softmax(z)
        float gq[MAXA];
        float gs = 0.f;
#pragma unroll
        for (int j = 0; j < MAXA; ++j)
            if (j < mb.A) {
                const float g_lp = -g_ent * r.q[j] + (j == a ? g_lpa : 0.f);
                const float g_c = g_lp / r.c[j];
                const bool mask = r.q[j] >= F32_EPS && r.q[j] <= 1.0f - F32_EPS;
                gq[j] = -g_ent * r.lp[j] + (mask ? g_c : 0.f);
                gs += -gq[j] * (r.q[j] / r.s);
            }
        float dot = 0.f;
        float gp[MAXA];
#pragma unroll
        for (int j = 0; j < MAXA; ++j)
            if (j < mb.A) {
                gp[j] = gq[j] / r.s + gs;
                dot += gp[j] * r.p[j];
            }
        float* dz = dlogits + b * mb.A;
#pragma unroll
        for (int j = 0; j < MAXA; ++j)
            if (j < mb.A) dz[j] = r.p[j] * (gp[j] - dot);
        // value heads
        const float v = mb.values[b], ov = mb.old_values[e], rt = mb.ret[e];
        const float dv = v - ov;
        const float vc = ov + clampf(dv, -mb.clip, mb.clip);
        const float gvl = vf_coef * scale;
        float gv = wA * gvl * (-(two_invB * (rt - v)));
        if (dv >= -mb.clip && dv <= mb.clip) gv += wB * gvl * (-(two_invB * (rt - vc)));
        dvalues[b] = gv;
        if (DUAL) {
            const float iv = mb.int_values[b], oiv = mb.old_int_values[e], irt = mb.int_ret[e];
            const float div = iv - oiv;
            const float ivc = oiv + clampf(div, -mb.clip, mb.clip);
            const float givl = int_vf_coef * scale;
            float giv = iwA * givl * (-(two_invB * (irt - iv)));
            if (div >= -mb.clip && div <= mb.clip) giv += iwB * givl * (-(two_invB * (irt - ivc)));
            dint_values[b] = giv;
        }
    }
}

// per-minibatch advantage moments over the GLOBAL permutation slices
__global__ void __launch_bounds__(256) adv_stats_kernel(const float* __restrict__ adv, const float* __restrict__ iadv,
                                                        const long long* __restrict__ perm, long long total,
                                                        long long batch, long long T, long long N,
                                                        double* __restrict__ out) {
    __shared__ double red[4][4];
    const long long k = blockIdx.x;
    const long long s = k * batch, e_ = min(total, s + batch);
    double a1 = 0, a2 = 0, b1 = 0, b2 = 0;
    for (long long i = s + threadIdx.x; i < e_; i += blockDim.x) {
        const long long e = elem(perm[i], T, N);
        const double x = adv[e];
        a1 += x;
        a2 += x * x;
        if (iadv) {
            const double y = iadv[e];
            b1 += y;
            b2 += y * y;
        }
    }
    double v[4] = {a1, a2, b1, b2};
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        double x = v[q];
        for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o, 64);
        if (lane == 0) red[q][wv] = x;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double t[4];
        for (int q = 0; q < 4; ++q) t[q] = red[q][0] + red[q][1] + red[q][2] + red[q][3];
        const double n = (double)(e_ - s);
        const double m = t[0] / n, im = t[2] / n;
        // torch std: unbiased (n-1); n == 1 gives nan exactly like the reference
        const double var = (t[1] - n * m * m) / (n - 1.0), ivar = (t[3] - n * im * im) / (n - 1.0);
        out[k * 4 + 0] = m;
        out[k * 4 + 1] = sqrt(var > 0 ? var : (var == var ? 0.0 : var));
        out[k * 4 + 2] = im;
        out[k * 4 + 3] = sqrt(ivar > 0 ? ivar : (ivar == ivar ? 0.0 : ivar));
    }
}

// collect-time head: sample a ~ Categorical(probs=softmax(z)), log_prob(a)
template <int MAXA>
__global__ void __launch_bounds__(256) categorical_sample_kernel(const float* __restrict__ logits, long long N, int A,
                                                                 long long env_offset, uint64_t seed,
                                                                 long long counter, const long long* __restrict__ cbase,
                                                                 int32_t* __restrict__ actions,
                                                                 float* __restrict__ logp) {
    const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    if (cbase) counter += *cbase;  // device-resident counter (graph-captured collect)
    CatRow<MAXA> r;
    categorical_forward<MAXA>(logits + n * A, A, r);
    const ppox::u32x4 w = ppox::philox4x32_10(
        ppox::u32x4{0xA5A5A5A5u, (uint32_t)(env_offset + n), (uint32_t)counter, (uint32_t)(counter >> 32)},
        (uint32_t)seed, (uint32_t)(seed >> 32));
    // inverse CDF over the renormalised probabilities q
    const float u = ppox::u01(w.x);
    float cum = 0.f;
    int a = A - 1;
#pragma unroll
    for (int j = 0; j < MAXA; ++j)
        if (j < A - 1) {
            cum += r.q[j];
            if (u < cum && a == A - 1) a = j;
        }
    float lpa = r.lp[0];
#pragma unroll
    for (int j = 0; j < MAXA; ++j)
        if (j == a) lpa = r.lp[j];
    actions[n] = a;
    logp[n] = lpa;
}

Minibatch make_mb(const float* logits, const float* values, const float* int_values, int64_t B, int A,
                  const int64_t* idx, int64_t T, int64_t N, const int32_t* actions, const float* old_logp,
                  const float* old_values, const float* adv, const float* ret, const float* old_int_values,
                  const float* int_adv, const float* int_ret, const double* adv_stats, float clip) {
    Minibatch m;
    m.logits = logits;
    m.values = values;
    m.int_values = int_values;
    m.B = B;
    m.A = A;
    m.idx = reinterpret_cast<const long long*>(idx);
    m.T = T;
    m.N = N;
    m.actions = actions;
    m.old_logp = old_logp;
    m.old_values = old_values;
    m.adv = adv;
    m.ret = ret;
    m.old_int_values = old_int_values;
    m.int_adv = int_adv;
    m.int_ret = int_ret;
    m.adv_stats = adv_stats;
    m.clip = clip;
    return m;
}

// ---------------------------------------------------------------------------
// Box (continuous) head: Normal(tanh(mu), exp(action_log_std)) — models.py:40-46
// / :66-71 / :159-164.  The buffer's actions are f64 (buffer.py:156), so
// Normal.log_prob promotes to f64 and so do the ratio and the surrogate
// (ppo.py:222-226): those run in f64 here, and every gradient is cast back to
// f32 where it reaches an f32 tensor (loc, 2*var, log_scale), as autograd does.
// The surrogate and entropy are per action dimension (ratio (B,D) x adv (B,1)).
// ---------------------------------------------------------------------------
constexpr double LOG_SQRT_2PI = 0.91893853320467274178;  // math.log(math.sqrt(2 * math.pi))
constexpr int MAXD = 64;

struct BoxMinibatch {
    Minibatch m;              // logits = actor pre-activations (B, D); actions unused
    const float* log_std;     // (D,)
    const float* box_actions; // (T, N, D) step-major
    int D;
    double clip64;            // the Python float clip_range (f64 ratio clamp)
};

__device__ inline float box_entropy(float log_scale) {
    return (float)(0.5 + LOG_SQRT_2PI) + log_scale;  // 0.5 + 0.5*log(2*pi) + log(scale), f32
}

template <bool DUAL>
__global__ void __launch_bounds__(256) box_partials_kernel(BoxMinibatch bm, double* __restrict__ partials) {
    __shared__ double red[NS][256 / 64];
    const Minibatch& mb = bm.m;
    const Scalars st = load_stats(mb.adv_stats, DUAL);
    const int D = bm.D;
    double acc[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) acc[k] = 0.0;
    const double lo = 1.0 - bm.clip64, hi = 1.0 + bm.clip64;
    for (long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x; b < mb.B; b += (long long)gridDim.x * blockDim.x) {
        const long long e = elem(mb.idx[b], mb.T, mb.N);
        float advn = norm_adv(mb.adv[e], st.mean, st.std);
        if (DUAL) advn = advn + norm_adv(mb.int_adv[e], st.imean, st.istd);
        for (int d = 0; d < D; ++d) {
            const float loc = tanhf(mb.logits[b * D + d]);
            const float sc = expf(bm.log_std[d]);
            const float var = sc * sc, log_scale = logf(sc);
            const double diff = (double)bm.box_actions[e * D + d] - (double)loc;
            const double lp = -(diff * diff) / (double)(2.f * var) - (double)log_scale - LOG_SQRT_2PI;
            const double ratio = exp(lp - (double)mb.old_logp[e * D + d]);
            const double s1 = (double)advn * ratio;
            const double s2 = (double)advn * fmin(fmax(ratio, lo), hi);
            acc[0] += fmin(s1, s2);
            acc[3] += (double)box_entropy(log_scale);
        }
        const float v = mb.values[b], ov = mb.old_values[e], rt = mb.ret[e];
        const float vc = ov + clampf(v - ov, -mb.clip, mb.clip);
        acc[1] += (double)((rt - v) * (rt - v));
        acc[2] += (double)((rt - vc) * (rt - vc));
        if (DUAL) {
            const float iv = mb.int_values[b], oiv = mb.old_int_values[e], irt = mb.int_ret[e];
            const float ivc = oiv + clampf(iv - oiv, -mb.clip, mb.clip);
            acc[4] += (double)((irt - iv) * (irt - iv));
            acc[5] += (double)((irt - ivc) * (irt - ivc));
        }
        acc[6] += 1.0;
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        double x = acc[k];
        for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o, 64);
        if (lane == 0) red[k][wv] = x;
    }
    __syncthreads();
    if (threadIdx.x < NS) {
        double x = 0.0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) x += red[threadIdx.x][w];
        partials[blockIdx.x * NS + threadIdx.x] = x;
    }
}

// dmu (B, D) = dL/d(actor pre-activation); dls_part [P][D] f64 = this block's
// share of dL/d(action_log_std) (reduced in block order by box_logstd_reduce)
template <bool DUAL>
__global__ void __launch_bounds__(256) box_backward_kernel(BoxMinibatch bm, const double* __restrict__ partials,
                                                           double Bglob, float ent_coef, float vf_coef,
                                                           float int_vf_coef, float scale, float* __restrict__ dmu,
                                                           double* __restrict__ dls_part, float* __restrict__ dvalues,
                                                           float* __restrict__ dint_values,
                                                           double* __restrict__ loss_accum) {
    __shared__ double tot[NS];
    __shared__ double dls[4][MAXD];
    const Minibatch& mb = bm.m;
    const int D = bm.D;
    if (threadIdx.x < NS) {
        double x = 0.0;
        for (int p = 0; p < P; ++p) x += partials[p * NS + threadIdx.x];
        tot[threadIdx.x] = x;
    }
    __syncthreads();
    const double BD = Bglob * D;
    const float vl1 = (float)(tot[1] / Bglob), vl2 = (float)(tot[2] / Bglob);
    const float wA = vl1 == vl2 ? 0.5f : (vl1 > vl2 ? 1.f : 0.f);
    const float wB = vl1 == vl2 ? 0.5f : (vl2 > vl1 ? 1.f : 0.f);
    float iwA = 0.f, iwB = 0.f;
    const float ivl1 = (float)(tot[4] / Bglob), ivl2 = (float)(tot[5] / Bglob);
    if (DUAL) {
        iwA = ivl1 == ivl2 ? 0.5f : (ivl1 > ivl2 ? 1.f : 0.f);
        iwB = ivl1 == ivl2 ? 0.5f : (ivl2 > ivl1 ? 1.f : 0.f);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && loss_accum) {
        const double pl = -(tot[0] / BD);  // f64 in the reference (f64 ratio)
        const double vl = (double)fmaxf(vl1, vl2);
        const double el = -(double)(float)(tot[3] / BD);
        const double ivl = DUAL ? (double)fmaxf(ivl1, ivl2) : 0.0;
        loss_accum[0] += pl;
        loss_accum[1] += vl;
        loss_accum[2] += el;
        loss_accum[3] += pl + (double)ent_coef * el + (double)vf_coef * vl + (DUAL ? (double)int_vf_coef * ivl : 0.0);
        loss_accum[4] += ivl;
        loss_accum[5] += 1.0;
    }
    const Scalars st = load_stats(mb.adv_stats, DUAL);
    const double lo = 1.0 - bm.clip64, hi = 1.0 + bm.clip64;
    const double g_min = -(double)scale / BD;                   // d(-mean(min))
    const float g_entropy = -(ent_coef * scale) / (float)BD;   // d(ent_coef * -mean(entropy)), f32
    const float two_invB = (float)(2.0 / Bglob);
    double my_dls[MAXD];
    for (int d = 0; d < D; ++d) my_dls[d] = 0.0;
    for (long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x; b < mb.B; b += (long long)gridDim.x * blockDim.x) {
        const long long e = elem(mb.idx[b], mb.T, mb.N);
        float advn = norm_adv(mb.adv[e], st.mean, st.std);
        if (DUAL) advn = advn + norm_adv(mb.int_adv[e], st.imean, st.istd);
        for (int d = 0; d < D; ++d) {
            const float loc = tanhf(mb.logits[b * D + d]);
            const float sc = expf(bm.log_std[d]);
            const float var = sc * sc, log_scale = logf(sc);
            const float var2 = 2.f * var;
            const double diff = (double)bm.box_actions[e * D + d] - (double)loc;
            const double num = -(diff * diff);
            const double lp = num / (double)var2 - (double)log_scale - LOG_SQRT_2PI;
            const double ratio = exp(lp - (double)mb.old_logp[e * D + d]);
            const double s1 = (double)advn * ratio;
            const double rc = fmin(fmax(ratio, lo), hi);
            const double s2 = (double)advn * rc;
            const double g1 = s1 < s2 ? g_min : (s1 == s2 ? g_min * 0.5 : 0.0);
            const double g2 = s2 < s1 ? g_min : (s1 == s2 ? g_min * 0.5 : 0.0);
            const double g_ratio = g1 * (double)advn + ((ratio >= lo && ratio <= hi) ? g2 * (double)advn : 0.0);
            const double g_lp = g_ratio * ratio;
            // lp = num / var2 - log_scale - c
            const float g_var2 = (float)(-g_lp * num / ((double)var2 * (double)var2));
            const float g_log_scale = (float)(-g_lp);
            const double g_num = g_lp / (double)var2;
            const float g_loc = (float)(-(-g_num * 2.0 * diff));  // num = -(diff^2), diff = a - loc
            dmu[b * D + d] = g_loc * (1.f - loc * loc);          // tanh backward
            // scale: var = scale^2, log_scale = log(scale) (twice: log_prob and entropy)
            const float g_scale = (g_var2 * 2.f) * (2.f * sc) + g_log_scale / sc + g_entropy / sc;
            my_dls[d] += (double)(g_scale * sc);  // scale = exp(log_std): grad * result
        }
        const float v = mb.values[b], ov = mb.old_values[e], rt = mb.ret[e];
        const float dv = v - ov;
        const float vc = ov + clampf(dv, -mb.clip, mb.clip);
        const float gvl = vf_coef * scale;
        float gv = wA * gvl * (-(two_invB * (rt - v)));
        if (dv >= -mb.clip && dv <= mb.clip) gv += wB * gvl * (-(two_invB * (rt - vc)));
        dvalues[b] = gv;
        if (DUAL) {
            const float iv = mb.int_values[b], oiv = mb.old_int_values[e], irt = mb.int_ret[e];
            const float div = iv - oiv;
            const float ivc = oiv + clampf(div, -mb.clip, mb.clip);
            const float givl = int_vf_coef * scale;
            float giv = iwA * givl * (-(two_invB * (irt - iv)));
            if (div >= -mb.clip && div <= mb.clip) giv += iwB * givl * (-(two_invB * (irt - ivc)));
            dint_values[b] = giv;
        }
    }
    // block partial of d(action_log_std): wave shuffles, then waves in order
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int d = 0; d < D; ++d) {
        double x = my_dls[d];
        for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o, 64);
        if (lane == 0) dls[wv][d] = x;
    }
    __syncthreads();
    for (int d = threadIdx.x; d < D; d += blockDim.x)
        dls_part[blockIdx.x * D + d] = dls[0][d] + dls[1][d] + dls[2][d] + dls[3][d];
}

__global__ void box_logstd_reduce(const double* __restrict__ dls_part, int D, float* __restrict__ dlog_std) {
    const int d = threadIdx.x;
    if (d >= D) return;
    double x = 0.0;
    for (int p = 0; p < P; ++p) x += dls_part[p * D + d];
    dlog_std[d] = (float)x;
}

// collect-time head: a ~ Normal(tanh(mu), exp(log_std)) by Box-Muller on Philox,
// log_prob(a) in f32 (the sampled actions are f32 there, models.py:42-45)
__global__ void __launch_bounds__(256) normal_sample_kernel(const float* __restrict__ mu, const float* __restrict__ log_std,
                                                            long long N, int D, long long env_offset, uint64_t seed,
                                                            long long counter, float* __restrict__ actions,
                                                            float* __restrict__ logp) {
    const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    for (int d = 0; d < D; d += 2) {
        const ppox::u32x4 w = ppox::philox4x32_10(
            ppox::u32x4{0x5A5A0000u | (uint32_t)d, (uint32_t)(env_offset + n), (uint32_t)counter,
                        (uint32_t)(counter >> 32)},
            (uint32_t)seed, (uint32_t)(seed >> 32));
        const float u1 = fmaxf(ppox::u01(w.x), 1e-12f), u2 = ppox::u01(w.y);
        const float r = sqrtf(-2.f * logf(u1));
        const float z[2] = {r * cosf(6.283185307179586f * u2), r * sinf(6.283185307179586f * u2)};
        for (int k = 0; k < 2 && d + k < D; ++k) {
            const int j = d + k;
            const float loc = tanhf(mu[n * D + j]);
            const float sc = expf(log_std[j]);
            const float a = loc + sc * z[k];
            const float diff = a - loc;
            actions[n * D + j] = a;
            logp[n * D + j] = -(diff * diff) / (2.f * (sc * sc)) - logf(sc) - (float)LOG_SQRT_2PI;
        }
    }
}

#define PPOX_DISPATCH_A(A, MAXA_NAME, ...)      \
    if ((A) <= 4) {                             \
        constexpr int MAXA_NAME = 4;            \
        __VA_ARGS__;                            \
    } else if ((A) <= 8) {                      \
        constexpr int MAXA_NAME = 8;            \
        __VA_ARGS__;                            \
    } else if ((A) <= 18) {                     \
        constexpr int MAXA_NAME = 18;           \
        __VA_ARGS__;                            \
    } else if ((A) <= 32) {                     \
        constexpr int MAXA_NAME = 32;           \
        __VA_ARGS__;                            \
    } else {                                    \
        constexpr int MAXA_NAME = 64;           \
        __VA_ARGS__;                            \
    }

int check_mb(const Minibatch& m, bool dual, const char* name) {
    PPOX_REQUIRE(m.A >= 1 && m.A <= 64, "%s: n_actions=%d outside [1,64]", name, m.A);
    PPOX_REQUIRE(m.B >= 0 && m.T > 0 && m.N > 0, "%s: bad sizes B=%lld T=%lld N=%lld", name, m.B, m.T, m.N);
    // a rank that owns no rows of a minibatch (B == 0) passes empty (null) row tensors; it still
    // writes its zero partials for the all-reduce
    const bool rows = m.B > 0;
    PPOX_REQUIRE((!rows || (m.logits && m.values && m.idx)) && m.actions && m.old_logp && m.old_values && m.adv &&
                     m.ret && m.adv_stats,
                 "%s: null pointer", name);
    if (dual)
        PPOX_REQUIRE((!rows || m.int_values) && m.old_int_values && m.int_adv && m.int_ret,
                     "%s: null intrinsic pointer", name);
    return PPOX_OK;
}

}  // namespace

extern "C" int ppox_minibatch_adv_stats(const float* advantages, const float* int_advantages, const int64_t* perm,
                                        int64_t total, int64_t batch_size, int64_t T, int64_t N, double* stats_out,
                                        void* stream) {
    PPOX_REQUIRE(advantages && perm && stats_out, "ppox_minibatch_adv_stats: null pointer");
    PPOX_REQUIRE(total > 0 && batch_size > 0 && T > 0 && N > 0 && total <= T * N,
                 "ppox_minibatch_adv_stats: bad sizes");
    const long long nmb = (total + batch_size - 1) / batch_size;
    adv_stats_kernel<<<(unsigned)nmb, 256, 0, ppox::as_stream(stream)>>>(
        advantages, int_advantages, reinterpret_cast<const long long*>(perm), total, batch_size, T, N, stats_out);
    PPOX_LAUNCHED("ppox_minibatch_adv_stats");
}

extern "C" int ppox_ppo_loss_partials(const float* logits, const float* values, const float* int_values,
                                      int64_t B, int32_t A, const int64_t* idx, int64_t T, int64_t N,
                                      const int32_t* actions, const float* old_logp, const float* old_values,
                                      const float* advantages, const float* returns, const float* old_int_values,
                                      const float* int_advantages, const float* int_returns,
                                      const double* adv_stats, float clip, double* partials, void* stream) {
    const bool dual = int_values != nullptr || (B == 0 && old_int_values != nullptr);
    Minibatch m = make_mb(logits, values, int_values, B, A, idx, T, N, actions, old_logp, old_values, advantages,
                          returns, old_int_values, int_advantages, int_returns, adv_stats, clip);
    int rc = check_mb(m, dual, "ppox_ppo_loss_partials");
    if (rc) return rc;
    PPOX_REQUIRE(partials, "ppox_ppo_loss_partials: null partials");
    hipStream_t s = ppox::as_stream(stream);
    PPOX_DISPATCH_A(A, MA, {
        if (dual)
            loss_partials_kernel<MA, true><<<P, 256, 0, s>>>(m, partials);
        else
            loss_partials_kernel<MA, false><<<P, 256, 0, s>>>(m, partials);
    });
    PPOX_LAUNCHED("ppox_ppo_loss_partials");
}

extern "C" int ppox_ppo_loss_backward(const float* logits, const float* values, const float* int_values,
                                      int64_t B, int32_t A, const int64_t* idx, int64_t T, int64_t N,
                                      const int32_t* actions, const float* old_logp, const float* old_values,
                                      const float* advantages, const float* returns, const float* old_int_values,
                                      const float* int_advantages, const float* int_returns,
                                      const double* adv_stats, float clip, const double* partials,
                                      int64_t B_global, float ent_coef, float vf_coef, float int_vf_coef,
                                      float scale, float* dlogits, float* dvalues, float* dint_values,
                                      double* loss_accum, void* stream) {
    const bool dual = int_values != nullptr || (B == 0 && old_int_values != nullptr);
    Minibatch m = make_mb(logits, values, int_values, B, A, idx, T, N, actions, old_logp, old_values, advantages,
                          returns, old_int_values, int_advantages, int_returns, adv_stats, clip);
    int rc = check_mb(m, dual, "ppox_ppo_loss_backward");
    if (rc) return rc;
    PPOX_REQUIRE(partials && (B == 0 || (dlogits && dvalues && (!dual || dint_values))),
                 "ppox_ppo_loss_backward: null output");
    PPOX_REQUIRE(B_global >= 1, "ppox_ppo_loss_backward: B_global must be >= 1");
    hipStream_t s = ppox::as_stream(stream);
    PPOX_DISPATCH_A(A, MA, {
        if (dual)
            loss_backward_kernel<MA, true><<<P, 256, 0, s>>>(m, partials, (double)B_global, ent_coef, vf_coef,
                                                             int_vf_coef, scale, dlogits, dvalues, dint_values,
                                                             loss_accum);
        else
            loss_backward_kernel<MA, false><<<P, 256, 0, s>>>(m, partials, (double)B_global, ent_coef, vf_coef,
                                                              int_vf_coef, scale, dlogits, dvalues, dint_values,
                                                              loss_accum);
    });
    PPOX_LAUNCHED("ppox_ppo_loss_backward");
}

extern "C" int ppox_ppo_box_loss_partials(const float* mu, const float* log_std, const float* values,
                                          const float* int_values, int64_t B, int32_t D, const int64_t* idx, int64_t T,
                                          int64_t N, const float* actions, const float* old_logp,
                                          const float* old_values, const float* advantages, const float* returns,
                                          const float* old_int_values, const float* int_advantages,
                                          const float* int_returns, const double* adv_stats, double clip,
                                          double* partials, void* stream) {
    const bool dual = int_values != nullptr || (B == 0 && old_int_values != nullptr);
    BoxMinibatch bm{make_mb(mu, values, int_values, B, 1, idx, T, N, nullptr, old_logp, old_values, advantages,
                            returns, old_int_values, int_advantages, int_returns, adv_stats, (float)clip),
                    log_std, actions, D, clip};
    PPOX_REQUIRE(D >= 1 && D <= MAXD, "ppox_ppo_box_loss_partials: action dim %d outside [1,%d]", D, MAXD);
    PPOX_REQUIRE((B == 0 || (mu && values && idx)) && log_std && actions && old_logp && old_values && advantages &&
                     returns && adv_stats && partials && (!dual || (old_int_values && int_advantages && int_returns)),
                 "ppox_ppo_box_loss_partials: null pointer");
    PPOX_REQUIRE(B >= 0 && T > 0 && N > 0, "ppox_ppo_box_loss_partials: bad sizes");
    hipStream_t s = ppox::as_stream(stream);
    if (dual)
        box_partials_kernel<true><<<P, 256, 0, s>>>(bm, partials);
    else
        box_partials_kernel<false><<<P, 256, 0, s>>>(bm, partials);
    PPOX_LAUNCHED("ppox_ppo_box_loss_partials");
}

extern "C" int ppox_ppo_box_loss_backward(const float* mu, const float* log_std, const float* values,
                                          const float* int_values, int64_t B, int32_t D, const int64_t* idx, int64_t T,
                                          int64_t N, const float* actions, const float* old_logp,
                                          const float* old_values, const float* advantages, const float* returns,
                                          const float* old_int_values, const float* int_advantages,
                                          const float* int_returns, const double* adv_stats, double clip,
                                          const double* partials, int64_t B_global, float ent_coef, float vf_coef,
                                          float int_vf_coef, float scale, float* dmu, double* dlog_std_partials,
                                          float* dlog_std, float* dvalues, float* dint_values, double* loss_accum,
                                          void* stream) {
    const bool dual = int_values != nullptr || (B == 0 && old_int_values != nullptr);
    BoxMinibatch bm{make_mb(mu, values, int_values, B, 1, idx, T, N, nullptr, old_logp, old_values, advantages,
                            returns, old_int_values, int_advantages, int_returns, adv_stats, (float)clip),
                    log_std, actions, D, clip};
    PPOX_REQUIRE(D >= 1 && D <= MAXD, "ppox_ppo_box_loss_backward: action dim %d outside [1,%d]", D, MAXD);
    PPOX_REQUIRE((B == 0 || (mu && values && idx && dmu && dvalues && (!dual || dint_values))) && log_std &&
                     actions && old_logp && old_values && advantages && returns && adv_stats && partials &&
                     dlog_std_partials && dlog_std && (!dual || (old_int_values && int_advantages && int_returns)),
                 "ppox_ppo_box_loss_backward: null pointer");
    PPOX_REQUIRE(B >= 0 && T > 0 && N > 0 && B_global >= 1, "ppox_ppo_box_loss_backward: bad sizes");
    hipStream_t s = ppox::as_stream(stream);
    if (dual)
        box_backward_kernel<true><<<P, 256, 0, s>>>(bm, partials, (double)B_global, ent_coef, vf_coef, int_vf_coef,
                                                    scale, dmu, dlog_std_partials, dvalues, dint_values, loss_accum);
    else
        box_backward_kernel<false><<<P, 256, 0, s>>>(bm, partials, (double)B_global, ent_coef, vf_coef, int_vf_coef,
                                                     scale, dmu, dlog_std_partials, dvalues, dint_values, loss_accum);
    PPOX_LAUNCHED_NORET("ppox_ppo_box_loss_backward");
    box_logstd_reduce<<<1, 64, 0, s>>>(dlog_std_partials, D, dlog_std);
    PPOX_LAUNCHED("ppox_ppo_box_loss_backward");
}

extern "C" int ppox_normal_sample(const float* mu, const float* log_std, int64_t N, int32_t D, int64_t env_offset,
                                  uint64_t seed, int64_t counter, float* actions, float* log_probs, void* stream) {
    if (N == 0) return PPOX_OK;  // empty shard / minibatch: no pointers to check
    PPOX_REQUIRE(mu && log_std && actions && log_probs, "ppox_normal_sample: null pointer");
    PPOX_REQUIRE(D >= 1 && D <= MAXD && N >= 0, "ppox_normal_sample: bad sizes");
    normal_sample_kernel<<<ppox::ceil_div(N, 256), 256, 0, ppox::as_stream(stream)>>>(mu, log_std, N, D, env_offset,
                                                                                     seed, counter, actions, log_probs);
    PPOX_LAUNCHED("ppox_normal_sample");
}

static int categorical_sample_impl(const float* logits, int64_t N, int32_t A, int64_t env_offset, uint64_t seed,
                                   int64_t counter, const int64_t* cbase, int32_t* actions, float* log_probs,
                                   void* stream) {
    if (N == 0) return PPOX_OK;  // empty shard / minibatch: no pointers to check
    PPOX_REQUIRE(logits && actions && log_probs, "ppox_categorical_sample: null pointer");
    PPOX_REQUIRE(A >= 1 && A <= 64 && N >= 0, "ppox_categorical_sample: bad sizes");
    hipStream_t s = ppox::as_stream(stream);
    const long long* cb = reinterpret_cast<const long long*>(cbase);
    PPOX_DISPATCH_A(A, MA, {
        categorical_sample_kernel<MA><<<ppox::ceil_div(N, 256), 256, 0, s>>>(logits, N, A, env_offset, seed, counter,
                                                                             cb, actions, log_probs);
    });
    PPOX_LAUNCHED("ppox_categorical_sample");
}

extern "C" int ppox_categorical_sample(const float* logits, int64_t N, int32_t A, int64_t env_offset, uint64_t seed,
                                       int64_t counter, int32_t* actions, float* log_probs, void* stream) {
    return categorical_sample_impl(logits, N, A, env_offset, seed, counter, nullptr, actions, log_probs, stream);
}

extern "C" int ppox_categorical_sample_dc(const float* logits, int64_t N, int32_t A, int64_t env_offset,
                                          uint64_t seed, const int64_t* counter_base, int64_t counter_off,
                                          int32_t* actions, float* log_probs, void* stream) {
    PPOX_REQUIRE(counter_base || N == 0, "ppox_categorical_sample_dc: null counter");
    return categorical_sample_impl(logits, N, A, env_offset, seed, counter_off, counter_base, actions, log_probs,
                                   stream);
}
