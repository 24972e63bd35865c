// K11 — the Intrinsic Curiosity Module of PPO_ICM on image observations (reference
// models.py:270-320 IntrinsicCuriosityModule, ppo.py:629-630 int_reward in collect,
// ppo.py:684-699 the ICM loss / backward in train), for uint8 frame stacks, Discrete
// actions and the feature size 32 (int_hidden_size).
//
// The state encoder's first layer Linear(4*84*84 -> 32) is 99.6 % of the module's
// bytes and FLOPs.  Its input is the uint8 frame row, exact in ONE bf16 plane, so both
// of its GEMMs run on the bf16 matrix cores with the f32 operand split exactly into
// three bf16 planes (conv_split.hip): x*w0 + x*w1 + x*w2, every product exact in f32,
// a0 terms in one accumulator, the small terms in a second (fp32-class, see
// conv_common.h).  The frames are read where the rollout holds them (optional env-major
// row index, like the conv1 kernels): no gather, no u8 -> f32 copy.
//   encoder forward   y = x W1^T : split-K MFMA partials + a finishing kernel that sums
//                     them in a fixed order and runs the tiny rest of the encoder
//                     (+ b1, LeakyReLU, Linear(32, 32)) per row;
//   encoder wgrad     dW1 = g1^T x : MFMA over the rows, g1 pre-split into planes by the
//                     row backward kernel, 4-wave LDS reduction in a fixed order.
// Everything else is 32-wide per row or per pair and runs in two LDS kernels:
//   pair kernel       inverse model + forward model + both losses (cross entropy, MSE)
//                     and their backward for the pairs (row j, row j + 1) of the
//                     minibatch (ppo.py:684: observations[:-1], observations[1:]);
//   row kernel        dL/dphi -> through Linear(32, 32) and the LeakyReLU -> g1.
// Weight gradients are per-block partial sums in a slab, reduced in a fixed block order
// by one kernel that writes the ICM's gradient segment directly (deterministic: the same
// inputs give the same bits).
//
// Parameter segment: the ICM's flat parameter buffer (models.FlatParams) holds, after
// state_encoder[0].weight, every other parameter contiguously in module order; Seg gives
// their offsets (floats) from state_encoder[0].bias.
#include <algorithm>

#include "conv_common.h"

namespace {

constexpr int H = 32;           // ICM feature / hidden size
constexpr float SLOPE = 0.01f;  // nn.LeakyReLU() negative slope
constexpr int ROW_COLS = 1088;  // b1 (32) + W2 (32 x 32) + b2 (32): the row kernel's partial columns
#ifndef ICM_PB
#define ICM_PB 8
#endif
constexpr int PB = ICM_PB;      // pairs per pair-kernel block (8: 256 blocks at B = 2048)
constexpr int RB = 32;          // rows per row-kernel block

__device__ inline float leaky(float v) { return v > 0.f ? v : v * SLOPE; }

// sum_{b < nb} p[b * stride], added in order b = 0, 1, ... with the loads issued 8 at a time
__device__ inline float ordered_sum(const float* __restrict__ p, long long stride, int nb) {
    float s = 0.f;
    int b = 0;
    for (; b + 8 <= nb; b += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = p[(long long)(b + u) * stride];
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; b < nb; ++b) s += p[(long long)b * stride];
    return s;
}

// Software pipeline over n steps with S register stages: step i's loads go to slot i % S
// and are issued S steps ahead of its compute.  The steady-state loop has no conditionals,
// so the compiler's wait counts let S - 1 steps' loads stay in flight (a conditional load
// in the loop makes it drain every load at the loop head).  load(i, slot), compute(slot).
template <int S, typename L, typename C>
__device__ inline void pipeline(int n, L&& load, C&& compute) {
    if (n < S) {
#pragma unroll
        for (int u = 0; u < S; ++u)
            if (u < n) load(u, u);
#pragma unroll
        for (int u = 0; u < S; ++u)
            if (u < n) compute(u);
        return;
    }
#pragma unroll
    for (int u = 0; u < S; ++u) {
        load(u, u);  // slot order as in the loop (the loop-head wait counts assume it)
        __builtin_amdgcn_sched_barrier(0);
    }
    int i = 0;
#pragma unroll 1
    for (; i + 2 * S <= n; i += S) {
#pragma unroll
        for (int u = 0; u < S; ++u) {
            compute(u);
            // keep the refill right behind its slot's compute (the scheduler would sink every
            // load to the loop bottom, leaving one step in flight)
            __builtin_amdgcn_sched_barrier(0);
            load(i + S + u, u);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    // S .. 2S - 1 steps left, S of them loaded
#pragma unroll
    for (int u = 0; u < S; ++u) {
        compute(u);
        if (i + S + u < n) load(i + S + u, u);
    }
    i += S;
#pragma unroll
    for (int u = 0; u < S; ++u)
        if (i + u < n) compute(u);
}

struct Seg {
    int A;
    __host__ __device__ explicit Seg(int a) : A(a) {}
    __host__ __device__ int b1() const { return 0; }
    __host__ __device__ int w2() const { return 32; }                  // [32][32]
    __host__ __device__ int b2() const { return 32 + 1024; }
    __host__ __device__ int wf1() const { return ROW_COLS; }           // [32][32 + A]
    __host__ __device__ int bf1() const { return wf1() + 32 * (32 + A); }
    __host__ __device__ int wf2() const { return bf1() + 32; }         // [32][32]
    __host__ __device__ int bf2() const { return wf2() + 1024; }
    __host__ __device__ int wi1() const { return bf2() + 32; }         // [32][64]
    __host__ __device__ int bi1() const { return wi1() + 2048; }
    __host__ __device__ int wi2() const { return bi1() + 32; }         // [A][32]
    __host__ __device__ int bi2() const { return wi2() + 32 * A; }
    __host__ __device__ int wae() const { return bi2() + A; }          // [A][A] (nn.Embedding)
    __host__ __device__ int n() const { return wae() + A * A; }
    __host__ __device__ int stride() const { return n() + 2; }         // + cross-entropy sum, squared-error sum
};

// ---------------------------------------------------------------------------
// W1 [32][K] -> split planes, the B fragments of the encoder forward:
// q[((s * 3 + p) * 64 + lane) * 8 + e] = plane p of W1[lane & 31][k],
// k = 32 (s >> 1) + 16 (lane >> 5) + 8 (s & 1) + e  (s: MFMA k-step of 16)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) icm_pack_w1_kernel(const float* __restrict__ w, int K, u32x4* __restrict__ q) {
    const long long t = blockIdx.x * 256LL + threadIdx.x;
    const long long S = K / 16;
    if (t >= S * 64) return;
    const int lane = (int)(t & 63);
    const long long s = t >> 6;
    const int n = lane & 31, h = lane >> 5;
    const long long k0 = 32 * (s >> 1) + 16 * h + 8 * (s & 1);
    const float4* src = reinterpret_cast<const float4*>(w + (long long)n * K + k0);
    u32x4 p0, p1, p2;
    split8(src[0], src[1], p0, p1, p2);
    q[(s * 3 + 0) * 64 + lane] = p0;
    q[(s * 3 + 1) * 64 + lane] = p1;
    q[(s * 3 + 2) * 64 + lane] = p2;
}

// ---------------------------------------------------------------------------
// Encoder forward partials: workgroup (K chunk kc, row group rg), 8 waves; WR waves
// split the rows (64 each: two 32-row MFMA tiles), KG = 8 / WR waves split the chunk's K
// (interleaved double steps, summed through LDS in wave order).  One double step = 32 k:
// a lane loads 16 frame bytes per tile (row lane & 31, bytes 16 (lane >> 5) ..) and the
// six W1 fragments (2 k-steps x 3 planes) — 12 MFMAs.  slab[kc][row][32] = this chunk's
// x W1^T.  ENC_STAGES double steps are in flight per wave.
// ---------------------------------------------------------------------------
constexpr int ENC_STAGES = 3;

struct EncArgs {
    const uint8_t* x;
    const long long* idx;  // optional env-major rollout rows (sample r = frame row of idx[r])
    long long T, Nenv;
    long long M;
    int K;
    const u32x4* q;
    float* slab;
    int nkc, nrg;
};

template <int WR, int KG>
__global__ void __launch_bounds__(64 * WR * KG) icm_enc_fwd_kernel(EncArgs a) {
    __shared__ float red[KG > 1 ? (KG - 1) * WR * 32 * 64 : 1];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int rgw = wave % WR, kg = wave / WR;
    const long long j = xcd_remap(blockIdx.x, gridDim.x);  // a K chunk's row groups share an XCD (W1 in L2)
    const int kc = (int)(j / a.nrg), rg = (int)(j % a.nrg);
    const int ND = a.K / 32;
    const int d0 = (int)((long long)kc * ND / a.nkc), d1 = (int)((long long)(kc + 1) * ND / a.nkc);
    const long long rbase = (long long)rg * (WR * 64) + rgw * 64;
    const uint8_t* xp[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        long long r = rbase + 32 * i + (lane & 31);
        r = r < a.M ? r : a.M - 1;  // clamped rows are computed, never stored
        long long row = r;
        if (a.idx) {
            const long long s = a.idx[r];
            row = (s % a.T) * a.Nenv + s / a.T;
        }
        xp[i] = a.x + row * a.K + 16 * (lane >> 5);
    }
    const u32x4* qp = a.q + lane;
    f32x16 hi[2], lo[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) hi[i] = lo[i] = zero16();
    using Xs = uint4[2];
    using Ws = u32x4[6];
    auto load = [&](int d, Xs& xs, Ws& ws) {
#pragma unroll
        for (int i = 0; i < 2; ++i) xs[i] = *reinterpret_cast<const uint4*>(xp[i] + 32LL * d);
#pragma unroll
        for (int u = 0; u < 6; ++u) ws[u] = qp[(6LL * d + u) * 64];  // (s = 2d + u / 3, plane u % 3)
    };
    auto step = [&](const Xs& xs, const Ws& ws) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const u32x4 av = u8x8_to_bf16(h ? xs[i].z : xs[i].x, h ? xs[i].w : xs[i].y);
                hi[i] = mfma_bf16(av, ws[3 * h], hi[i]);
                lo[i] = mfma_bf16(av, ws[3 * h + 1], lo[i]);
                lo[i] = mfma_bf16(av, ws[3 * h + 2], lo[i]);
            }
    };
    constexpr int S = ENC_STAGES;
    Xs xs[S];
    Ws ws[S];
    const int ds = d0 + kg;
    const int cnt = ds < d1 ? (d1 - ds + KG - 1) / KG : 0;  // this wave's double steps ds + KG i
    pipeline<S>(cnt, [&](int i, int u) { load(ds + KG * i, xs[u], ws[u]); }, [&](int u) { step(xs[u], ws[u]); });
    float acc[2][16];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][e] = hi[i][e] + lo[i][e];
    if constexpr (KG > 1) {
        if (kg > 0) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int e = 0; e < 16; ++e) red[(((kg - 1) * WR + rgw) * 32 + i * 16 + e) * 64 + lane] = acc[i][e];
        }
        __syncthreads();
        if (kg == 0) {
#pragma unroll 1
            for (int g = 1; g < KG; ++g)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int e = 0; e < 16; ++e) acc[i][e] += red[(((g - 1) * WR + rgw) * 32 + i * 16 + e) * 64 + lane];
        }
    }
    if (kg != 0) return;
    // C/D map: col = lane & 31, row = (e & 3) + 8 (e >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const long long row = rbase + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
            if (row < a.M) a.slab[((long long)kc * a.M + row) * H + (lane & 31)] = acc[i][e];
        }
}

// Encoder forward finish: pre1 = sum_kc slab[kc] + b1 (kc ascending), phi = leaky(pre1)
// W2^T + b2; rowno[r] = the frame row of sample r (read by the weight-gradient kernel).
// 8 rows x 32 features per block.
__global__ void __launch_bounds__(256) icm_enc_finish_kernel(const float* __restrict__ slab, int nkc, long long M,
                                                              const float* __restrict__ seg,
                                                              const long long* __restrict__ idx, long long T,
                                                              long long Nenv, float* __restrict__ pre1,
                                                              float* __restrict__ phi, unsigned* __restrict__ rowno) {
    __shared__ float w2[32][33];
    __shared__ float a1[8][32];
    for (int i = threadIdx.x; i < 1024; i += 256) w2[i >> 5][i & 31] = seg[32 + i];
    const int n = threadIdx.x & 31, rr = threadIdx.x >> 5;
    const long long r = blockIdx.x * 8LL + rr;
    float s = 0.f;
    if (r < M) {
        s = ordered_sum(slab + r * H + n, M * H, nkc);
        s = s + seg[n];
        pre1[r * H + n] = s;
        if (rowno && n == 0) {
            long long row = r;
            if (idx) {
                const long long i = idx[r];
                row = (i % T) * Nenv + i / T;
            }
            rowno[r] = (unsigned)row;
        }
    }
    a1[rr][n] = leaky(s);
    __syncthreads();
    if (r < M) {
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < 32; ++k) acc += a1[rr][k] * w2[n][k];
        phi[r * H + n] = acc + seg[32 + 1024 + n];
    }
}

// ---------------------------------------------------------------------------
// Pair kernel: PB pairs per block.  Pair j = (row j, row j + 1) of the minibatch, action
// a = actions of row j.  Forward (models.py:300-309): u = Wi1 [s | n] + bi1, logits =
// Wi2 leaky(u) + bi2; v = Wf1 [s | Wae[a]] + bf1, nh = Wf2 leaky(v) + bf2.  Loss
// (ppo.py:686-688): (1 - beta) CE(logits, a) / npair + beta sum (nh - n)^2 / (npair 32).
// Backward: dS[j] / dN[j + 1] = dL/dphi through the pair's first / second row (the
// caller sums them per row), weight-gradient partials of this block's pairs.
// ---------------------------------------------------------------------------
struct PairArgs {
    const float* phi;        // [B][32] features of the whole minibatch
    long long B;
    const int32_t* actions;  // action of minibatch row j: actions[rowno ? rowno[j] : j]
    const unsigned* rowno;
    const long long* pairs;  // evaluated pairs (first rows j); null: all j < B - 1
    long long npl;           // number of evaluated pairs
    long long npair;         // pairs of the whole minibatch (B - 1): the losses' mean
    float c_inv, c_beta;     // (1 - beta), beta as f32
    const float* seg;
    int A;
    float* dS;
    float* dN;
    float* slab;
};

__global__ void __launch_bounds__(256) icm_pair_kernel(PairArgs a) {
    const Seg g(a.A);
    const int A = a.A, tid = threadIdx.x;
    __shared__ float Wi1[32][65], Wf1[32][65], Wf2[32][33], Wi2[32][33], Wae[32][33];
    __shared__ float bi1[32], bf1[32], bf2[32], bi2[32];
    __shared__ float S[PB][65];   // [s | n]
    __shared__ float Y[PB][65];   // [s | Wae[a]]
    __shared__ float U[PB][33], V[PB][33];  // pre-activations of the two hidden layers
    __shared__ float L[PB][33];   // logits, then dL/dlogits
    __shared__ float NH[PB][33];  // nh, then dL/dnh
    __shared__ float DU[PB][33], DV[PB][33], DAE[PB][33];
    __shared__ int act[PB];
    __shared__ long long jrow[PB];
    __shared__ float ce[PB], sq[PB];
    const float* sg = a.seg;
    for (int i = tid; i < 32 * 64; i += 256) Wi1[i >> 6][i & 63] = sg[g.wi1() + i];
    for (int i = tid; i < 32 * (32 + A); i += 256) Wf1[i / (32 + A)][i % (32 + A)] = sg[g.wf1() + i];
    for (int i = tid; i < 1024; i += 256) Wf2[i >> 5][i & 31] = sg[g.wf2() + i];
    for (int i = tid; i < 32 * A; i += 256) Wi2[i >> 5][i & 31] = sg[g.wi2() + i];
    for (int i = tid; i < A * A; i += 256) Wae[i / A][i % A] = sg[g.wae() + i];
    if (tid < 32) {
        bi1[tid] = sg[g.bi1() + tid];
        bf1[tid] = sg[g.bf1() + tid];
        bf2[tid] = sg[g.bf2() + tid];
        bi2[tid] = tid < A ? sg[g.bi2() + tid] : 0.f;
    }
    if (tid < PB) {
        const long long jj = blockIdx.x * (long long)PB + tid;
        long long j = -1;
        if (jj < a.npl) j = a.pairs ? a.pairs[jj] : jj;
        jrow[tid] = j;
        act[tid] = j >= 0 ? a.actions[a.rowno ? (long long)a.rowno[j] : j] : 0;
    }
    if (!a.pairs && blockIdx.x == 0 && tid < 32) {  // rows with no pair on one side
        a.dN[tid] = 0.f;
        a.dS[(a.B - 1) * H + tid] = 0.f;
    }
    __syncthreads();
    for (int i = tid; i < PB * 64; i += 256) {
        const int p = i >> 6, c = i & 63;
        const long long j = jrow[p];
        S[p][c] = j >= 0 ? a.phi[(j + (c >> 5)) * H + (c & 31)] : 0.f;
    }
    __syncthreads();
    for (int i = tid; i < PB * 64; i += 256) {
        const int p = i >> 6, c = i & 63;
        if (c < 32) Y[p][c] = S[p][c];
        else if (c - 32 < A) Y[p][c] = Wae[act[p]][c - 32];
    }
    __syncthreads();
    const int o = tid & 31, pg = tid >> 5;
    for (int p = pg; p < PB; p += 8) {
        float u = 0.f, v = 0.f;
#pragma unroll 8
        for (int c = 0; c < 64; ++c) u += Wi1[o][c] * S[p][c];
        for (int c = 0; c < 32 + A; ++c) v += Wf1[o][c] * Y[p][c];
        U[p][o] = u + bi1[o];
        V[p][o] = v + bf1[o];
    }
    __syncthreads();
    for (int p = pg; p < PB; p += 8) {
        if (o < A) {
            float l = 0.f;
#pragma unroll 8
            for (int k = 0; k < 32; ++k) l += Wi2[o][k] * leaky(U[p][k]);
            L[p][o] = l + bi2[o];
        }
        float nh = 0.f;
#pragma unroll 8
        for (int k = 0; k < 32; ++k) nh += Wf2[o][k] * leaky(V[p][k]);
        NH[p][o] = nh + bf2[o];
    }
    __syncthreads();
    const float inv_np = 1.f / (float)a.npair;
    if (tid < PB) {
        const int p = tid;
        const bool valid = jrow[p] >= 0;
        float m = L[p][0];
        for (int q = 1; q < A; ++q) m = fmaxf(m, L[p][q]);
        float se = 0.f;
        for (int q = 0; q < A; ++q) se += expf(L[p][q] - m);
        const float lse = m + logf(se);
        ce[p] = valid ? lse - L[p][act[p]] : 0.f;
        const float cI = a.c_inv * inv_np;
        for (int q = 0; q < A; ++q) L[p][q] = valid ? cI * (expf(L[p][q] - lse) - (q == act[p] ? 1.f : 0.f)) : 0.f;
        float s2 = 0.f;
        for (int c = 0; c < 32; ++c) {
            const float d = NH[p][c] - S[p][32 + c];
            s2 += d * d;
        }
        sq[p] = valid ? s2 : 0.f;
    }
    __syncthreads();
    const float cF = 2.f * a.c_beta * (inv_np / 32.f);
    for (int p = pg; p < PB; p += 8) NH[p][o] = jrow[p] >= 0 ? cF * (NH[p][o] - S[p][32 + o]) : 0.f;
    __syncthreads();
    for (int p = pg; p < PB; p += 8) {
        float du = 0.f, dv = 0.f;
        for (int q = 0; q < A; ++q) du += L[p][q] * Wi2[q][o];
#pragma unroll 8
        for (int c = 0; c < 32; ++c) dv += NH[p][c] * Wf2[c][o];
        DU[p][o] = U[p][o] > 0.f ? du : du * SLOPE;
        DV[p][o] = V[p][o] > 0.f ? dv : dv * SLOPE;
    }
    __syncthreads();
    for (int p = pg; p < PB; p += 8) {
        const long long j = jrow[p];
        if (j < 0) continue;
        float dsi = 0.f, dsf = 0.f, dni = 0.f, dae = 0.f;
#pragma unroll 8
        for (int k = 0; k < 32; ++k) {
            dsi += DU[p][k] * Wi1[k][o];
            dni += DU[p][k] * Wi1[k][32 + o];
            dsf += DV[p][k] * Wf1[k][o];
        }
        if (o < A) {
#pragma unroll 8
            for (int k = 0; k < 32; ++k) dae += DV[p][k] * Wf1[k][32 + o];
            DAE[p][o] = dae;
        }
        a.dS[j * H + o] = dsi + dsf;
        a.dN[(j + 1) * H + o] = dni - NH[p][o];
    }
    __syncthreads();
    float* out = a.slab + (long long)blockIdx.x * g.stride();
    for (int c2 = ROW_COLS + tid; c2 < g.stride(); c2 += 256) {
        float s = 0.f;
        if (c2 < g.bf1()) {
            const int k = c2 - g.wf1(), oo = k / (32 + A), c = k % (32 + A);
            for (int p = 0; p < PB; ++p) s += DV[p][oo] * Y[p][c];
        } else if (c2 < g.wf2()) {
            for (int p = 0; p < PB; ++p) s += DV[p][c2 - g.bf1()];
        } else if (c2 < g.bf2()) {
            const int k = c2 - g.wf2(), c = k >> 5, oo = k & 31;
            for (int p = 0; p < PB; ++p) s += NH[p][c] * leaky(V[p][oo]);
        } else if (c2 < g.wi1()) {
            for (int p = 0; p < PB; ++p) s += NH[p][c2 - g.bf2()];
        } else if (c2 < g.bi1()) {
            const int k = c2 - g.wi1(), oo = k >> 6, c = k & 63;
            for (int p = 0; p < PB; ++p) s += DU[p][oo] * S[p][c];
        } else if (c2 < g.wi2()) {
            for (int p = 0; p < PB; ++p) s += DU[p][c2 - g.bi1()];
        } else if (c2 < g.bi2()) {
            const int k = c2 - g.wi2(), q = k >> 5, oo = k & 31;
            for (int p = 0; p < PB; ++p) s += L[p][q] * leaky(U[p][oo]);
        } else if (c2 < g.wae()) {
            for (int p = 0; p < PB; ++p) s += L[p][c2 - g.bi2()];
        } else if (c2 < g.n()) {
            const int k = c2 - g.wae(), q = k / A, c = k % A;
            for (int p = 0; p < PB; ++p)
                if (jrow[p] >= 0 && act[p] == q) s += DAE[p][c];
        } else if (c2 == g.n()) {
            for (int p = 0; p < PB; ++p) s += ce[p];
        } else {
            for (int p = 0; p < PB; ++p) s += sq[p];
        }
        out[c2] = s;
    }
}

// ---------------------------------------------------------------------------
// Row kernel: RB rows per block.  dphi = dS + dN of the row's minibatch position;
// g1 = (dphi W2) * leaky'(pre1); partials of db1, dW2 = dphi^T leaky(pre1), db2; g1
// written as split planes in the A-fragment order of the weight-gradient MFMA:
// gq[((rs * 3 + p) * 64 + lane) * 8 + e] = plane p of g1[16 rs + 8 (lane >> 5) + e][lane & 31].
// ---------------------------------------------------------------------------
struct RowArgs {
    const float* dS;
    const float* dN;         // may be null (already summed into dS)
    const long long* pos;    // local row -> minibatch position (null: identity)
    long long M;
    const float* pre1;
    const float* seg;
    u32x4* gq;
    float* slab;
    int stride;
};

__global__ void __launch_bounds__(256) icm_row_bwd_kernel(RowArgs a) {
    __shared__ float W2[32][33], D[RB][33], A1[RB][33], P[RB][33], G[RB][33];
    const int tid = threadIdx.x;
    for (int i = tid; i < 1024; i += 256) W2[i >> 5][i & 31] = a.seg[32 + i];
    for (int i = tid; i < RB * 32; i += 256) {
        const int rr = i >> 5, c = i & 31;
        const long long r = blockIdx.x * (long long)RB + rr;
        float d = 0.f, pre = 0.f;
        if (r < a.M) {
            const long long src = a.pos ? a.pos[r] : r;
            d = a.dS[src * H + c];
            if (a.dN) d = d + a.dN[src * H + c];
            pre = a.pre1[r * H + c];
        }
        D[rr][c] = d;
        P[rr][c] = pre;
        A1[rr][c] = leaky(pre);
    }
    __syncthreads();
    for (int i = tid; i < RB * 32; i += 256) {
        const int rr = i >> 5, jj = i & 31;
        float da = 0.f;
#pragma unroll 8
        for (int c = 0; c < 32; ++c) da += D[rr][c] * W2[c][jj];
        G[rr][jj] = P[rr][jj] > 0.f ? da : da * SLOPE;
    }
    __syncthreads();
    if (tid < 64 * (RB / 16)) {
        const int rsl = tid >> 6, lane = tid & 63, n = lane & 31, h = lane >> 5;
        const int r0 = rsl * 16 + 8 * h;
        const float4 v0 = make_float4(G[r0][n], G[r0 + 1][n], G[r0 + 2][n], G[r0 + 3][n]);
        const float4 v1 = make_float4(G[r0 + 4][n], G[r0 + 5][n], G[r0 + 6][n], G[r0 + 7][n]);
        u32x4 p0, p1, p2;
        split8(v0, v1, p0, p1, p2);
        const long long rs = blockIdx.x * (long long)(RB / 16) + rsl;
        a.gq[(rs * 3 + 0) * 64 + lane] = p0;
        a.gq[(rs * 3 + 1) * 64 + lane] = p1;
        a.gq[(rs * 3 + 2) * 64 + lane] = p2;
    }
    float* out = a.slab + (long long)blockIdx.x * a.stride;
    for (int col = tid; col < ROW_COLS; col += 256) {
        float s = 0.f;
        if (col < 32) {
            for (int rr = 0; rr < RB; ++rr) s += G[rr][col];
        } else if (col < 32 + 1024) {
            const int c = (col - 32) >> 5, jj = (col - 32) & 31;
            for (int rr = 0; rr < RB; ++rr) s += D[rr][c] * A1[rr][jj];
        } else {
            for (int rr = 0; rr < RB; ++rr) s += D[rr][col - 1056];
        }
        out[col] = s;
    }
}

// Partials -> the gradient segment + this call's loss share.  64 columns per block, each
// summed by 4 threads over consecutive quarters of the blocks, quarters added in order
// ((q0 + q1) + (q2 + q3)).
__global__ void __launch_bounds__(256) icm_grad_reduce_kernel(const float* __restrict__ slab, int stride, int ncols,
                                                               int nblk_row, int nblk_pair, float* __restrict__ gseg,
                                                               double* __restrict__ loss_acc, float c_inv,
                                                               float c_beta, long long npair) {
    __shared__ float part[4][64];
    const int cl = threadIdx.x & 63, q = threadIdx.x >> 6;
    // the last block: columns ncols, ncols + 1 = the pairs' cross-entropy and squared-error sums
    const bool loss_blk = blockIdx.x == gridDim.x - 1;
    const int col = loss_blk ? ncols + cl : blockIdx.x * 64 + cl;
    const bool ok = loss_blk ? cl < 2 : col < ncols;
    const int nb = col < ROW_COLS ? nblk_row : nblk_pair;
    const int b0 = (int)((long long)q * nb / 4), b1 = (int)((long long)(q + 1) * nb / 4);
    part[q][cl] = ok ? ordered_sum(slab + (long long)b0 * stride + col, stride, b1 - b0) : 0.f;
    __syncthreads();
    if (q != 0 || !ok) return;
    const float s = (part[0][cl] + part[1][cl]) + (part[2][cl] + part[3][cl]);
    if (!loss_blk) {
        gseg[col] = s;
    } else if (cl == 0 && loss_acc) {
        const float sq = (part[0][cl + 1] + part[1][cl + 1]) + (part[2][cl + 1] + part[3][cl + 1]);
        const float inv = s / (float)npair, fwd = sq / (float)(npair * H);
        loss_acc[0] += (double)(c_inv * inv + c_beta * fwd);
    }
}

// ---------------------------------------------------------------------------
// Encoder weight gradient dW1 = g1^T x: workgroup = 128 columns of W1 (4 MFMA tiles of
// 32 columns, column 4 j + t of the block in tile t), all rows, 8 waves.  Wave w takes the
// 16-row steps rs = w, w + 8, ...: per step a lane loads one dword (4 columns) from each of
// 8 rows (row 16 rs + 8 (lane >> 5) + e) — 128 contiguous bytes per row per half-wave —
// and byte t of the 8 dwords is tile t's B fragment; the A fragments are g1's planes.
// WG_STAGES steps are in flight per wave (the kernel is bound by HBM latency x bytes in
// flight: 8 waves x 3 steps x 2 KB per CU).  The waves' sums are added in LDS in wave
// order and stored as float4 rows.
// ---------------------------------------------------------------------------
constexpr int WG_CHUNK = 2048;  // rows whose frame-row numbers are staged in LDS at a time
constexpr int WG_WAVES = 8;
constexpr int WG_STAGES = 3;

struct WgArgs {
    const uint8_t* x;
    const unsigned* rowno;
    long long M;
    int K;
    const u32x4* gq;
    float* dw;
};

__global__ void __launch_bounds__(64 * WG_WAVES) icm_enc_wgrad_kernel(WgArgs a) {
    __shared__ unsigned rows_l[WG_CHUNK];
    __shared__ float4 red[WG_WAVES][32][32];  // [wave][n][column quad]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 31, hb = lane >> 5;
    const long long k0 = blockIdx.x * 128LL;
    // columns past K (last block): a valid address, results never stored
    const uint8_t* xc = a.x + std::min<long long>(k0 + 4 * j, a.K - 4);
    f32x16 hi[4], lo[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) hi[t] = lo[t] = zero16();
    const long long RS = (a.M + 15) / 16;
    using Xs = uint32_t[8];
    using Gs = u32x4[3];
    auto load = [&](long long rs, long long c0, Xs& xv, Gs& gv) {
        const int rl = (int)(rs * 16 - c0) + 8 * hb;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const unsigned row = rows_l[rl + e];
            xv[e] = *reinterpret_cast<const uint32_t*>(xc + (long long)row * a.K);
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) gv[p] = a.gq[(rs * 3 + p) * 64 + lane];
    };
    auto step = [&](const Xs& xv, const Gs& gv) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            u32x4 b;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                b[q] = pack_hi((float)((xv[2 * q] >> (8 * t)) & 0xFFu), (float)((xv[2 * q + 1] >> (8 * t)) & 0xFFu));
            hi[t] = mfma_bf16(gv[0], b, hi[t]);
            lo[t] = mfma_bf16(gv[1], b, lo[t]);
            lo[t] = mfma_bf16(gv[2], b, lo[t]);
        }
    };
    constexpr int W = WG_WAVES, S = WG_STAGES;
    for (long long c0 = 0; c0 < a.M; c0 += WG_CHUNK) {
        __syncthreads();
        for (int i = tid; i < WG_CHUNK; i += 64 * W) {
            const long long r = c0 + i;
            rows_l[i] = r < a.M ? a.rowno[r] : 0u;  // rows past M: g1 is zero there
        }
        __syncthreads();
        const long long rs_end = std::min(RS, (c0 + WG_CHUNK) / 16);
        const long long rs0 = c0 / 16 + wave;
        const int cnt = rs0 < rs_end ? (int)((rs_end - rs0 + W - 1) / W) : 0;  // this wave's steps rs0 + W i
        Xs xv[S];
        Gs gv[S];
        pipeline<S>(cnt, [&](int i, int u) { load(rs0 + (long long)W * i, c0, xv[u], gv[u]); },
                    [&](int u) { step(xv[u], gv[u]); });
    }
    // C/D map: col j = lane & 31 (W1 column k0 + 4 j + t of tile t), row n = (e & 3) + 8 (e >> 2) + 4 hb
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int n = (e & 3) + 8 * (e >> 2) + 4 * hb;
        red[wave][n][j] = make_float4(hi[0][e] + lo[0][e], hi[1][e] + lo[1][e], hi[2][e] + lo[2][e],
                                      hi[3][e] + lo[3][e]);
    }
    __syncthreads();
    for (int f = tid; f < 32 * 32; f += 64 * W) {
        const int n = f >> 5, jq = f & 31;
        if (k0 + 4 * jq >= a.K) continue;
        float4 s = red[0][n][jq];
#pragma unroll
        for (int w = 1; w < W; ++w) {
            const float4 v = red[w][n][jq];
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
        *reinterpret_cast<float4*>(a.dw + (long long)n * a.K + k0 + 4 * jq) = s;
    }
}

// ---------------------------------------------------------------------------
// Collect (ppo.py:629-630, models.py:311-320): int_reward = clamp(mean((forward_model(
// [phi_s | Wae[a]]) - phi_n)^2), -5, 5); rewards = (1 - eta) rewards + eta int_reward.
// 8 rows per block.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) icm_int_reward_kernel(const float* __restrict__ phi_s,
                                                              const float* __restrict__ phi_n,
                                                              const int32_t* __restrict__ actions, long long N, int A,
                                                              const float* __restrict__ seg, float c_keep, float c_eta,
                                                              float* __restrict__ rewards, float* __restrict__ ir) {
    const Seg g(A);
    __shared__ float Wf1[32][65], Wf2[32][33], Y[8][65], Vv[8][33], SQ[8][33];
    const int tid = threadIdx.x, c = tid & 31, rr = tid >> 5;
    for (int i = tid; i < 32 * (32 + A); i += 256) Wf1[i / (32 + A)][i % (32 + A)] = seg[g.wf1() + i];
    for (int i = tid; i < 1024; i += 256) Wf2[i >> 5][i & 31] = seg[g.wf2() + i];
    const long long r = blockIdx.x * 8LL + rr;
    const bool ok = r < N;
    const int act = ok ? actions[r] : 0;
    Y[rr][c] = ok ? phi_s[r * H + c] : 0.f;
    if (c < A) Y[rr][32 + c] = seg[g.wae() + act * A + c];
    __syncthreads();
    float v = 0.f;
    for (int k = 0; k < 32 + A; ++k) v += Wf1[c][k] * Y[rr][k];
    Vv[rr][c] = leaky(v + seg[g.bf1() + c]);
    __syncthreads();
    float nh = 0.f;
#pragma unroll 8
    for (int k = 0; k < 32; ++k) nh += Wf2[c][k] * Vv[rr][k];
    nh = nh + seg[g.bf2() + c];
    const float d = nh - (ok ? phi_n[r * H + c] : 0.f);
    SQ[rr][c] = d * d;
    __syncthreads();
    if (c == 0 && ok) {
        float s = 0.f;
        for (int k = 0; k < 32; ++k) s += SQ[rr][k];
        const float m = fminf(fmaxf(s * (1.f / 32.f), -5.f), 5.f);
        ir[r] = m;
        rewards[r] = c_keep * rewards[r] + c_eta * m;
    }
}

// host: encoder-forward launch shape for `rows`
struct EncShape {
    int wr, nrg, nkc;
};
#ifndef ICM_FWD_WGS
#define ICM_FWD_WGS 256
#endif
EncShape enc_shape(long long M, int K) {
    EncShape s;
    s.wr = M >= 1024 ? 4 : 1;
    s.nrg = (int)ppox::ceil_div(M, 64LL * s.wr);
    const int nd = K / 32, kg = 8 / s.wr;
    s.nkc = std::max(1, std::min<int>(ppox::ceil_div(ICM_FWD_WGS, s.nrg), std::max(1, nd / kg)));
    return s;
}

bool icm_shape_ok(long long K) { return K > 0 && K % 32 == 0 && K < (1LL << 30); }

}  // namespace

extern "C" int64_t ppox_icm_param_elems(int32_t n_actions) {
    if (n_actions < 1 || n_actions > 32) return -1;
    return Seg(n_actions).n();
}

extern "C" int64_t ppox_icm_w1_pack_elems(int64_t K) { return icm_shape_ok(K) ? 3LL * H * K : -1; }

extern "C" int ppox_icm_pack_w1(const float* w1, int64_t K, uint16_t* q, void* stream) {
    PPOX_REQUIRE(w1 && q && icm_shape_ok(K), "ppox_icm_pack_w1: bad arguments (K must be a positive multiple of 32)");
    PPOX_REQUIRE(ppox::aligned16(w1) && ppox::aligned16(q), "ppox_icm_pack_w1: 16-byte alignment");
    icm_pack_w1_kernel<<<ppox::ceil_div(K / 16 * 64, 256), 256, 0, ppox::as_stream(stream)>>>(
        w1, (int)K, reinterpret_cast<u32x4*>(q));
    PPOX_LAUNCHED("ppox_icm_pack_w1");
}

extern "C" int64_t ppox_icm_encode_workspace_bytes(int64_t rows, int64_t K) {
    if (rows <= 0 || !icm_shape_ok(K)) return 0;
    return (int64_t)enc_shape(rows, (int)K).nkc * rows * H * 4;
}

extern "C" int ppox_icm_encode(const void* x, int64_t rows, const int64_t* idx, int64_t T, int64_t N_env, int64_t K,
                               const uint16_t* q, const float* seg, void* workspace, float* pre1, float* phi,
                               uint32_t* rowno, void* stream) {
    if (rows == 0) return PPOX_OK;
    PPOX_REQUIRE(x && q && seg && workspace && pre1 && phi && rows > 0 && icm_shape_ok(K),
                 "ppox_icm_encode: bad arguments (K must be a positive multiple of 32)");
    PPOX_REQUIRE(ppox::aligned16(x) && ppox::aligned16(q), "ppox_icm_encode: 16-byte alignment");
    if (idx) PPOX_REQUIRE(T > 0 && N_env > 0 && T * N_env < (1LL << 32), "ppox_icm_encode: idx needs T, N_env");
    else PPOX_REQUIRE(rows < (1LL << 32), "ppox_icm_encode: too many rows");
    const EncShape s = enc_shape(rows, (int)K);
    hipStream_t st = ppox::as_stream(stream);
    float* slab = reinterpret_cast<float*>(workspace);
    EncArgs a{reinterpret_cast<const uint8_t*>(x), reinterpret_cast<const long long*>(idx), T, N_env, rows, (int)K,
              reinterpret_cast<const u32x4*>(q), slab, s.nkc, s.nrg};
    const unsigned grid = (unsigned)(s.nkc * s.nrg);
    if (s.wr == 4) icm_enc_fwd_kernel<4, 2><<<grid, 512, 0, st>>>(a);
    else icm_enc_fwd_kernel<1, 8><<<grid, 512, 0, st>>>(a);
    PPOX_LAUNCHED_NORET("ppox_icm_encode");
    icm_enc_finish_kernel<<<ppox::ceil_div(rows, 8), 256, 0, st>>>(slab, s.nkc, rows, seg,
                                                                   reinterpret_cast<const long long*>(idx), T, N_env,
                                                                   pre1, phi, rowno);
    PPOX_LAUNCHED("ppox_icm_encode");
}

extern "C" int64_t ppox_icm_partials_bytes(int64_t rows, int32_t n_actions) {
    if (rows < 0 || n_actions < 1 || n_actions > 32) return 0;
    const long long nb = std::max<long long>(1, ppox::ceil_div(std::max<int64_t>(rows, 1), std::min(PB, RB)));
    return nb * Seg(n_actions).stride() * 4;
}

extern "C" int64_t ppox_icm_g1_pack_elems(int64_t rows) {
    return rows <= 0 ? 0 : (int64_t)ppox::ceil_div(rows, RB) * (RB / 16) * 3 * 64 * 8;
}

extern "C" int ppox_icm_pair_backward(const float* phi, int64_t B, const int32_t* actions, const uint32_t* rowno,
                                      const int64_t* pairs, int64_t n_pairs, int64_t n_pairs_global,
                                      int32_t n_actions, float beta, const float* seg, float* dS, float* dN,
                                      float* partials, void* stream) {
    PPOX_REQUIRE(phi && actions && seg && dS && dN && partials && B >= 1 && n_pairs >= 0 && n_pairs < B &&
                     n_pairs_global < B && n_actions >= 1 && n_actions <= 32,
                 "ppox_icm_pair_backward: bad arguments");
    PPOX_REQUIRE(pairs || n_pairs == B - 1, "ppox_icm_pair_backward: without a pair list every j < B - 1 is a pair");
    PairArgs a{phi, B, actions, rowno, reinterpret_cast<const long long*>(pairs), n_pairs, n_pairs_global,
               1.f - beta, beta, seg, n_actions, dS, dN, partials};
    const unsigned nb = std::max(1u, ppox::ceil_div(n_pairs, PB));
    icm_pair_kernel<<<nb, 256, 0, ppox::as_stream(stream)>>>(a);
    PPOX_LAUNCHED("ppox_icm_pair_backward");
}

extern "C" int ppox_icm_row_backward(const float* dS, const float* dN, const int64_t* pos, int64_t rows,
                                     const float* pre1, const float* seg, int32_t n_actions, uint16_t* g1q,
                                     float* partials, void* stream) {
    if (rows == 0) return PPOX_OK;
    PPOX_REQUIRE(dS && pre1 && seg && g1q && partials && rows > 0 && n_actions >= 1 && n_actions <= 32,
                 "ppox_icm_row_backward: bad arguments");
    PPOX_REQUIRE(ppox::aligned16(g1q), "ppox_icm_row_backward: 16-byte alignment");
    RowArgs a{dS, dN, reinterpret_cast<const long long*>(pos), rows, pre1, seg, reinterpret_cast<u32x4*>(g1q),
              partials, Seg(n_actions).stride()};
    icm_row_bwd_kernel<<<ppox::ceil_div(rows, RB), 256, 0, ppox::as_stream(stream)>>>(a);
    PPOX_LAUNCHED("ppox_icm_row_backward");
}

extern "C" int ppox_icm_grad_reduce(const float* partials, int64_t rows, int64_t n_pairs, int32_t n_actions,
                                    float beta, int64_t n_pairs_global, float* grad_seg, double* loss_accum,
                                    void* stream) {
    PPOX_REQUIRE(partials && grad_seg && rows >= 1 && n_pairs >= 0 && n_actions >= 1 && n_actions <= 32,
                 "ppox_icm_grad_reduce: bad arguments");
    const Seg g(n_actions);
    const int nbr = (int)ppox::ceil_div(rows, RB), nbp = (int)std::max(1u, ppox::ceil_div(n_pairs, PB));
    icm_grad_reduce_kernel<<<ppox::ceil_div(g.n(), 64) + 1, 256, 0, ppox::as_stream(stream)>>>(
        partials, g.stride(), g.n(), nbr, nbp, grad_seg, loss_accum, 1.f - beta, beta, n_pairs_global);
    PPOX_LAUNCHED("ppox_icm_grad_reduce");
}

extern "C" int ppox_icm_enc_wgrad(const void* x, const uint32_t* rowno, int64_t rows, int64_t K, const uint16_t* g1q,
                                  float* dw1, void* stream) {
    PPOX_REQUIRE(x && rowno && g1q && dw1 && rows >= 1 && icm_shape_ok(K), "ppox_icm_enc_wgrad: bad arguments");
    PPOX_REQUIRE(ppox::aligned16(g1q) && ppox::aligned16(dw1) && !(reinterpret_cast<uintptr_t>(x) & 3),
                 "ppox_icm_enc_wgrad: alignment");
    // the g1 planes cover whole RB-row blocks: the last 16-row step is inside them
    WgArgs a{reinterpret_cast<const uint8_t*>(x), rowno, rows, (int)K, reinterpret_cast<const u32x4*>(g1q), dw1};
    icm_enc_wgrad_kernel<<<ppox::ceil_div(K, 128), 64 * WG_WAVES, 0, ppox::as_stream(stream)>>>(a);
    PPOX_LAUNCHED("ppox_icm_enc_wgrad");
}

extern "C" int ppox_icm_int_reward(const float* phi_s, const float* phi_n, const int32_t* actions, int64_t N,
                                   int32_t n_actions, const float* seg, float eta, float* rewards,
                                   float* int_rewards, void* stream) {
    if (N == 0) return PPOX_OK;
    PPOX_REQUIRE(phi_s && phi_n && actions && seg && rewards && int_rewards && N > 0 && n_actions >= 1 &&
                     n_actions <= 32,
                 "ppox_icm_int_reward: bad arguments");
    icm_int_reward_kernel<<<ppox::ceil_div(N, 8), 256, 0, ppox::as_stream(stream)>>>(
        phi_s, phi_n, actions, N, n_actions, seg, 1.f - eta, eta, rewards, int_rewards);
    PPOX_LAUNCHED("ppox_icm_int_reward");
}
