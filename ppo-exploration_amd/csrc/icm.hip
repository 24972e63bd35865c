// K11 — the Intrinsic Curiosity Module of PPO_ICM on image observations (reference
// models.py:270-320 IntrinsicCuriosityModule, ppo.py:629-630 int_reward in collect,
// ppo.py:684-699 the ICM loss / backward in train), for uint8 frame stacks, Discrete
// actions and the feature size 32 (int_hidden_size).
//
// The state encoder's first layer Linear(4*84*84 -> 32) is 99.6 % of the module's
// bytes and FLOPs.  Its input is the uint8 frame row, exact in ONE f16 plane, so both of
// its GEMMs run split-f16 on v_mfma_f32_32x32x16_f16 (conv_common.h): the f32 operand
// times a power of two 2^E is split exactly into two f16 planes, x*h + x*l, every product
// exact in f32, the h terms in one accumulator and the l terms in a second (fp32-class).
// E is per output feature n (W1 row n / g1 column n: the MFMA tile's row or column, so
// the unscale is one multiply per accumulator).  The frames are read where the rollout
// holds them (optional env-major row index, like the conv1 kernels): no gather, no
// u8 -> f32 copy.
//   encoder forward   y = x W1^T : split-K MFMA partials — frame rows and W1 planes
//                     copied global -> LDS by global_load_lds_dwordx4 into a three-slot
//                     ring (64-B row pieces, XOR-swizzled) — + a finishing kernel that
//                     sums them in a fixed order and runs the tiny rest of the encoder
//                     (+ b1, LeakyReLU, Linear(32, 32)) per row;
//   encoder wgrad     dW1 = g1^T x : MFMA over the rows, g1 written in fragment order by
//                     the row backward kernel with its per-column amax partials, split in
//                     registers; 8-wave LDS reduction in a fixed order.
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
constexpr int ICM_PB = 8;
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
// W1 [32][K] -> its two f16 planes, row n times 2^E[n] (E[n] = split_scale_exp of the row's
// own amax), in the B-fragment order of the encoder forward's 64-k chunks:
// q[(((c * 4 + s) * 2 + p) * 64 + lane) * 8 + e] = plane p of W1[lane & 31][k] 2^E,
// k = 64 c + 32 (s >> 1) + 16 (lane >> 5) + 8 (s & 1) + e; the 32 int32 exponents follow
// the planes.  One workgroup per row n: its amax, then its 8-k runs.
// ---------------------------------------------------------------------------
constexpr int ENC_CK = 64;  // k (frame bytes per row) of one forward chunk

// ICM_W1_PARTS workgroups per row: each derives the row's amax from the whole row (the redundant reads hit
// L2) and packs its own 1/ICM_W1_PARTS of the row's 8-k runs, so the launch has 32 x ICM_W1_PARTS workgroups
// instead of one latency-bound workgroup per row (a second launch for a shared amax would cost more)
constexpr int ICM_W1_PARTS = 8;
__global__ void __launch_bounds__(1024) icm_pack_w1_kernel(const float* __restrict__ w, int K, u32x4* __restrict__ q) {
    __shared__ uint32_t red[16];
    const int n = blockIdx.x / ICM_W1_PARTS, part = blockIdx.x % ICM_W1_PARTS, tid = threadIdx.x;
    const float* wr = w + (long long)n * K;
    uint32_t m = 0u;
    for (int k = tid * 4; k < K; k += 4096) {
        const float4 v = *reinterpret_cast<const float4*>(wr + k);
        m = max(max(m, max(__float_as_uint(fabsf(v.x)), __float_as_uint(fabsf(v.y)))),
                max(__float_as_uint(fabsf(v.z)), __float_as_uint(fabsf(v.w))));
    }
    m = wave_max_u32(m);
    if ((tid & 63) == 0) red[tid >> 6] = m;
    __syncthreads();
    m = red[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) m = max(m, red[i]);
    const int E = split_scale_exp(m);
    const float sc = exp2i(E);
    const int per = (K / 8 + ICM_W1_PARTS - 1) / ICM_W1_PARTS, g1 = min(K / 8, (part + 1) * per);
    for (int g = part * per + tid; g < g1; g += 1024) {
        const int k0 = g * 8, c = k0 / ENC_CK, r = k0 % ENC_CK;
        const int st = 2 * (r >> 5) + ((r >> 3) & 1), lane = n + 32 * ((r >> 4) & 1);
        u32x4 p0, p1;
        split8h(*reinterpret_cast<const float4*>(wr + k0), *reinterpret_cast<const float4*>(wr + k0 + 4), sc, p0, p1);
        q[((c * 4 + st) * 2 + 0) * 64 + lane] = p0;
        q[((c * 4 + st) * 2 + 1) * 64 + lane] = p1;
    }
    if (tid == 0 && part == 0) reinterpret_cast<int*>(q + (long long)K / 16 * 2 * 64)[n] = E;
}

// ---------------------------------------------------------------------------
// Encoder forward partials: workgroup (K range kc, 256 rows rg), 4 waves x 64 rows (two
// 32-row MFMA tiles sharing each B fragment).  Per 64-k chunk the frame rows (16 KB: 64 B
// per row) and the chunk's W1 planes (8 KB) are copied global -> LDS by
// global_load_lds_dwordx4 into a three-slot ring: each wave copies its own 64 rows (4 x
// 1 KB, 16 rows each) and two of the eight 1 KB W1 pieces.  K loop (as the sg2 GEMM in
// conv.hip): wait for this wave's copies of chunk c (the next chunk's may stay in flight),
// one barrier (every wave's copies landed, every wave done with chunk c - 1), issue chunk
// c + 2 into chunk c - 1's slot, then 12 ds_read_b128 + 16 MFMAs.  A row's four 16-B
// pieces sit XOR-swizzled by (row >> 2) & 3 (the copy is lane-linear in LDS, so the
// swizzle is on each lane's global source), which makes every fragment read
// conflict-free.  MFMA k-step s of the chunk, lane half h: k = 32 (s >> 1) + 16 h +
// 8 (s & 1) + e, so one ds_read_b128 of piece 2 (s >> 1) + h feeds two k-steps.
// slab[kc][row][32] = this K range's x W1^T (unscaled).  Measured (MI355X): 15.5 us at 2048 rows
// (3.7 TB/s of frames), 104 us at 16384 (4.4 TB/s); deeper rings (4, 5 slots), 512 workgroups
// and 128-row x 256-B super-chunks (whole 256-B runs per row, twice the W1 bytes per frame
// byte) all measured slower.
// ---------------------------------------------------------------------------
constexpr int ENC_WAVES = 4, ENC_ROWS = 64 * ENC_WAVES, ENC_SLOTS = 3;
constexpr int ENC_AB = ENC_ROWS * ENC_CK;      // frame bytes of a chunk
constexpr int ENC_BB = 4 * 2 * 64 * 16;        // W1 plane bytes of a chunk (4 k-steps x 2 planes)
constexpr int ENC_SLOT = ENC_AB + ENC_BB;
constexpr int ENC_NDMA = 4 + ENC_BB / 1024 / ENC_WAVES;  // copies per wave per chunk

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

__device__ inline u32x4 enc_ds_read(uint32_t addr) {
    u32x4 r;
    asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(addr));
    return r;
}
// wait until at most N LDS reads are outstanding; the four registers are tied, so no use of
// them is scheduled above the wait
template <int N>
__device__ inline void enc_lgkm_wait(u32x4& a, u32x4& b, u32x4& c, u32x4& d) {
    asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "n"(N));
}
template <int N>
__device__ inline void enc_vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__global__ void __launch_bounds__(64 * ENC_WAVES, 2) icm_enc_fwd_kernel(EncArgs a) {
    // all LDS in ONE __shared__ object (a second one can make hipcc wait vmcnt(0) in the loop)
    __shared__ __attribute__((aligned(16))) uint8_t lds[ENC_SLOTS * ENC_SLOT];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: copy bases go to M0
    const long long j = xcd_remap(blockIdx.x, gridDim.x);  // a K range's row groups share an XCD (W1 in L2)
    const int kc = (int)(j / a.nrg), rg = (int)(j % a.nrg);
    const int NC = a.K / ENC_CK;
    const int c0 = (int)((long long)kc * NC / a.nkc), nchunk = (int)((long long)(kc + 1) * NC / a.nkc) - c0;
    // copy sources: A copy i of this wave covers rows 64 wave + 16 i + (lane >> 2), LDS piece
    // lane & 3, which holds global piece (lane & 3) ^ ((row >> 2) & 3) = (lane & 3) ^ ((lane >> 4) & 3)
    const uint8_t* asrc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        long long r = (long long)rg * ENC_ROWS + wave * 64 + 16 * i + (lane >> 2);
        r = r < a.M ? r : a.M - 1;  // rows past the end: a valid clamped row, computed, never stored
        long long row = r;
        if (a.idx) {
            const long long s = a.idx[r];
            row = (s % a.T) * a.Nenv + s / a.T;
        }
        asrc[i] = a.x + row * a.K + (long long)c0 * ENC_CK + (((lane & 3) ^ ((lane >> 4) & 3)) << 4);
    }
    const u32x4* bsrc = a.q + (long long)c0 * (ENC_BB / 16) + lane;
    auto issue = [&](int c, auto S) {
        constexpr int slot = decltype(S)::value;
        c = c < nchunk ? c : nchunk - 1;  // past the end: the last chunk again, never read
        uint8_t* base = lds + slot * ENC_SLOT;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(asrc[i] + c * ENC_CK),
                                             (__attribute__((address_space(3))) void*)(base + (wave * 64 + 16 * i) *
                                                                                                  ENC_CK),
                                             16, 0, 0);
#pragma unroll
        for (int i = 0; i < ENC_NDMA - 4; ++i) {
            const int piece = (ENC_NDMA - 4) * wave + i;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(bsrc + (long long)c * (ENC_BB / 16) + piece * 64),
                (__attribute__((address_space(3))) void*)(base + ENC_AB + piece * 1024), 16, 0, 0);
        }
    };
    const int r = lane & 31, h = lane >> 5, sw = (r >> 2) & 3;
    const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)lds);
    const uint32_t a_lane = lds0 + (wave * 64 + r) * ENC_CK, b_lane = lds0 + ENC_AB + lane * 16;
    f32x16 hi[2], lo[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) hi[t] = lo[t] = zero16();
    auto compute = [&](auto S) {
        constexpr int slot = decltype(S)::value;
        const uint32_t ab = a_lane + slot * ENC_SLOT, bb = b_lane + slot * ENC_SLOT;
        u32x4 f[2][4];  // k-step pair qq: A pieces of tiles 0, 1, then B planes 0, 1 of k-step 2 qq ...
        u32x4 g[2][2];  // ... and of k-step 2 qq + 1
#pragma unroll
        for (int qq = 0; qq < 2; ++qq) {
#pragma unroll
            for (int t = 0; t < 2; ++t) f[qq][t] = enc_ds_read(ab + t * 32 * ENC_CK + (((2 * qq + h) ^ sw) << 4));
#pragma unroll
            for (int p = 0; p < 2; ++p) f[qq][2 + p] = enc_ds_read(bb + ((2 * qq) * 2 + p) * 1024);
#pragma unroll
            for (int p = 0; p < 2; ++p) g[qq][p] = enc_ds_read(bb + ((2 * qq + 1) * 2 + p) * 1024);
        }
        auto pair = [&](int qq) {
#pragma unroll
            for (int so = 0; so < 2; ++so) {
                const u32x4 b0 = so ? g[qq][0] : f[qq][2], b1 = so ? g[qq][1] : f[qq][3];
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const u32x4 av = u8x8_to_f16(f[qq][t][2 * so], f[qq][t][2 * so + 1]);
                    hi[t] = mfma_f16(av, b0, hi[t]);
                    lo[t] = mfma_f16(av, b1, lo[t]);
                }
            }
        };
        enc_lgkm_wait<6>(f[0][0], f[0][1], f[0][2], f[0][3]);
        enc_lgkm_wait<6>(g[0][0], g[0][1], f[0][2], f[0][3]);
        pair(0);
        enc_lgkm_wait<0>(f[1][0], f[1][1], f[1][2], f[1][3]);
        enc_lgkm_wait<0>(g[1][0], g[1][1], f[1][2], f[1][3]);
        pair(1);
    };
    // one pipeline step: this wave's copies of chunk c waited for (chunk c + 1's may stay in
    // flight: the clamped re-issues past the end count too, so the count is the same in every
    // step), one barrier, chunk c + 2 issued into the slot chunk c - 1 used, chunk c computed
    auto step = [&](int c, auto S, auto S2) {
        enc_vm_wait<ENC_NDMA * (ENC_SLOTS - 2)>();
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        issue(c + ENC_SLOTS - 1, S2);
        compute(S);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    issue(0, I0{});
    issue(1, I1{});
#pragma unroll 1
    for (int c = 0; c < nchunk; c += 3) {
        step(c, I0{}, I2{});
        if (c + 1 < nchunk) step(c + 1, I1{}, I0{});
        if (c + 2 < nchunk) step(c + 2, I2{}, I1{});
    }
    enc_vm_wait<0>();  // the clamped tail copies, before the LDS is released
    // unscale by the lane's feature exponent; C/D map: col n = lane & 31, row = (e & 3) + 8 (e >> 2) + 4 h
    const int* wexp = reinterpret_cast<const int*>(a.q + (long long)NC * (ENC_BB / 16));
    const float uw = exp2i(-wexp[r]);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const long long row = (long long)rg * ENC_ROWS + wave * 64 + 32 * t + (e & 3) + 8 * (e >> 2) + 4 * h;
            if (row < a.M) a.slab[((long long)kc * a.M + row) * H + r] = (hi[t][e] + lo[t][e]) * uw;
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
    {
        float v[4];  // the four loads in flight together
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = seg[32 + threadIdx.x + 256 * k];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = threadIdx.x + 256 * k;
            w2[i >> 5][i & 31] = v[k];
        }
    }
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
    // the weight tiles staged with all of a thread's global loads in flight together (clamped
    // indices, no branches around them; a load -> LDS store loop waits a memory round trip per
    // iteration): Wi1 2048, Wf1 <= 2048, Wf2 1024, Wi2 and Wae <= 1024 floats (A <= 32)
    const int nf1 = 32 * (32 + A), ni2 = 32 * A, nae = A * A, bt = tid & 31;
    auto cl = [](int i, int n) { return i < n ? i : n - 1; };
    float ri1[8], rf1[8], rf2[4], ri2[4], rae[4], rb[4];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        ri1[k] = sg[g.wi1() + tid + 256 * k];
        rf1[k] = sg[g.wf1() + cl(tid + 256 * k, nf1)];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        rf2[k] = sg[g.wf2() + tid + 256 * k];
        ri2[k] = sg[g.wi2() + cl(tid + 256 * k, ni2)];
        rae[k] = sg[g.wae() + cl(tid + 256 * k, nae)];
    }
    rb[0] = sg[g.bi1() + bt];
    rb[1] = sg[g.bf1() + bt];
    rb[2] = sg[g.bf2() + bt];
    rb[3] = sg[g.bi2() + cl(bt, A)];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int i = tid + 256 * k;
        Wi1[i >> 6][i & 63] = ri1[k];
        if (i < nf1) Wf1[i / (32 + A)][i % (32 + A)] = rf1[k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = tid + 256 * k;
        Wf2[i >> 5][i & 31] = rf2[k];
        if (i < ni2) Wi2[i >> 5][i & 31] = ri2[k];
        if (i < nae) Wae[i / A][i % A] = rae[k];
    }
    if (tid < 32) {
        bi1[tid] = rb[0];
        bf1[tid] = rb[1];
        bf2[tid] = rb[2];
        bi2[tid] = tid < A ? rb[3] : 0.f;
    }
    if (tid < PB) {
        const long long jj = blockIdx.x * (long long)PB + tid;
        long long j = -1;
        if (jj < a.npl) j = a.pairs ? a.pairs[jj] : jj;
        if (j >= a.B - 1) j = -1;  // a listed position with no pair (the minibatch's last row)
        jrow[tid] = j;
        // actions NULL: the minibatch's actions are the B floats after phi (ppox_icm_scatter_positions)
        act[tid] = j < 0 ? 0
                   : a.actions ? a.actions[a.rowno ? (long long)a.rowno[j] : j]
                               : (int)a.phi[a.B * H + j];
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
// written in the A-fragment order of the weight-gradient MFMA,
// gq[(rs * 64 + lane) * 8 + e] = g1[16 rs + 8 (lane >> 5) + e][lane & 31] (f32), and each
// block's per-column max |g1| (f32 bits) into gmax[block][32] (the split scale of column n).
// ---------------------------------------------------------------------------
struct RowArgs {
    const float* dS;
    const float* dN;         // may be null (already summed into dS)
    const long long* pos;    // local row -> minibatch position (null: identity)
    long long M;
    const float* pre1;
    const float* seg;
    float4* gq;
    uint32_t* gmax;
    float* slab;
    int stride;
};

__global__ void __launch_bounds__(256) icm_row_bwd_kernel(RowArgs a) {
    __shared__ float W2[32][33], D[RB][33], A1[RB][33], P[RB][33], G[RB][33];
    const int tid = threadIdx.x;
    // a thread's four rows loaded with no branch around the loads (clamped rows, dN read from dS
    // when absent and not added), so they are in flight together; then the LDS stores
    static_assert(RB * 32 == 4 * 256, "row kernel: four elements per thread");
    const float* dN = a.dN ? a.dN : a.dS;
    float w2v[4], dv[4], nv[4], pv[4];
    long long src[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = tid + 256 * k;
        const long long r = blockIdx.x * (long long)RB + (i >> 5), rc = r < a.M ? r : a.M - 1;
        w2v[k] = a.seg[32 + i];
        src[k] = rc;
        pv[k] = a.pre1[rc * H + (i & 31)];
    }
    if (a.pos) {  // uniform
#pragma unroll
        for (int k = 0; k < 4; ++k) src[k] = a.pos[src[k]];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int c = (tid + 256 * k) & 31;
        dv[k] = a.dS[src[k] * H + c];
        nv[k] = dN[src[k] * H + c];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = tid + 256 * k, rr = i >> 5, c = i & 31;
        const bool ok = blockIdx.x * (long long)RB + rr < a.M;
        W2[i >> 5][i & 31] = w2v[k];
        const float d = a.dN ? dv[k] + nv[k] : dv[k], pre = pv[k];
        D[rr][c] = ok ? d : 0.f;
        P[rr][c] = ok ? pre : 0.f;
        A1[rr][c] = leaky(ok ? pre : 0.f);
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
        const long long rs = blockIdx.x * (long long)(RB / 16) + rsl;
        a.gq[(rs * 64 + lane) * 2] = make_float4(G[r0][n], G[r0 + 1][n], G[r0 + 2][n], G[r0 + 3][n]);
        a.gq[(rs * 64 + lane) * 2 + 1] = make_float4(G[r0 + 4][n], G[r0 + 5][n], G[r0 + 6][n], G[r0 + 7][n]);
    } else if (tid < 64 * (RB / 16) + 32) {
        const int n = tid - 64 * (RB / 16);
        uint32_t m = 0u;
        for (int rr = 0; rr < RB; ++rr) m = max(m, __float_as_uint(fabsf(G[rr][n])));
        a.gmax[blockIdx.x * 32LL + n] = m;
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
// 32 columns, column 4 j + t of the block in tile t), all rows, 8 waves.  Column n of g1 is
// split with its own exponent E[n] (from the row blocks' gmax: every lane splits the column
// n = lane & 31 of its A fragment, the output row n is unscaled by 2^-E[n]).  Wave w takes
// the 16-row steps rs = w, w + 8, ...: per step a lane loads one dword (4 columns) from
// each of 8 rows (row 16 rs + 8 (lane >> 5) + e) — 128 contiguous bytes per row per
// half-wave — and byte t of the 8 dwords is tile t's B fragment (exact f16: 0x64bb is
// 1024 + b); the A fragment is the lane's 8 g1 values split into two f16 planes.
// WG_STAGES steps are in flight per wave.  The waves' sums are added in LDS in wave order
// and stored as float4 rows.
// ---------------------------------------------------------------------------
constexpr int WG_CHUNK = 2048;  // rows whose frame-row numbers are staged in LDS at a time
constexpr int WG_WAVES = 8;
constexpr int ICM_WG_STAGES = 3;
constexpr int WG_STAGES = ICM_WG_STAGES;

struct WgArgs {
    const uint8_t* x;
    const unsigned* rowno;
    long long M;
    int K;
    const float4* gq;
    const uint32_t* gmax;
    int nblk;
    float* dw;
};

// byte t of rows (w0, w1) as an exact f16 pair
__device__ inline uint32_t u8pair_to_f16(uint32_t w0, uint32_t w1, int t) {
    // v_perm (selector t: byte t of w0, 4 + t: of w1, 12: 0x00) -> [b0, 0, b1, 0], | the 0x64
    // exponent bytes, minus 1024
    const uint32_t sel = (uint32_t)t | (12u << 8) | ((uint32_t)(4 + t) << 16) | (12u << 24);
    const uint32_t v = __builtin_amdgcn_perm(w1, w0, sel) | 0x64006400u;
    const f16x2 k1024 = {(_Float16)1024.f, (_Float16)1024.f};
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(f16x2, v) - k1024);
}

__global__ void __launch_bounds__(64 * WG_WAVES) icm_enc_wgrad_kernel(WgArgs a) {
    __shared__ unsigned rows_l[WG_CHUNK];
    __shared__ float4 red[WG_WAVES][32][32];  // [wave][n][column quad]
    __shared__ uint32_t em[WG_WAVES * 64];
    __shared__ int ex[32];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 31, hb = lane >> 5;
    // column n's exponent: max over the row blocks' gmax (thread tid: column tid & 31, blocks
    // tid >> 5, + 16, ...)
    {
        uint32_t m = 0u;
        for (int b = tid >> 5; b < a.nblk; b += WG_WAVES * 2) m = max(m, a.gmax[b * 32LL + (tid & 31)]);
        em[tid] = m;
        __syncthreads();
        if (tid < 32) {
            uint32_t mm = em[tid];
#pragma unroll
            for (int i = 1; i < WG_WAVES * 2; ++i) mm = max(mm, em[i * 32 + tid]);
            ex[tid] = split_scale_exp(mm);
        }
        __syncthreads();
    }
    const float sg = exp2i(ex[j]);  // the lane's A column n = j
    // an XCD's workgroups take adjacent column blocks, so the 128-B pieces of one frame row that
    // they read at about the same time are neighbours (2048 rows: 20.0 -> 18.3 us)
    const long long k0 = xcd_remap(blockIdx.x, gridDim.x) * 128LL;
    // columns past K (last block): a valid address, results never stored
    const uint8_t* xc = a.x + std::min<long long>(k0 + 4 * j, a.K - 4);
    f32x16 hi[4], lo[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) hi[t] = lo[t] = zero16();
    const long long RS = (a.M + 15) / 16;
    using Xs = uint32_t[8];
    using Gs = float4[2];
    auto load = [&](long long rs, long long c0, Xs& xv, Gs& gv) {
        const int rl = (int)(rs * 16 - c0) + 8 * hb;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const unsigned row = rows_l[rl + e];
            xv[e] = *reinterpret_cast<const uint32_t*>(xc + (long long)row * a.K);
        }
        gv[0] = a.gq[(rs * 64 + lane) * 2];
        gv[1] = a.gq[(rs * 64 + lane) * 2 + 1];
    };
    auto step = [&](const Xs& xv, const Gs& gv) {
        u32x4 g0, g1;
        split8h(gv[0], gv[1], sg, g0, g1);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            u32x4 b;
#pragma unroll
            for (int q = 0; q < 4; ++q) b[q] = u8pair_to_f16(xv[2 * q], xv[2 * q + 1], t);
            hi[t] = mfma_f16(g0, b, hi[t]);
            lo[t] = mfma_f16(g1, b, lo[t]);
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
        const float u = exp2i(-ex[n]);
        red[wave][n][j] = make_float4((hi[0][e] + lo[0][e]) * u, (hi[1][e] + lo[1][e]) * u,
                                      (hi[2][e] + lo[2][e]) * u, (hi[3][e] + lo[3][e]) * u);
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
    // every global load of a thread issued before its LDS stores (clamped, branch-free; see the
    // pair kernel): Wf1 <= 2048 and Wf2 1024 floats, the row's features, action and biases
    const int nf1 = 32 * (32 + A);
    const long long r = blockIdx.x * 8LL + rr;
    const bool ok = r < N;
    const long long rc = ok ? r : N - 1;
    float rf1[8], rf2[4];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int i = tid + 256 * k;
        rf1[k] = seg[g.wf1() + (i < nf1 ? i : nf1 - 1)];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) rf2[k] = seg[g.wf2() + tid + 256 * k];
    const int act = actions[rc];
    const float ys = phi_s[rc * H + c], yn = phi_n[rc * H + c];
    const float b1 = seg[g.bf1() + c], b2 = seg[g.bf2() + c];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int i = tid + 256 * k;
        if (i < nf1) Wf1[i / (32 + A)][i % (32 + A)] = rf1[k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = tid + 256 * k;
        Wf2[i >> 5][i & 31] = rf2[k];
    }
    Y[rr][c] = ok ? ys : 0.f;
    if (c < A) Y[rr][32 + c] = seg[g.wae() + (ok ? act : 0) * A + c];
    __syncthreads();
    float v = 0.f;
    for (int k = 0; k < 32 + A; ++k) v += Wf1[c][k] * Y[rr][k];
    Vv[rr][c] = leaky(v + b1);
    __syncthreads();
    float nh = 0.f;
#pragma unroll 8
    for (int k = 0; k < 32; ++k) nh += Wf2[c][k] * Vv[rr][k];
    nh = nh + b2;
    const float d = nh - (ok ? yn : 0.f);
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

// host: encoder-forward launch shape for `rows`: ceil(M / 256) row groups x nkc K ranges,
// ~ICM_FWD_WGS workgroups, at least 4 chunks per K range
struct EncShape {
    int nrg, nkc;
};
constexpr int ICM_FWD_WGS = 256;
EncShape enc_shape(long long M, int K) {
    EncShape s;
    s.nrg = (int)ppox::ceil_div(M, (long long)ENC_ROWS);
    const int nc = K / ENC_CK;
    s.nkc = std::max(1, std::min<int>(ppox::ceil_div(ICM_FWD_WGS, s.nrg), std::max(1, nc / 4)));
    return s;
}

bool icm_shape_ok(long long K) { return K > 0 && K % ENC_CK == 0 && K < (1LL << 30); }
long long g1_blocks(long long rows) { return ppox::ceil_div(rows, (long long)RB); }
long long g1_frag_floats(long long rows) { return g1_blocks(rows) * (RB / 16) * 64 * 8; }

}  // namespace

extern "C" int64_t ppox_icm_param_elems(int32_t n_actions) {
    if (n_actions < 1 || n_actions > 32) return -1;
    return Seg(n_actions).n();
}

extern "C" int64_t ppox_icm_w1_pack_elems(int64_t K) { return icm_shape_ok(K) ? 2LL * H * K + 2 * H : -1; }

extern "C" int ppox_icm_pack_w1(const float* w1, int64_t K, uint16_t* q, void* stream) {
    PPOX_REQUIRE(w1 && q && icm_shape_ok(K), "ppox_icm_pack_w1: bad arguments (K must be a positive multiple of 64)");
    PPOX_REQUIRE(ppox::aligned16(w1) && ppox::aligned16(q), "ppox_icm_pack_w1: 16-byte alignment");
    icm_pack_w1_kernel<<<H * ICM_W1_PARTS, 1024, 0, ppox::as_stream(stream)>>>(w1, (int)K, reinterpret_cast<u32x4*>(q));
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
                 "ppox_icm_encode: bad arguments (K must be a positive multiple of 64)");
    PPOX_REQUIRE(ppox::aligned16(x) && ppox::aligned16(q), "ppox_icm_encode: 16-byte alignment");
    if (idx) PPOX_REQUIRE(T > 0 && N_env > 0 && T * N_env < (1LL << 32), "ppox_icm_encode: idx needs T, N_env");
    else PPOX_REQUIRE(rows < (1LL << 32), "ppox_icm_encode: too many rows");
    const EncShape s = enc_shape(rows, (int)K);
    hipStream_t st = ppox::as_stream(stream);
    float* slab = reinterpret_cast<float*>(workspace);
    EncArgs a{reinterpret_cast<const uint8_t*>(x), reinterpret_cast<const long long*>(idx), T, N_env, rows, (int)K,
              reinterpret_cast<const u32x4*>(q), slab, s.nkc, s.nrg};
    icm_enc_fwd_kernel<<<(unsigned)(s.nkc * s.nrg), 64 * ENC_WAVES, 0, st>>>(a);
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

// g1 in fragment order (f32) then the row blocks' per-column gmax, in uint16 units
extern "C" int64_t ppox_icm_g1_pack_elems(int64_t rows) {
    return rows <= 0 ? 0 : 2 * (g1_frag_floats(rows) + g1_blocks(rows) * 32);
}

// The sharded minibatch's features and actions at their minibatch positions (world > 1): fa = [B x 32
// features | B actions as f32], zero where another rank owns the row, for one all-reduce.  Thread t of
// the grid: feature float4 (t >> 3) of owned row ((t >> 3) / 8) ... one float4 per thread, the action with
// the row's first quarter.
__global__ void __launch_bounds__(256) icm_scatter_kernel(const float4* __restrict__ phi,
                                                          const int32_t* __restrict__ actions,
                                                          const uint32_t* __restrict__ rowno,
                                                          const long long* __restrict__ pos, long long rows,
                                                          long long B, float* __restrict__ fa) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;  // (row, float4 of its 8)
    if (t >= rows * (H / 4)) return;
    const long long i = t / (H / 4);
    const int q = (int)(t % (H / 4));
    const long long p = pos[i];
    reinterpret_cast<float4*>(fa + p * H)[q] = phi[t];
    if (q == 0) fa[B * H + p] = (float)actions[rowno[i]];
}

extern "C" int ppox_icm_scatter_positions(const float* phi, const int32_t* actions, const uint32_t* rowno,
                                          const int64_t* pos, int64_t rows, int64_t B, float* fa, void* stream) {
    PPOX_REQUIRE(fa && B >= 1 && rows >= 0 && rows <= B && (rows == 0 || (phi && actions && rowno && pos)),
                 "ppox_icm_scatter_positions: bad arguments");
    PPOX_REQUIRE(ppox::aligned16(fa) && (!phi || ppox::aligned16(phi)), "ppox_icm_scatter_positions: 16B alignment");
    hipStream_t s = ppox::as_stream(stream);
    PPOX_REQUIRE(hipMemsetAsync(fa, 0, sizeof(float) * B * (H + 1), s) == hipSuccess,
                 "ppox_icm_scatter_positions: memset failed");
    if (rows == 0) return PPOX_OK;
    icm_scatter_kernel<<<ppox::ceil_div(rows * (H / 4), 256LL), 256, 0, s>>>(
        reinterpret_cast<const float4*>(phi), actions, rowno, reinterpret_cast<const long long*>(pos), rows, B, fa);
    PPOX_LAUNCHED("ppox_icm_scatter_positions");
}

extern "C" int ppox_icm_pair_backward(const float* phi, int64_t B, const int32_t* actions, const uint32_t* rowno,
                                      const int64_t* pairs, int64_t n_pairs, int64_t n_pairs_global,
                                      int32_t n_actions, float beta, const float* seg, float* dS, float* dN,
                                      float* partials, void* stream) {
    PPOX_REQUIRE(phi && (actions || pairs) && seg && dS && dN && partials && B >= 1 && n_pairs >= 0 &&
                     n_pairs <= B && n_pairs_global < B && n_actions >= 1 && n_actions <= 32,
                 "ppox_icm_pair_backward: bad arguments");
    PPOX_REQUIRE(pairs || n_pairs == B - 1, "ppox_icm_pair_backward: without a pair list every j < B - 1 is a pair");
    hipStream_t s = ppox::as_stream(stream);
    if (pairs) {  // only the listed pairs' rows are written: the rest of dS / dN is zero
        PPOX_REQUIRE(hipMemsetAsync(dS, 0, sizeof(float) * B * H, s) == hipSuccess &&
                         hipMemsetAsync(dN, 0, sizeof(float) * B * H, s) == hipSuccess,
                     "ppox_icm_pair_backward: memset failed");
    }
    PairArgs a{phi, B, actions, rowno, reinterpret_cast<const long long*>(pairs), n_pairs, n_pairs_global,
               1.f - beta, beta, seg, n_actions, dS, dN, partials};
    const unsigned nb = std::max(1u, ppox::ceil_div(n_pairs, PB));
    icm_pair_kernel<<<nb, 256, 0, s>>>(a);
    PPOX_LAUNCHED("ppox_icm_pair_backward");
}

extern "C" int ppox_icm_row_backward(const float* dS, const float* dN, const int64_t* pos, int64_t rows,
                                     const float* pre1, const float* seg, int32_t n_actions, uint16_t* g1q,
                                     float* partials, void* stream) {
    if (rows == 0) return PPOX_OK;
    PPOX_REQUIRE(dS && pre1 && seg && g1q && partials && rows > 0 && n_actions >= 1 && n_actions <= 32,
                 "ppox_icm_row_backward: bad arguments");
    PPOX_REQUIRE(ppox::aligned16(g1q), "ppox_icm_row_backward: 16-byte alignment");
    float* gq = reinterpret_cast<float*>(g1q);
    RowArgs a{dS, dN, reinterpret_cast<const long long*>(pos), rows, pre1, seg, reinterpret_cast<float4*>(gq),
              reinterpret_cast<uint32_t*>(gq + g1_frag_floats(rows)), partials, Seg(n_actions).stride()};
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
    // the g1 fragments cover whole RB-row blocks: the last 16-row step is inside them
    const float* gq = reinterpret_cast<const float*>(g1q);
    WgArgs a{reinterpret_cast<const uint8_t*>(x), rowno, rows, (int)K, reinterpret_cast<const float4*>(gq),
             reinterpret_cast<const uint32_t*>(gq + g1_frag_floats(rows)), (int)g1_blocks(rows), dw1};
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
