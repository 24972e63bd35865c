// K6 — NatureCNN convolutions as implicit GEMMs on the fp32 matrix cores
// (v_mfma_f32_32x32x2_f32: exact f32 FMAs at the gfx950 fp32 matrix rate,
// 157 TF/s dense).  Replaces torch.nn.Conv2d + ReLU (forward) and their
// autograd (backward) of .ipynb_checkpoints/models-checkpoint.py:52-58:
//   conv1 4->32 k8 s4 (84x84 -> 20x20), conv2 32->64 k4 s2 (-> 9x9),
//   conv3 64->64 k3 s1 (-> 7x7).
//
// Activation layout: NHWC between layers (a 32-channel run = one 128-byte row
// segment, so every im2col gather is coalesced); the trunk output is NCHW (the
// reference's Flatten order feeding Linear(3136, 512)).  conv1 reads the uint8
// frame stack (N, 4, 84, 84) directly: the torch.FloatTensor(obs) conversion is
// fused (u8 -> f32 is exact), and so is the minibatch gather (rows via idx).
//
// Forward / dgrad: M = output rows, N = channels, K = taps x channels.  One
// 256-thread workgroup owns BM = 128 rows x all N channels; each wave 32 rows
// (N/32 MFMA tiles).  K is walked in BK = 32 chunks, register-staged and
// double-buffered in LDS (one barrier per chunk) so the gathers of chunk c+1 fly
// under the MFMAs of chunk c.  Each thread's four staged rows are fixed for the
// whole K walk, so their base addresses are computed once.
//   forward epilogue: + bias, ReLU
//   dgrad epilogue:   x (previous activation > 0) — the previous layer's ReLU
//                     backward is fused, the result is that layer's output grad
//   conv2 dgrad (stride 2) runs as 4 parity classes of the input grid, each a
//   dense GEMM over its 2x2 contributing taps (no zero MACs).
// Wgrad: dW[k][co] = sum_m A[m][k] G[m][co] — a GEMM whose reduction runs over
// all output pixels.  Workgroups own a K-block and a slice of M (split-K over
// pixels), write partial slabs, and a reduce kernel sums the slabs in a FIXED
// order (deterministic) straight into the PyTorch [co][ci][ky][kx] layout; the
// bias gradient is fused into the k-block-0 workgroups.  The k-blocks of one
// M-slice are mapped to one XCD (blockIdx % 8) so their shared G rows and
// overlapping input patches are served from that XCD's L2.
#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <type_traits>
#include <unordered_set>

#include <utility>

#include "conv_common.h"

namespace {


constexpr int BK = 32;
constexpr int AST = BK + 1;  // padded LDS row stride (floats): conflict-free column reads

// ---------------------------------------------------------------------------
// A stagers: global -> registers (load) -> LDS (store), 4*MT slots per thread.
// Slot i of thread t covers element w = i*256 + t of the (128*MT) x BK chunk.
// Rows past the end read a valid clamped address and are zeroed by a select: a
// conditional load would make hipcc branch around every load (execz) and
// serialise them.
// ---------------------------------------------------------------------------
struct RowTile {  // forward: a contiguous run of output pixels
    long long m0, M;
};

// f32 rows of 32 floats (8 float4 per row) -> LDS
template <int SL>
__device__ inline void store_rows_f4(float* As, const float4 (&r)[SL]) {
#pragma unroll
    for (int i = 0; i < SL; ++i) {
        const int w = i * 256 + threadIdx.x;
        float* d = As + (w >> 3) * AST + (w & 7) * 4;
        d[0] = r[i].x;
        d[1] = r[i].y;
        d[2] = r[i].z;
        d[3] = r[i].w;
    }
}

// NHWC f32 forward (conv2, conv3): K order (ky, kx, ci); chunk = 32 channels of one tap.
template <class L, int MT>
struct StageFwdNHWC {
    static constexpr int SL = 4 * MT;
    const float* base[SL];
    bool ok[SL];
    float4 r[SL];
    __device__ StageFwdNHWC(const Args& a, const RowTile& t) {
        const float* x = reinterpret_cast<const float*>(a.x);
#pragma unroll
        for (int i = 0; i < SL; ++i) {
            const int w = i * 256 + threadIdx.x;
            const int row = w >> 3, q = w & 7;
            const long long m = t.m0 + row;
            ok[i] = m < t.M;
            const long long mm = ok[i] ? m : t.m0;
            const long long n = mm / L::P;
            const int p = (int)(mm - n * L::P), oy = p / L::OW, ox = p % L::OW;
            base[i] = x + ((n * L::IH + oy * L::S) * L::IW + ox * L::S) * L::CIN + q * 4;
        }
    }
    __device__ inline void load(int chunk) { load_to(chunk, r); }
    __device__ inline void load_to(int chunk, float4 (&r)[SL]) const {
        constexpr int CPT = L::CIN / BK;
        const int tap = chunk / CPT, ky = tap / L::KW, kx = tap % L::KW;
        const int off = (ky * L::IW + kx) * L::CIN + (chunk % CPT) * BK;
        // rows past the end read a clamped valid row; their C rows are never stored
#pragma unroll
        for (int i = 0; i < SL; ++i) r[i] = *reinterpret_cast<const float4*>(base[i] + off);
    }
    __device__ inline void store(float* As) const { store_rows_f4<SL>(As, r); }
};

template <int NOUT>
struct StageB {
    static constexpr int V = BK * NOUT / 4 / 256;  // float4 per thread
    float4 r[V];
    __device__ inline void load(const float* chunk_base) {
        const float4* src = reinterpret_cast<const float4*>(chunk_base);
#pragma unroll
        for (int i = 0; i < V; ++i) r[i] = src[i * 256 + threadIdx.x];
    }
    __device__ inline void store(float* Bs) const {
#pragma unroll
        for (int i = 0; i < V; ++i) reinterpret_cast<float4*>(Bs)[i * 256 + threadIdx.x] = r[i];
    }
};

// ---------------------------------------------------------------------------
// Problems: tile of a block, chunk count, stagers, packed-B chunk, epilogue.
// ---------------------------------------------------------------------------
template <class L, bool OUT_NCHW, int MT_>
struct FwdBase {
    static constexpr int NOUT = L::COUT, MT = MT_, BMR = 128 * MT;
    static constexpr bool A_PLANES = false;  // sg2: A rows are f32 (split in registers), not H1P planes
    static constexpr bool PLANES_OUT = false;  // sg2: the output as PX planes (Px<> below)
    using Tile = RowTile;
    __device__ static bool tile(const Args& a, Tile& t) {
        t.m0 = (long long)blockIdx.x * BMR;
        t.M = a.batch * L::P;
        return true;
    }
    __device__ static int nchunk(const Tile&) { return L::K / BK; }
    __device__ static const float* bchunk(const Args& a, const Tile&, int c) { return a.wp + (long long)c * BK * NOUT; }
    __device__ static int bchunk_id(const Tile&, int c) { return c; }  // 32-row block of the packed [K][NOUT]
    __device__ static float prefetch(const Args& a, const Tile&, int, int co) { return a.bias[co]; }
    // stores one output element; returns it (0 for rows past the end: the amax of the output)
    __device__ static float store_pre(const Args& a, const Tile& t, int row, int co, float acc, float bias) {
        const long long m = t.m0 + row;
        if (m >= t.M) return 0.f;
        const float v = fmaxf(acc + bias, 0.f);
        if constexpr (OUT_NCHW) {
            const long long n = m / L::P;
            a.y[(n * L::COUT + co) * L::P + (m - n * L::P)] = v;
        } else {
            a.y[m * L::COUT + co] = v;
        }
        return v;
    }
    // PX epilogue (NHWC output): the value (0 past the end) and its f32-layout element index (-1: none)
    __device__ static float value(const Args&, const Tile& t, int row, int, float acc, float bias) {
        return t.m0 + row < t.M ? fmaxf(acc + bias, 0.f) : 0.f;
    }
    __device__ static long long out_elem(const Args&, const Tile& t, int row, int co) {
        const long long m = t.m0 + row;
        return m < t.M ? m * L::COUT + co : -1;
    }
};

template <class L, bool OUT_NCHW, int MT>
struct FwdNHWCProblem : FwdBase<L, OUT_NCHW, MT> {
    using Stager = StageFwdNHWC<L, MT>;
};

// dgrad (transposed conv) of layer L, position-major: a block owns ONE input
// pixel (iy, ix) of 128*MT consecutive samples, so every row of the tile has the
// same contributing taps — exactly those (ky, kx) with iy = S*oy + ky inside the
// output grid.  The K walk covers only those taps (no zero MACs: conv3 borders
// have 4-6 of 9, every conv2 pixel 1-4 of 16).  K order (tap, co); chunk = 32
// output channels of one tap, gathered from the NHWC output grad G at the same
// (oy, ox) for every row.  Epilogue: x (previous activation > 0), NHWC.
// Blocks -> (sample tile, pixel) XCD-aware: one XCD walks the pixels of one
// sample tile, whose G rows then stay in that XCD's L2.
struct PixelTile {
    long long n0;
    int pos, iy, ix, ky0, kx0, nx, nchunk;
};

template <class L, int MT>
struct StageDgradPM {
    static constexpr int SL = 4 * MT, CPT = L::COUT / BK;
    const float* base[SL];
    bool ok[SL];
    float4 r[SL];
    int iy, ix, ky0, kx0, nx;
    __device__ StageDgradPM(const Args& a, const PixelTile& t)
        : iy(t.iy), ix(t.ix), ky0(t.ky0), kx0(t.kx0), nx(t.nx) {
        const float* g = reinterpret_cast<const float*>(a.x);
#pragma unroll
        for (int i = 0; i < SL; ++i) {
            const int w = i * 256 + threadIdx.x;
            const long long n = t.n0 + (w >> 3);
            ok[i] = n < a.batch;
            base[i] = g + (ok[i] ? n : t.n0) * (L::P * L::COUT) + (w & 7) * 4;
        }
    }
    __device__ inline void load(int chunk) { load_to(chunk, r); }
    __device__ inline void load_to(int chunk, float4 (&r)[SL]) const {
        const int tap = chunk / CPT, ty = tap / nx, tx = tap - ty * nx;
        const int oy = (iy - ky0) / L::S - ty, ox = (ix - kx0) / L::S - tx;
        const int off = (oy * L::OW + ox) * L::COUT + (chunk % CPT) * BK;
        // rows past the end read a clamped valid row; their C rows are never stored
#pragma unroll
        for (int i = 0; i < SL; ++i) r[i] = *reinterpret_cast<const float4*>(base[i] + off);
    }
    __device__ inline void store(float* As) const { store_rows_f4<SL>(As, r); }
};

template <class L, int MT_>
struct DgradPMProblem {
    static constexpr int NOUT = L::CIN, MT = MT_, BMR = 128 * MT, NPOS = L::IH * L::IW, CPT = L::COUT / BK;
    static constexpr bool A_PLANES = false;
    static constexpr bool PLANES_OUT = false;
    using Tile = PixelTile;
    using Stager = StageDgradPM<L, MT>;
    __device__ static bool tile(const Args& a, Tile& t) {
        const long long w = xcd_remap(blockIdx.x, gridDim.x);
        t.n0 = (w / NPOS) * BMR;
        t.pos = (int)(w % NPOS);
        t.iy = t.pos / L::IW;
        t.ix = t.pos % L::IW;
        int ny, nx;
        tap_range<L::S, L::OH, L::KH>(t.iy, t.ky0, ny);
        tap_range<L::S, L::OW, L::KW>(t.ix, t.kx0, nx);
        t.nx = nx;
        t.nchunk = ny * nx * CPT;
        return true;
    }
    __device__ static int nchunk(const Tile& t) { return t.nchunk; }
    __device__ static const float* bchunk(const Args& a, const Tile& t, int c) {
        const int tap = c / CPT, ty = tap / t.nx, tx = tap - ty * t.nx;
        const int ky = t.ky0 + L::S * ty, kx = t.kx0 + L::S * tx;
        return a.wp + ((long long)(ky * L::KW + kx) * L::COUT + (c % CPT) * BK) * L::CIN;
    }
    __device__ static int bchunk_id(const Tile& t, int c) {
        const int tap = c / CPT, ty = tap / t.nx, tx = tap - ty * t.nx;
        return ((t.ky0 + L::S * ty) * L::KW + t.kx0 + L::S * tx) * CPT + c % CPT;
    }
    // the epilogue's ReLU-mask values are loaded before the K walk (their latency
    // hides under it) — 16 per lane per column tile, in the C/D layout
    __device__ static float prefetch(const Args& a, const Tile& t, int row, int ci) {
        long long n = t.n0 + row;
        n = n < a.batch ? n : t.n0;
        return a.mask[(n * NPOS + t.pos) * L::CIN + ci];
    }
    __device__ static float store_pre(const Args& a, const Tile& t, int row, int ci, float acc, float m) {
        const long long n = t.n0 + row;
        if (n >= a.batch) return 0.f;
        const float v = m > 0.f ? acc : 0.f;
        a.y[(n * NPOS + t.pos) * L::CIN + ci] = v;
        return v;
    }
    __device__ static float value(const Args& a, const Tile& t, int row, int, float acc, float m) {
        return t.n0 + row < a.batch && m > 0.f ? acc : 0.f;
    }
    __device__ static long long out_elem(const Args& a, const Tile& t, int row, int ci) {
        const long long n = t.n0 + row;
        return n < a.batch ? (n * NPOS + t.pos) * L::CIN + ci : -1;
    }
};

// One 256-thread workgroup: 128*MT rows x NOUT columns; each wave 32*MT rows
// (MT x NT MFMA tiles).  K walked in BK = 32 chunks, register-staged and
// double-buffered in LDS, one barrier per chunk.
template <class Prob>
__global__ void __launch_bounds__(256, 2) igemm_kernel(Args a) {
    constexpr int NOUT = Prob::NOUT, NT = NOUT / 32, MT = Prob::MT, BMR = 128 * MT;
    __shared__ float As[2][BMR * AST];
    __shared__ __attribute__((aligned(16))) float Bs[2][BK * NOUT];
    typename Prob::Tile t;
    if (!Prob::tile(a, t)) return;
    const int nchunk = Prob::nchunk(t);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;

    f32x16 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = zero16();
    // epilogue operands (bias / ReLU mask) in the C/D layout, loaded up front
    f32x16 pre[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                pre[i][j][r] = Prob::prefetch(a, t, wave * 32 * MT + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5),
                                              j * 32 + (lane & 31));

    typename Prob::Stager sa(a, t);
    StageB<NOUT> sb;
    if (nchunk > 0) {
        sa.load(0);
        sb.load(Prob::bchunk(a, t, 0));
        sa.store(As[0]);
        sb.store(Bs[0]);
    }
    __syncthreads();

    const int arow = wave * 32 * MT + (lane & 31);
    const int khalf = lane >> 5;
    for (int c = 0; c < nchunk; ++c) {
        const int cur = c & 1;
        if (c + 1 < nchunk) {
            sa.load(c + 1);
            sb.load(Prob::bchunk(a, t, c + 1));
        }
        const float* A = As[cur] + arow * AST + khalf;
        const float* B = Bs[cur] + khalf * NOUT + (lane & 31);
#pragma unroll
        for (int kk = 0; kk < BK / 2; ++kk) {
            float av[MT];
#pragma unroll
            for (int i = 0; i < MT; ++i) av[i] = A[i * 32 * AST + kk * 2];
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const float bv = B[kk * 2 * NOUT + j * 32];
#pragma unroll
                for (int i = 0; i < MT; ++i)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv, acc[i][j], 0, 0, 0);
            }
        }
        if (c + 1 < nchunk) {
            sa.store(As[cur ^ 1]);
            sb.store(Bs[cur ^ 1]);
        }
        __syncthreads();
    }
    // C/D map: col = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int col = j * 32 + (lane & 31);
#pragma unroll
            for (int r = 0; r < 16; ++r)
                Prob::store_pre(a, t, wave * 32 * MT + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5), col,
                                acc[i][j][r], pre[i][j][r]);
        }
}


// ---------------------------------------------------------------------------
// Pre-split B operands of the split-f16 GEMMs (sgemm_kernel, the wgrad-free kernels): a
// [K][NOUT] matrix times 2^E as two fp16 planes in MFMA fragment order, followed by the
// buffer's tail (pack_tail): the weight tensor's amax partials and the exponent E.
// ---------------------------------------------------------------------------
// packed position of natural element (row k, col) of a [K][nout] matrix, plane p:
// chunk (k / 32) x k-step s x column tile j x plane x lane (h, col & 31) x e
__host__ __device__ constexpr long long split_frag_index(int k, int col, int nout, int p) {
    const int ch = k >> 5, kl = k & 31, s = kl >> 4, h = (kl >> 3) & 1, e = kl & 7;
    const int nt = nout / 32, j = col >> 5, l = h * 32 + (col & 31);
    return ((((long long)(ch * 2 + s) * nt + j) * NPL + p) * 64 + l) * 8 + e;
}

// Output-major split packing: unit u = one 16-B fragment run (8 consecutive k of one
// column, both planes) of the split_frag_index layout of a [K][NOUT] matrix — its
// eight source values are gathered (coalesced across lanes: adjacent units are adjacent
// columns), scaled by s and written as two 16-B stores, instead of 2-B stores scattered.
template <int NOUT, class Src>
__device__ inline void pack_frag_unit(const Src& src, float s, uint16_t* __restrict__ q, long long u) {
    constexpr int NT = NOUT / 32;
    const int l = (int)(u & 63);
    const long long r = u >> 6;
    const int j = (int)(r % NT);
    const long long cs = r / NT;  // 32-row chunk * 2 + 16-row step
    const int col = j * 32 + (l & 31), k0 = (int)(cs * 16) + (l >> 5) * 8;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = src(k0 + e, col);
    u32x4 p0, p1;
    split8h(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), s, p0, p1);
    u32x4* d = reinterpret_cast<u32x4*>(q + ((cs * NT + j) * NPL) * 512) + l;
    d[0] = p0;
    d[64] = p1;
}

// ---------------------------------------------------------------------------
// NatureCNN hidden linear layer Linear(3136, 512) (.ipynb_checkpoints/
// models-checkpoint.py:58-59) on the split-f16 implicit-GEMM kernel: a plain GEMM
// C[M][N] = A[M][K] B[K][N] with A f32 rows (split in registers), B pre-split per
// column block of NB (zero-padded), workgroups over (row tile, column block), the
// column blocks of a row tile on one XCD (its A rows then come from that XCD's L2).
//   FC_FWD:   A = h3 (M x 3136, Flatten order), B = W^T; epilogue relu(acc + bias)
//   FC_DGRAD: A = dL/df * relu'(f) (M x 512), B = W; epilogue: the element (m, c*49 + p)
//             goes to g3[m][p][c] (NHWC) times (h3 > 0) — the trunk's ReLU backward and
//             NCHW -> NHWC transpose fused (replaces the dh3 round trip + nchw_to_nhwc_mask)
// ---------------------------------------------------------------------------
//   HEAD_DGRAD: the 512-wide hidden head layer's input grad, accumulated and masked in place:
//             y (= df) <- (f > 0) ? y + acc : 0  (the grads of the heads before it already in y)
enum { FC_FWD = 0, FC_DGRAD = 1, HEAD_DGRAD = 2 };
// The split fc kernels run in NHWC feature order: feature f = p * 64 + c of the conv3 output
// (the layout conv3's split forward writes, 128-B channel runs) is the reference's Flatten
// feature c * 49 + p of Linear(3136, 512) — the weights are packed through this permutation,
// so the forward reads h3 rows and the dgrad writes g3 rows as they lie, no transposes.
__host__ __device__ constexpr int fc_nchw_feature(int f) { return (f & 63) * 49 + (f >> 6); }
struct GemmTile {
    long long m0, M;
    int cb;
};

template <int K>
struct StageGemmRows {
    static constexpr int SL = 4;
    const float* base[SL];
    float4 r[SL];
    __device__ StageGemmRows(const Args& a, const GemmTile& t) {
        const float* x = reinterpret_cast<const float*>(a.x);
#pragma unroll
        for (int i = 0; i < SL; ++i) {
            const int w = i * 256 + threadIdx.x;
            long long m = t.m0 + (w >> 3);
            m = m < t.M ? m : t.m0;  // rows past the end: a valid clamped row, never stored
            base[i] = x + m * K + (w & 7) * 4;
        }
    }
    __device__ inline void load(int c) { load_to(c, r); }
    __device__ inline void load_to(int c, float4 (&r)[SL]) const {
#pragma unroll
        for (int i = 0; i < SL; ++i) r[i] = *reinterpret_cast<const float4*>(base[i] + c * BK);
    }
};

template <int K_, int N_, int NB, int MODE>
struct GemmRowsProblem {
    static constexpr int K = K_, N = N_, NOUT = NB, MT = 1, BMR = 128, NCB = (N + NB - 1) / NB, KC = K / BK;
    static constexpr bool LATE_EPILOGUE = true;
    static constexpr bool A_PLANES = false;
    static constexpr bool PLANES_OUT = false;
    static_assert(K % BK == 0, "K multiple of 32");
    using Tile = GemmTile;
    using Stager = StageGemmRows<K>;
    __device__ static bool tile(const Args& a, Tile& t) {
        const long long w = xcd_remap(blockIdx.x, gridDim.x);
        t.cb = (int)(w % NCB);
        t.m0 = (w / NCB) * BMR;
        t.M = a.batch;
        return true;
    }
    __device__ static int nchunk(const Tile&) { return KC; }
    __device__ static int bchunk_id(const Tile& t, int c) { return t.cb * KC + c; }
    // B is packed in 64-column blocks; a 128-column tile (NB = 128) reads blocks 2 cb and 2 cb + 1
    // (past the last block: the last again, its columns never stored)
    static constexpr int NCB64 = (N + 63) / 64;
    __device__ static int bchunk_blk(const Tile& t, int c, int b) {
        const int blk = t.cb * (NB / 64) + b;
        return (blk < NCB64 ? blk : NCB64 - 1) * KC + c;
    }
    // branch-free (clamped indices), so an epilogue can issue all its loads before any wait
    // (HEAD_DGRAD: the mask and the accumulated grad)
    __device__ static auto prefetch(const Args& a, const Tile& t, int row, int col) {
        const int n = t.cb * NB + col, nc = n < N ? n : N - 1;
        long long m = t.m0 + row;
        m = m < t.M ? m : t.m0;
        if constexpr (MODE == FC_FWD)
            return a.bias[nc];
        else if constexpr (MODE == FC_DGRAD)
            return a.mask[m * N + nc];
        else
            return make_float2(a.mask[m * N + nc], a.y[m * N + nc]);
    }
    template <class Pre>
    __device__ static float store_pre(const Args& a, const Tile& t, int row, int col, float acc, Pre e) {
        const long long m = t.m0 + row;
        const int n = t.cb * NB + col;
        if (m >= t.M || n >= N) return 0.f;
        // FC_FWD: relu(acc + bias); FC_DGRAD: g3 (NHWC) times the ReLU mask of h3 (NHWC), the same
        // index; HEAD_DGRAD: (accumulated grad + acc) times the ReLU mask of f
        float v;
        if constexpr (MODE == FC_FWD)
            v = fmaxf(acc + e, 0.f);
        else if constexpr (MODE == FC_DGRAD)
            v = e > 0.f ? acc : 0.f;
        else
            v = e.x > 0.f ? e.y + acc : 0.f;
        a.y[m * N + n] = v;
        return v;
    }
    // PX epilogue: the fc dgrad's masked g3 (FC_DGRAD only)
    __device__ static float value(const Args&, const Tile& t, int row, int col, float acc, float e) {
        static_assert(MODE == FC_DGRAD, "PX output: the fc dgrad");
        return t.m0 + row < t.M && t.cb * NB + col < N && e > 0.f ? acc : 0.f;
    }
    __device__ static long long out_elem(const Args&, const Tile& t, int row, int col) {
        const long long m = t.m0 + row;
        const int n = t.cb * NB + col;
        return m < t.M && n < N ? m * N + n : -1;
    }
};

// a Problem with PX operands: A rows as f16 planes (a.xexp; no split in registers) and / or the
// output written as planes at a bound-derived exponent (a.yexp_out, conv_common.h)
template <class Base, bool AP, bool PO = false>
struct Px : Base {
    static constexpr bool A_PLANES = AP, PLANES_OUT = PO;
};

constexpr int FC_FWD_G = 8;  // fc forward: column blocks per tile group (SgRows): all 8, each h3 row tile read once
constexpr int FC_DGRAD_G = 12;  // fc dgrad: column blocks per tile group
constexpr int FC_NB = 64;  // the packed fc / head B blocks (64 columns)
// columns per sg2 tile of the fc / head GEMMs: 64; 128 (A staged once per 128 columns, four
// column tiles per wave) measured slower — 358 registers, one wave per SIMD (round 4 same-box
// A/B: 1-GPU 427.4k vs 439.6k env-steps/s, per-rank 225.8 vs 215.5 ms)
constexpr int SG_FC_NB = 64;
// column-block groups of the wide tiles: the same column span per group as the 64-column FC_*_G
constexpr int FC_FWD_GW = FC_FWD_G * 64 / SG_FC_NB, FC_DGRAD_GW = FC_DGRAD_G * 64 / SG_FC_NB;
constexpr int HEAD_GW = 512 / SG_FC_NB;
using FcFwd = GemmRowsProblem<3136, 512, FC_NB, FC_FWD>;
using FcDgrad = GemmRowsProblem<512, 3136, FC_NB, FC_DGRAD>;
// the heads' hidden layer Linear(512, 512) + ReLU (models-checkpoint.py:62-66 extra_layer)
using HeadFwd = GemmRowsProblem<512, 512, FC_NB, FC_FWD>;
using HeadDgrad = GemmRowsProblem<512, 512, FC_NB, HEAD_DGRAD>;
static_assert(FC_NB == 64, "sg2 runs the fc layer in 64-column blocks");

// ---------------------------------------------------------------------------
// conv2 dgrad in the col2im form (split-f16), the default conv2 split dgrad.
// GEMM rows = output-grad pixels (n, oy, ox), K = the 64 output channels, columns =
// (tap, ci): 16 taps x 32 = 512.  Every A value (one G row of 64 floats) is loaded
// once, split once into its two f16 planes and kept in registers for all 512
// columns — 16x the MFMA work per A byte of the position-major form, whose
// 32-column tiles re-gathered each G row for every one of its 16 input pixels.
// A triple (3 whole samples, 243 rows on 8 waves x 32) keeps the col2im overlap inside
// one workgroup: four passes, one per input-pixel parity class (py, px), each computing
// the class's four taps (ky in {py, py+2}, kx in {px, px+2}) and adding them, in the
// fixed tap order, into an LDS image of the class's 10x10 pixels (tap (ky, kx) sends
// row (oy, ox) to class pixel (oy + ky/2, ox + kx/2)).  The class image is then masked
// with the ReLU of the layer below and written NHWC.  B = the taps' split planes
// (position-major dgrad packing: ppox_nature_pack_split which = 12).  Deterministic: a
// fixed sum order per output.
//
// Persistent: one 512-thread workgroup per CU walks the triples t = blockIdx.x,
// + gridDim.x, ... so nothing is exposed at a triple's start:
//   * B lives in a 4-slot tap ring (tap k in slot k & 3, 12 KB each) refilled two taps at
//     a time at odd steps (taps k+3, k+4 by LDS-DMA), waited one step later;
//   * the NEXT triple's G rows are DMA'd into LDS (64 KB, 16-B chunks XOR-swizzled by row
//     so the boundary's b128 reads are conflict-free) during the current triple and split
//     into the A registers at the boundary;
//   * each class's ReLU-mask operands are loaded a class ahead (at the previous class's
//     output step), and the output stores are unconditional (threads with nothing to store
//     write a dummy), so every wave's vmcnt sequence is static and the waits are counted.
// LDS: 32 KB ring + 64 KB next rows + 37.5 KB class image = 134 KB (one workgroup per CU).
// (0.645 vs 0.695 ms for the one-triple-per-workgroup form at B = 16384, same box.)
// ---------------------------------------------------------------------------
constexpr int C2S = 3, C2ROWS = C2S * 81, C2PIX = 100;
constexpr int C2OV = (C2S * C2PIX * 8 + 511) / 512;  // float4 outputs per thread per pass
constexpr int C2_ROW_DMAS = 8;                       // dmaA: the next triple's G rows, DMAs per thread
constexpr int C2_TAP_DMAS = 2;                       // dmaB2: a tap pair, DMAs per thread
// s_waitcnt immediate (gfx9 encoding) waiting for all but the n youngest vector-memory operations:
// vmcnt bits [3:0] and [15:14], expcnt [6:4] and lgkmcnt [11:8] left at "don't wait"
constexpr int waitcnt_vm(int n) { return (n & 15) | ((n >> 4) << 14) | (0x7 << 4) | (0xF << 8); }
// the class-tap step i = 0 waits for the tap pair DMA'd at the step before (i = 3 of the previous
// class); behind it that step issued the class's C2OV output stores and the next class's C2OV
// mask loads (one memory instruction each: the stores are unconditional, the loads clamped), and
// after class 0 the next triple's row DMAs
constexpr int C2_WAIT_I0 = 2 * C2OV, C2_WAIT_I0_ROWS = 2 * C2OV + C2_ROW_DMAS;
static_assert(waitcnt_vm(0) == 0x0F70 && waitcnt_vm(10) == 0x0F7A && waitcnt_vm(18) == 0x4F72, "s_waitcnt encoding");
static_assert(C2_WAIT_I0_ROWS < 64, "vmcnt is 6 bits");

// workgroup barrier that waits only for this wave's LDS operations: global loads and
// stores stay in flight across it (__syncthreads also drains vmcnt, which would expose
// every output store and prefetch at each col2im step)
__device__ inline void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

constexpr int C2P_TAP = 4 * NPL * 64;                  // u32x4 per tap: 4 k-steps x 2 planes x 64 lanes
constexpr int C2P_AN = 256 * 16;                       // u32x4: 256 G rows x 64 f32
// u32x4: class image + the dummy region (the rows past a triple's 243 land there at any tap offset)
constexpr int C2P_IMG = (C2S * C2PIX * 32 + (11 * 32 + 32)) / 4;
__device__ float4 kC2Dummy[512];                       // store target of threads with nothing to store

__device__ inline int c2_nat_tap(int k) {  // class tap k (0..15) -> natural tap ky * 4 + kx
    k &= 15;
    const int cls = k >> 2, i = k & 3;
    return ((cls >> 1) + 2 * (i >> 1)) * G2::KW + (cls & 1) + 2 * (i & 1);
}

// BITS: the ReLU mask of conv1 from the forward's bitmask (a.bits_mask, 4 B per pixel) instead
// of its f32 activations (a.mask, 128 B per pixel): 26 MB instead of 839 MB at B = 16384
// SAFE: every counted wait is vmcnt(0) (PPOX_COLP_VMCNT0=1; the tests compare both bitwise)
template <bool BITS, bool SAFE = false>
__global__ void __launch_bounds__(512, 1) dgrad2_colp_kernel(Args a, const u32x4* __restrict__ wq,
                                                            long long ntriples) {
    using L = G2;
    __shared__ u32x4 lds[4 * C2P_TAP + C2P_AN + C2P_IMG];
    u32x4* Bring = lds;
    u32x4* An = lds + 4 * C2P_TAP;
    float* Ds = reinterpret_cast<float*>(lds + 4 * C2P_TAP + C2P_AN);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const long long rows_total = a.batch * L::P;
    const float* g2 = reinterpret_cast<const float*>(a.x);

    // operand scales: G by its tensor's amax, B as packed; the output is unscaled
    const int ex = split_scale_exp(amax_read(a.amax_x)), ew = *a.wexp;
    const float sg = exp2i(ex), uo = exp2i(-ex) * exp2i(-ew);
    float om = 0.f;  // the largest |value| this thread stored (the output's amax)
    // taps k, k+1 (class-tap indices, mod 16) -> ring slots: 2 DMAs per thread
    auto dmaB2 = [&](int k) {
        static_assert(2 * C2P_TAP / 512 == C2_TAP_DMAS, "dmaB2: DMAs per thread");
#pragma unroll
        for (int r = 0; r < C2_TAP_DMAS; ++r) {
            const int e0 = r * 512 + wave * 64, which = e0 / C2P_TAP, within0 = e0 - which * C2P_TAP;
            const int kk = (k + which) & 15;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(wq + c2_nat_tap(kk) * C2P_TAP + within0 + lane),
                (__attribute__((address_space(3))) void*)(Bring + (kk & 3) * C2P_TAP + within0), 16, 0, 0);
        }
    };
    // triple t's 256 G rows (rows past the batch clamped; rows 243.. are never stored) ->
    // An, row r's 16-B chunk c at position c ^ (r & 15): 8 DMAs per thread
    auto dmaA = [&](long long t) {
        long long row0 = t * C2ROWS;
        row0 = row0 < rows_total ? row0 : rows_total - 1;  // (past the last triple: clamped, never stored)
        // uniform 64-bit base at the triple's first row + 32-bit byte offset (< 64 KB): the saddr
        // form, whose address VGPR hipcc does not make each DMA wait for (vmcnt(0)) before reusing
        const char* base = reinterpret_cast<const char*>(g2) + row0 * 256;
        const long long last = rows_total - 1 - row0;
        static_assert(C2_ROW_DMAS * 512 * 16 == 256 * 256, "dmaA: 256 rows of 256 B per triple");
#pragma unroll
        for (int j = 0; j < C2_ROW_DMAS; ++j) {
            const int r = (wave * 8 + j) * 4 + (lane >> 4), c = (lane & 15) ^ (r & 15);
            const unsigned rr = (unsigned)(r < last ? r : last);
            const unsigned off = rr * 256u + (unsigned)c * 16u;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(base + off),
                                             (__attribute__((address_space(3))) void*)(An + (wave * 8 + j) * 64), 16,
                                             0, 0);
        }
    };
    // A: this lane's row of the triple in An, k = 16q + 8h .. +8 -> two f16 planes (scaled)
    u32x4 af[4][NPL];
    auto take_A = [&]() {
        const int r = wave * 32 + (lane & 31), sw = r & 15;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int c0 = (lane >> 5) * 2 + 4 * q;
            const u32x4 v0 = An[r * 16 + (c0 ^ sw)], v1 = An[r * 16 + ((c0 + 1) ^ sw)];
            split8h(__builtin_bit_cast(float4, v0), __builtin_bit_cast(float4, v1), sg, af[q][0], af[q][1]);
        }
    };
    auto mfma_tap = [&](int k, f32x16& c) {
        const u32x4* Bt = Bring + (k & 3) * C2P_TAP + lane;
        c = zero16();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const u32x4 bf[NPL] = {Bt[q * NPL * 64], Bt[q * NPL * 64 + 64]};
            mfma_split3(af[q], bf, c, c);
        }
    };
    // col2im add of tap k into the class image: row (oy, ox) -> class pixel (oy + (i >> 1),
    // ox + (i & 1)); eight reads, then eight writes; rows past the samples -> dummy slot
    // this lane's 16 accumulator rows -> their class-image pixel at tap offset 0 (float index,
    // computed once: a tap adds only its constant offset, folded into the ds instructions);
    // rows past the triple's 243 -> the dummy region
    int dbase[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int rho = wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int s = rho / 81, p = rho - s * 81, oy = p / 9, ox = p - oy * 9;
        dbase[r] = (rho < C2ROWS ? (s * C2PIX + oy * 10 + ox) * 32 : C2S * C2PIX * 32) + (lane & 31);
    }
    auto rmw_tap = [&](auto i_tag, const f32x16& c) {
        constexpr int i = decltype(i_tag)::value;
        constexpr int toff = ((i >> 1) * 10 + (i & 1)) * 32;
#pragma unroll
        for (int r0 = 0; r0 < 16; r0 += 8) {
            float dv[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) dv[r] = Ds[dbase[r0 + r] + toff];
#pragma unroll
            for (int r = 0; r < 8; ++r) Ds[dbase[r0 + r] + toff] = dv[r] + c[r0 + r];
        }
    };
    std::conditional_t<BITS, uint32_t, float4> mk[C2OV];
    auto load_mask = [&](long long n0, int cls) {
        const int py = cls >> 1, px = cls & 1;
#pragma unroll
        for (int j = 0; j < C2OV; ++j) {
            const int e = j * 512 + tid, s = e / 800, rem = e - s * 800, pix = rem >> 3, c4 = rem & 7;
            const long long n = n0 + s;
            const int iy = 2 * (pix / 10) + py, ix = 2 * (pix % 10) + px;
            const bool ok = e < C2S * C2PIX * 8 && n < a.batch;
            const long long p = ok ? (n * L::IH + iy) * L::IW + ix : 0;
            if constexpr (BITS)
                mk[j] = a.bits_mask[p];  // one load either way: the counted vmcnt waits hold
            else
                mk[j] = *reinterpret_cast<const float4*>(a.mask + p * L::CIN + c4 * 4);
        }
    };
    // the image is read and re-zeroed with inline-asm LDS ops: a C++ access here, after the
    // step's tap DMAs, makes hipcc wait vmcnt(0) first (it cannot tell the two LDS regions apart)
    const uint32_t img0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)Ds);
    auto output = [&](long long n0, int cls) {
        const int py = cls >> 1, px = cls & 1;
        const u32x4 zero4 = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int j = 0; j < C2OV; ++j) {
            const int e = j * 512 + tid, s = e / 800, rem = e - s * 800, pix = rem >> 3, c4 = rem & 7;
            const bool in = e < C2S * C2PIX * 8;
            const uint32_t da = img0 + (uint32_t)(in ? e : C2S * C2PIX * 8) * 16u;
            u32x4 dr;
            asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)\n\tds_write_b128 %1, %2"
                         : "=&v"(dr) : "v"(da), "v"(zero4) : "memory");
            const float4 d = __builtin_bit_cast(float4, dr);
            bool on[4];
            if constexpr (BITS) {
                const uint32_t w = mk[j] >> (c4 * 4);
                on[0] = w & 1u, on[1] = w & 2u, on[2] = w & 4u, on[3] = w & 8u;
            } else {
                on[0] = mk[j].x > 0.f, on[1] = mk[j].y > 0.f, on[2] = mk[j].z > 0.f, on[3] = mk[j].w > 0.f;
            }
            const float4 y = make_float4(on[0] ? d.x * uo : 0.f, on[1] ? d.y * uo : 0.f, on[2] ? d.z * uo : 0.f,
                                         on[3] ? d.w * uo : 0.f);
            const long long n = n0 + s;
            const float ym = fmaxf(fmaxf(fabsf(y.x), fabsf(y.y)), fmaxf(fabsf(y.z), fabsf(y.w)));
            om = (in && n < a.batch) ? fmaxf(om, ym) : om;  // the dummy slot's sums are not output
            const int iy = 2 * (pix / 10) + py, ix = 2 * (pix % 10) + px;
            float4* dst = (in && n < a.batch)
                              ? reinterpret_cast<float4*>(a.y + ((n * L::IH + iy) * L::IW + ix) * L::CIN + c4 * 4)
                              : kC2Dummy + tid;
            *dst = y;
        }
    };

    long long t = blockIdx.x;
    // prologue: the first triple's rows, taps 0..3, class 0's mask operands, a zero image
    dmaA(t);
    dmaB2(0);
    dmaB2(2);
    load_mask(t * C2S, 0);
    for (int e = tid; e < C2S * C2PIX * 8; e += 512) reinterpret_cast<float4*>(Ds)[e] = make_float4(0.f, 0.f, 0.f, 0.f);
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));  // the builtin, so hipcc's own wait bookkeeping sees it
    lds_barrier();
    take_A();
    lds_barrier();  // An free for the next triple's rows

    // one class-tap step (i = k & 3 at compile time): tap k+1's MFMAs beside tap k's col2im
    // adds.  vmcnt bookkeeping per wave (every count static: stores unconditional, loads
    // clamped): i = 1, 3 DMA the tap pair k+3, k+4; i = 3 then stores the class, loads the
    // next class's mask operands and (class 0) DMAs the next triple's rows; i = 0 waits for
    // the pair of the step before (behind it: 5 stores + 5 mask loads (+ 8 row DMAs after
    // class 0) = vmcnt(10) / vmcnt(18)); i = 2 drains everything (vmcnt(0)).
    auto step = [&](long long tt, int cls, auto i_tag, f32x16& next, const f32x16& cur) {
        constexpr int i = decltype(i_tag)::value;
        const int k = 4 * cls + i;
        const long long n0 = tt * C2S;
        if constexpr (i & 1) dmaB2(k + 3);  // taps k+3, k+4 (mod 16) into the slots of k-1, k
        if (i < 3 || cls < 3) mfma_tap(k + 1, next);
        rmw_tap(i_tag, cur);
        if constexpr (i == 0) {
            if (SAFE)
                __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
            else if (cls == 1)
                __builtin_amdgcn_s_waitcnt(waitcnt_vm(C2_WAIT_I0_ROWS));  // + class 0's row DMAs
            else
                __builtin_amdgcn_s_waitcnt(waitcnt_vm(C2_WAIT_I0));
        }
        if constexpr (i == 2) __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
        lds_barrier();
        if constexpr (i == 3) {
            output(n0, cls);
            // one load path (two paths would merge into register copies that wait vmcnt(0))
            load_mask(cls < 3 ? n0 : (tt + gridDim.x) * C2S, (cls + 1) & 3);
            if (cls == 0) dmaA(tt + gridDim.x);  // the next triple's rows (clamped past the end)
            lds_barrier();
        }
    };
    f32x16 acc0, acc1;
#pragma unroll 1
    for (; t < ntriples; t += gridDim.x) {
        mfma_tap(0, acc0);
#pragma unroll 1
        for (int cls = 0; cls < 4; ++cls) {
            step(t, cls, std::integral_constant<int, 0>{}, acc1, acc0);
            step(t, cls, std::integral_constant<int, 1>{}, acc0, acc1);
            step(t, cls, std::integral_constant<int, 2>{}, acc1, acc0);
            step(t, cls, std::integral_constant<int, 3>{}, acc0, acc1);
        }
        take_A();  // the next triple's rows (drained at class 1's i = 2, ordered by the barriers since)
        lds_barrier();
    }
    amax_record(a.amax_y, om);
}


// ---------------------------------------------------------------------------
// Split-f16 GEMM, LDS-DMA pipelined ("sg2"): the forward-style GEMMs (conv2/conv3
// forward, conv3 dgrad, fc forward, fc dgrad) with the Problems' fused epilogues (bias +
// ReLU, ReLU-mask, NHWC / Flatten order).  512-thread workgroups (8 waves, two per SIMD, one workgroup per
// CU), 256 rows x 64 columns per workgroup, each wave 32 rows x 64 columns (hi/lo f32
// accumulators for two 32x32 tiles: three v_mfma_f32_32x32x16_f16 per tile and 16-k step).
// Per 32-k chunk the A rows (f32, im2col-gathered: one 128-B run per row) and the
// pre-split B chunk (12 KB, split_frag_index order) are copied global -> LDS by
// global_load_lds_dwordx4 into a three-slot ring, so no VGPR staging and no ds_write:
//   * each wave DMAs exactly its own 32 A rows (4 x 1 KB), so A needs no cross-wave
//     ordering, only the wave's own counted vmcnt;
//   * B is shared: waves 0-3 DMA two 1 KB pieces, waves 4-7 one;
//   * K loop: wait for this wave's DMAs of chunk c (vmcnt = the DMAs of chunk c+1 still
//     allowed in flight), one raw s_barrier (everyone's B of chunk c has landed; everyone
//     has finished reading chunk c-1), DMA chunk c+2 into the slot chunk c-1 used, then
//     split A in registers and run the 24 MFMAs of chunk c.  No ordinary global load is in
//     flight in the loop (hipcc would wait vmcnt(0) on it): the epilogue operands are
//     loaded after it.
// A rows are 128 B in LDS with their 16-B pieces XOR-swizzled by (row >> 1) & 7, which
// makes every ds_read_b128 of the fragments conflict-free (rows 0-3 / 12-15 / 20-27 of a
// lane group land on distinct bank quads); the DMA writes LDS lane-linearly, so the
// swizzle is applied to each lane's GLOBAL source address.
// ---------------------------------------------------------------------------
constexpr int SG_BQ = 2 * 2 * NPL * 64;  // u32x4 per B chunk at 64 columns (8 KB)
constexpr int SG_BP = SG_BQ / 64;        // its 1 KB DMA pieces

// LDS fragment reads in inline asm: hipcc's wait insertion cannot tell a ds_read from the
// ring slot being read apart from the DMAs in flight into the other slots, and puts a
// vmcnt(0) before the first read of every chunk (which would drain the prefetch).  Issued
// here, the reads are ordered by the kernel's own counted vmcnt + barrier, and their data
// by an lgkmcnt wait that takes the destination registers as operands (so no use of them
// can be scheduled above it).
__device__ inline u32x4 sg_ds_read(uint32_t addr) {
    u32x4 r;
    asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(addr));
    return r;
}
template <int N>
__device__ inline void sg_lgkm_wait(u32x4 (&v)[6]) {
    asm volatile("s_waitcnt lgkmcnt(%6)"
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5])
                 : "n"(N));
}
template <int N>
__device__ inline void sg_lgkm_wait(u32x4 (&v)[10]) {
    asm volatile("s_waitcnt lgkmcnt(%10)"
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]),
                   "+v"(v[8]), "+v"(v[9])
                 : "n"(N));
}
template <int N>
__device__ inline void sg_vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// WAVES waves x 32 rows per workgroup, SLOTS ring slots of one 32-k chunk (A: 128 B per row;
// B: 8 KB per 64 columns).  8 waves / 3 slots: one workgroup per CU, waves 4-7 staggered; 4 waves / 2 slots:
// two workgroups per CU (48 KB each), whose K walks, prologues and epilogues interleave on
// every SIMD.  A is split in registers with its tensor's scale (a.amax_x), B was packed with
// its own (a.wexp); the epilogue unscales, and records the output's amax (a.amax_y).
// Prob::NOUT = 128 (round 4, the fc layer and the heads' hidden layer: "wide" tiles): each wave
// runs 32 rows x 128 columns, the A fragments of a k-step feeding four column tiles, so A is
// staged once per 128 output columns instead of once per 64; B is two consecutive 64-column
// packed blocks (Prob::bchunk_blk), 16 KB per chunk.
template <class Prob, int WAVES, int SLOTS>
__global__ void __launch_bounds__(64 * WAVES, 8 / WAVES) sgemm_kernel(Args a, const u32x4* __restrict__ wq) {
    constexpr int NT = Prob::NOUT / 32, NBLK = NT / 2;  // column tiles; 64-column packed B blocks
    constexpr int ROWS = 32 * WAVES, AB = ROWS * BK * 4, SLOT = AB + NBLK * SG_BQ * 16;
    constexpr int BP = NBLK * SG_BP;                 // B pieces of a chunk (1 KB each)
    constexpr int BPW = (BP + WAVES - 1) / WAVES;    // B pieces DMA'd per wave
    constexpr int NDMA = 4 + BPW;                  // this wave's DMAs per chunk
    constexpr int NF = 2 + NT * NPL;                 // fragment reads per k-step
    constexpr bool STAGGER = WAVES == 8;
    static_assert((Prob::NOUT == 64 || (Prob::NOUT == 128 && !STAGGER)) && Prob::ROWS == ROWS,
                  "sg2: 32 rows per wave x 64 or 128 columns");
    static_assert(NF <= 15, "lgkmcnt is 4 bits");
    static_assert(SLOTS == 2 || SLOTS == 3, "sg2: two or three ring slots");
    // all LDS in ONE __shared__ object (a second one can make hipcc wait vmcnt(0) in the loop)
    __shared__ __attribute__((aligned(16))) uint8_t lds[SLOTS * SLOT];
    typename Prob::Tile t;
    if (!Prob::tile(a, t)) return;
    const int nchunk = Prob::nchunk(t);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: DMA bases go to M0

    // DMA sources: A instruction j of this wave covers its rows 8j + (lane >> 3), LDS piece
    // lane & 7, which holds global piece (lane & 7) ^ swz(row)
    const uint8_t* asrc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int r = 8 * j + (lane >> 3);
        asrc[j] = reinterpret_cast<const uint8_t*>(Prob::row_ptr(a, t, wave * 32 + r)) +
                  ((((lane & 7) ^ ((r >> 1) & 7))) << 4);
    }
    // B: BP pieces of 1 KB per chunk, BPW per wave (pieces past the last re-copy it: the
    // same bytes to the same place), so every wave issues NDMA DMAs per chunk; piece pc is piece
    // pc % SG_BP of the chunk of 64-column block pc / SG_BP
    int bp[BPW];
#pragma unroll
    for (int i = 0; i < BPW; ++i) bp[i] = min(BPW * wave + i, BP - 1);
    // operand scales: A by its tensor's amax (H1P planes: their exponent), B as packed; the epilogue
    // multiplies by both inverses
    const int ex = Prob::A_PLANES ? *a.xexp : split_scale_exp(amax_read(a.amax_x)), ew = *a.wexp;
    const float sa = exp2i(ex), ua = exp2i(-ex), uw = exp2i(-ew);
    // PX output: its exponent from the bound amax(x) * max column norm + max |bias| (every workgroup
    // derives the same; workgroup 0 publishes it).  A non-finite bound makes the output NaN (loud).
    float sy = 1.f;
    if constexpr (Prob::PLANES_OUT) {
        const uint32_t am = amax_read(a.amax_x), nm = amax_read(a.ynorm), bm = *a.ybias;
        const int ey = bound_exp(am, nm, bm);
        const float bnd = __uint_as_float(am) * __uint_as_float(nm) + __uint_as_float(bm);
        sy = __builtin_isfinite(bnd) ? exp2i(ey) : __builtin_nanf("");
        if (blockIdx.x == 0 && threadIdx.x == 0) *a.yexp_out = ey;
    }
    // chunk c into ring slot S; the chunk index is clamped, not branched on (past the end:
    // the last chunk again, never read)
    auto issue = [&](int c, auto S) {
        constexpr int slot = decltype(S)::value;
        c = c < nchunk ? c : nchunk - 1;
        uint8_t* base = lds + slot * SLOT;
        const long long off = (long long)Prob::chunk_off(t, c) * 4;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(asrc[j] + off),
                (__attribute__((address_space(3))) void*)(base + (wave * 32 + 8 * j) * 128), 16, 0, 0);
        if constexpr (NBLK == 1) {
            const u32x4* bsrc = wq + (long long)Prob::bchunk_id(t, c) * SG_BQ + lane;
#pragma unroll
            for (int i = 0; i < BPW; ++i)
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(bsrc + bp[i] * 64),
                                                 (__attribute__((address_space(3))) void*)(base + AB + bp[i] * 1024),
                                                 16, 0, 0);
        } else {
#pragma unroll
            for (int i = 0; i < BPW; ++i) {
                const u32x4* bsrc = wq + (long long)Prob::bchunk_blk(t, c, bp[i] / SG_BP) * SG_BQ + lane;
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(bsrc + (bp[i] % SG_BP) * 64),
                    (__attribute__((address_space(3))) void*)(base + AB + bp[i] * 1024), 16, 0, 0);
            }
        }
    };

    f32x16 hi[NT], lo[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) hi[j] = lo[j] = zero16();
    const int r = lane & 31, h = lane >> 5, sw = (r >> 1) & 7;
    const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)lds);
    const uint32_t a_lane = lds0 + (wave * 32 + r) * 128, b_lane = lds0 + AB + lane * 16;
    // Stagger (8 waves: the two waves of a SIMD out of phase): waves 4-7 defer each chunk's
    // second k-step MFMAs past the next barrier, so right after a barrier one wave of every
    // SIMD runs matrix work (the deferred k-step) while its partner reads and splits (VALU).
    // The deferred k-step's operands (split A planes + B fragments) stay in registers.
    const bool late = STAGGER && wave >= 4;
    u32x4 daf[NPL], dbf[NT * NPL];
    auto mfma3 = [&](const u32x4 (&af)[NPL], const u32x4* bf) {
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const u32x4 b2[NPL] = {bf[NPL * j], bf[NPL * j + 1]};
            mfma_split3(af, b2, hi[j], lo[j]);
        }
    };
    auto split_a = [&](const u32x4 (&g)[NF], u32x4 (&af)[NPL]) {
        if constexpr (Prob::A_PLANES) {  // H1P: the two pieces read are the planes
            af[0] = g[0];
            af[1] = g[1];
        } else {
            split8h(__builtin_bit_cast(float4, g[0]), __builtin_bit_cast(float4, g[1]), sa, af[0], af[1]);
        }
    };
    // chunk in slot S: 2 NF fragment reads up front (k-step 0's NF, then k-step 1's), k-step 0
    // computed once its NF have landed (lgkmcnt(NF)) while k-step 1's are in flight
    auto compute = [&](auto S) {
        constexpr int slot = decltype(S)::value;
        u32x4 f[2][NF];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            // the lane's 8 k of k-step s: f32 pieces g0, g0 + 1 (16 B = 4 values each), or H1P
            // pieces 2s + h (hi plane: 8 f16) and 4 + 2s + h (lo plane)
            const int g0 = Prob::A_PLANES ? 2 * s + h : 4 * s + 2 * h, g1 = Prob::A_PLANES ? 4 + g0 : g0 + 1;
            f[s][0] = sg_ds_read(a_lane + slot * SLOT + ((g0 ^ sw) << 4));
            f[s][1] = sg_ds_read(a_lane + slot * SLOT + ((g1 ^ sw) << 4));
#pragma unroll
            for (int j = 0; j < NT; ++j)
#pragma unroll
                for (int p = 0; p < NPL; ++p)
                    // column tile j: tile j & 1 of 64-column block j >> 1 (split_frag_index: [s][j][p][lane])
                    f[s][2 + NPL * j + p] = sg_ds_read(b_lane + slot * SLOT + (j >> 1) * (SG_BQ * 16) +
                                                       (((s * 2 + (j & 1)) * NPL + p) * 64) * 16);
        }
        u32x4 af[NPL];
        sg_lgkm_wait<NF>(f[0]);
        split_a(f[0], af);
        mfma3(af, f[0] + 2);
        sg_lgkm_wait<0>(f[1]);
        if (late) {  // k-step 1 split now, multiplied after the next barrier
            split_a(f[1], daf);
#pragma unroll
            for (int i = 0; i < NT * NPL; ++i) dbf[i] = f[1][2 + i];
        } else {
            split_a(f[1], af);
            mfma3(af, f[1] + 2);
        }
    };
    // one pipeline step: this wave's DMAs of chunk c waited for (those of the next SLOTS - 2
    // chunks may stay in flight: the clamped re-issues past the end count too, so the count is
    // the same in every step), one barrier (every wave's DMAs of chunk c landed, every wave done
    // with chunk c - 1), chunk c + SLOTS - 1 issued into the slot chunk c - 1 used, chunk c computed
    auto step = [&](int c, auto S, auto S2) {
        sg_vm_wait<NDMA * (SLOTS - 2)>();
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        issue(c + SLOTS - 1, S2);
        if (late && c > 0) mfma3(daf, dbf);  // chunk c - 1's deferred k-step
        compute(S);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    issue(0, I0{});
    if constexpr (SLOTS == 3) {
        issue(1, I1{});
#pragma unroll 1
        for (int c = 0; c < nchunk; c += 3) {
            step(c, I0{}, I2{});
            if (c + 1 < nchunk) step(c + 1, I1{}, I0{});
            if (c + 2 < nchunk) step(c + 2, I2{}, I1{});
        }
    } else {
#pragma unroll 1
        for (int c = 0; c < nchunk; c += 2) {
            step(c, I0{}, I1{});
            if (c + 1 < nchunk) step(c + 1, I1{}, I0{});
        }
    }
    if (late && nchunk > 0) mfma3(daf, dbf);
    sg_vm_wait<0>();  // the clamped tail DMAs, before the LDS is released
    // epilogue, per column tile: its operand loads first (all issued before its first store);
    // om = the largest |value| this lane stored.  BITS_OUT: the ReLU bitmask word of tile row L and
    // column tile j is half (L >> 2) & 1 of the ballot of element q = (L & 3) + 4 (L >> 3) — lane L
    // (< 32) collects both words of its row and stores them together
    float om = 0.f;
    uint32_t bw[NT];
    const int qL = (lane & 3) + 4 * ((lane >> 3) & 3), hL = (lane >> 2) & 1;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        bw[j] = 0u;
        decltype(Prob::prefetch(a, t, 0, 0)) e[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) e[q] = Prob::prefetch(a, t, wave * 32 + (q & 3) + 8 * (q >> 2) + 4 * h, j * 32 + r);
        // one wait for all of them (a real s_waitcnt the compiler tracks): the row-bounded
        // stores below are branches, and a load pending at a branch makes hipcc wait vmcnt(0)
        // inside every one of them — behind every earlier store
        __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int row = wave * 32 + (q & 3) + 8 * (q >> 2) + 4 * h, col = j * 32 + r;
            float v;
            if constexpr (Prob::PLANES_OUT) {
                // every lane runs the pair swap; the pair (col & ~1, col | 1) shares its row, so both
                // lanes store or neither does
                v = Prob::value(a, t, row, col, (hi[j][q] + lo[j][q]) * ua * uw, e[q]);
                const uint32_t w = px_pair_word(v, sy, lane & 1);
                const long long el = Prob::out_elem(a, t, row, col & ~1);
                if (el >= 0) *reinterpret_cast<uint32_t*>(reinterpret_cast<uint16_t*>(a.y) + px_index(el) + 32 * (lane & 1)) = w;
            } else {
                v = Prob::store_pre(a, t, row, col, (hi[j][q] + lo[j][q]) * ua * uw, e[q]);
            }
            om = fmaxf(om, fabsf(v));
            if constexpr (Prob::BITS_OUT) {
                if (a.bits_y) {  // uniform
                    const unsigned long long b = __ballot(v > 0.f);
                    bw[j] = qL == q ? (uint32_t)(hL ? b >> 32 : b) : bw[j];
                }
            }
        }
    }
    if constexpr (Prob::BITS_OUT) {
        static_assert(NT == 2, "bitmask: 64 channels = two words per pixel");
        const long long m = t.m0 + wave * 32 + lane;
        if (a.bits_y && lane < 32 && m < t.M) *reinterpret_cast<uint2*>(a.bits_y + m * 2) = make_uint2(bw[0], bw[1]);
    }
    amax_record(a.amax_y, om);
}

constexpr int SG_WAVES = 4;  // 4: two 128-row workgroups per CU (2 ring slots); 8: one 256-row workgroup (3 slots)
// ring slots (chunks in flight + 1) per Problem (Prob::SLOTS): 3 for the plain fc / head GEMMs
// (their DMA latency was exposed with one chunk of lookahead: fc forward 0.190 -> 0.174 ms,
// dgrad 0.255 -> 0.238), 2 for the conv forms (3 measured slower for the conv3 dgrad, 0.31 ->
// 0.34 ms); 3 x 24 KB per workgroup keeps two workgroups per CU.
constexpr int SG_ROWS = 32 * SG_WAVES;
constexpr int SG_FWD2_PARITY = 1;  // conv2 forward taps in input-parity classes (SgFwd)

template <class Prob>
int launch_sgemm(const Args& a, const uint16_t* wq, long long blocks, hipStream_t s, const char* name) {
    if (blocks == 0) return PPOX_OK;
    constexpr int slots = SG_WAVES == 8 ? 3 : Prob::SLOTS;
    sgemm_kernel<Prob, SG_WAVES, slots><<<(unsigned)blocks, 64 * SG_WAVES, 0, s>>>(
        a, reinterpret_cast<const u32x4*>(wq));
    PPOX_LAUNCHED(name);
}

// sg2 Problems: the f32 Problems' chunk walk and epilogues on SG_ROWS-row tiles, plus
// each row's A base pointer (rows past the end clamped to a valid row, never stored) and
// the chunk's element offset within a row (the same for every row of the tile)
template <class L, bool OUT_NCHW>
struct SgFwd : FwdNHWCProblem<L, OUT_NCHW, 1> {
    static constexpr int ROWS = SG_ROWS, CPT = L::CIN / BK;
    static constexpr bool BITS_OUT = true;  // a.bits_y: the output's ReLU bitmask (2 words per pixel)
    static constexpr int SLOTS = 2;
    __device__ static bool tile(const Args& a, RowTile& t) {
        t.m0 = xcd_remap(blockIdx.x, gridDim.x) * ROWS;
        t.M = a.batch * L::P;
        return true;
    }
    __device__ static const float* row_ptr(const Args& a, const RowTile& t, int row) {
        long long m = t.m0 + row;
        m = m < t.M ? m : t.M - 1;
        const long long n = m / L::P;
        const int p = (int)(m - n * L::P), oy = p / L::OW, ox = p % L::OW;
        return reinterpret_cast<const float*>(a.x) + ((n * L::IH + oy * L::S) * L::IW + ox * L::S) * L::CIN;
    }
    // conv2 (4x4 taps, stride 2, one chunk per tap): the taps walked in input-parity classes —
    // (ky, kx), (ky, kx + 2), (ky + 2, kx), (ky + 2, kx + 2) read the same input pixels (one output
    // column / row apart), so a class taken consecutively keeps a quarter of the tile's input
    // live in L2 instead of all of it for half the K walk
    static constexpr bool PARITY = SG_FWD2_PARITY && L::S == 2 && L::KH == 4 && L::KW == 4 && CPT == 1;
    __device__ static int tap_of(int c) {
        if constexpr (PARITY) {
            const int cls = c >> 2, i = c & 3;
            return ((cls >> 1) + 2 * (i >> 1)) * 4 + (cls & 1) + 2 * (i & 1);
        } else {
            return c / CPT;
        }
    }
    __device__ static int chunk_off(const RowTile&, int c) {
        const int tap = tap_of(c);
        return ((tap / L::KW) * L::IW + tap % L::KW) * L::CIN + (c % CPT) * BK;
    }
    __device__ static int bchunk_id(const RowTile&, int c) { return PARITY ? tap_of(c) : c; }
};

// the conv2 forward on H1P input (conv1's output as f16 planes): a pixel's 128 B are its 32 hi then
// 32 lo f16 instead of 32 f32, so the DMA addressing is unchanged and the k-step's two pieces are
// the fragments' planes (no split in registers)
struct SgFwd2P : SgFwd<G2, false> {
    static constexpr bool A_PLANES = true;
};

// BITS_IN: the ReLU mask of the layer below from its forward's bitmask (a.bits_mask, CIN / 32
// words per pixel) instead of its f32 activations
template <class L, bool BITS_IN = false>
struct SgDgradPM : DgradPMProblem<L, 1> {
    using Base = DgradPMProblem<L, 1>;
    static constexpr int ROWS = SG_ROWS, NPOS = Base::NPOS, CPT = Base::CPT;
    static constexpr bool BITS_OUT = false;
    static constexpr int SLOTS = 2;
    __device__ static float prefetch(const Args& a, const PixelTile& t, int row, int ci) {
        if constexpr (!BITS_IN) {
            return Base::prefetch(a, t, row, ci);
        } else {
            long long n = t.n0 + row;
            n = n < a.batch ? n : t.n0;
            const uint32_t w = a.bits_mask[(n * NPOS + t.pos) * (L::CIN / 32) + (ci >> 5)];
            return (float)((w >> (ci & 31)) & 1u);
        }
    }
    __device__ static bool tile(const Args& a, PixelTile& t) {
        const long long w = xcd_remap(blockIdx.x, gridDim.x);
        t.n0 = (w / NPOS) * ROWS;
        t.pos = (int)(w % NPOS);
        t.iy = t.pos / L::IW;
        t.ix = t.pos % L::IW;
        int ny, nx;
        tap_range<L::S, L::OH, L::KH>(t.iy, t.ky0, ny);
        tap_range<L::S, L::OW, L::KW>(t.ix, t.kx0, nx);
        t.nx = nx;
        t.nchunk = ny * nx * CPT;
        return true;
    }
    __device__ static const float* row_ptr(const Args& a, const PixelTile& t, int row) {
        long long n = t.n0 + row;
        n = n < a.batch ? n : a.batch - 1;
        return reinterpret_cast<const float*>(a.x) + n * (L::P * L::COUT);
    }
    __device__ static int chunk_off(const PixelTile& t, int c) {
        const int tap = c / CPT, ty = tap / t.nx, tx = tap - ty * t.nx;
        const int oy = (t.iy - t.ky0) / L::S - ty, ox = (t.ix - t.kx0) / L::S - tx;
        return (oy * L::OW + ox) * L::COUT + (c % CPT) * BK;
    }
};

// Tile order: column-block groups of G outermost, then row tiles, then the G column blocks of
// the group — so the workgroups an XCD runs together share one A row tile, and one group's B
// (G x 196 KB / 1.2 MB for the dgrad / forward) stays in that XCD's L2 while its row tiles
// stream past (A is read NCB / G times, B about once per XCD).
// BITS_IN (FC_DGRAD): h3's ReLU mask from the conv3 forward's bitmask (N / 32 words per row)
template <int K, int N, int MODE, int G, bool BITS_IN = false, int NB = 64>
struct SgRows : GemmRowsProblem<K, N, NB, MODE> {
    using Base = GemmRowsProblem<K, N, NB, MODE>;
    static constexpr int ROWS = SG_ROWS, NCB = Base::NCB;
    static constexpr bool BITS_OUT = false;
    static constexpr int SLOTS = 3;
    __device__ static auto prefetch(const Args& a, const GemmTile& t, int row, int col) {
        if constexpr (!BITS_IN) {
            return Base::prefetch(a, t, row, col);
        } else {
            static_assert(MODE == FC_DGRAD && N % 32 == 0, "bitmask: the fc dgrad's h3 mask");
            const int n = t.cb * NB + col, nc = n < N ? n : N - 1;
            long long m = t.m0 + row;
            m = m < t.M ? m : t.m0;
            const uint32_t w = a.bits_mask[m * (N / 32) + (nc >> 5)];
            return (float)((w >> (nc & 31)) & 1u);
        }
    }
    __device__ static bool tile(const Args& a, GemmTile& t) {
        const long long w = xcd_remap(blockIdx.x, gridDim.x);
        const long long rt = (a.batch + ROWS - 1) / ROWS;      // row tiles
        const long long grp = w / (rt * G), in = w - grp * rt * G;
        const int g0 = (int)grp * G, gn = NCB - g0 < G ? NCB - g0 : G;  // the last group may be narrower
        t.m0 = (in / gn) * ROWS;
        t.cb = g0 + (int)(in % gn);
        t.M = a.batch;
        return true;
    }
    __device__ static const float* row_ptr(const Args& a, const GemmTile& t, int row) {
        long long m = t.m0 + row;
        m = m < t.M ? m : t.M - 1;
        return reinterpret_cast<const float*>(a.x) + m * K;
    }
    __device__ static int chunk_off(const GemmTile&, int c) { return c * BK; }
};

// fc forward split over K for small batches (128-row tiles x 8 column blocks leave most CUs
// idle below ~8192 rows): S K-ranges per (row tile, column block), each workgroup's partial
// product stored to slab[ks][row][512]; fc_fwd_sk_reduce adds the S partials in order, then
// the bias, then the ReLU.
template <int K, int N, int S>
struct SgRowsSK : GemmRowsProblem<K, N, 64, FC_FWD> {
    using Base = GemmRowsProblem<K, N, 64, FC_FWD>;
    static constexpr int ROWS = SG_ROWS, NCB = Base::NCB, KC = Base::KC;
    static constexpr bool BITS_OUT = false;
    static constexpr int SLOTS = 3;
    struct Tile {
        long long m0, M;
        int cb, ks, c0, nc;
    };
    __device__ static bool tile(const Args& a, Tile& t) {
        const long long w = xcd_remap(blockIdx.x, gridDim.x);  // a row tile's S x 8 workgroups share an XCD
        t.cb = (int)(w % NCB);
        const long long r = w / NCB;
        t.ks = (int)(r % S);
        t.m0 = (r / S) * ROWS;
        t.M = a.batch;
        t.c0 = t.ks * KC / S;
        t.nc = (t.ks + 1) * KC / S - t.c0;
        return true;
    }
    __device__ static int nchunk(const Tile& t) { return t.nc; }
    __device__ static int bchunk_id(const Tile& t, int c) { return t.cb * KC + t.c0 + c; }
    __device__ static const float* row_ptr(const Args& a, const Tile& t, int row) {
        long long m = t.m0 + row;
        m = m < t.M ? m : t.M - 1;
        return reinterpret_cast<const float*>(a.x) + m * K;
    }
    __device__ static int chunk_off(const Tile& t, int c) { return (t.c0 + c) * BK; }
    __device__ static float prefetch(const Args&, const Tile&, int, int) { return 0.f; }
    __device__ static float store_pre(const Args& a, const Tile& t, int row, int col, float acc, float) {
        const long long m = t.m0 + row;
        if (m >= t.M) return 0.f;
        a.y[((long long)t.ks * t.M + m) * N + t.cb * 64 + col] = acc;
        return acc;
    }
};

// am (nullable): f's amax slots (the heads' split hidden layer reads f)
template <int N, int S>
__global__ void __launch_bounds__(256) fc_fwd_sk_reduce(const float4* __restrict__ slab, long long M,
                                                         const float* __restrict__ bias, float4* __restrict__ y,
                                                         uint32_t* __restrict__ am) {
    const long long i = blockIdx.x * 256LL + threadIdx.x, n4 = M * N / 4;
    float m = 0.f;
    if (i < n4) {
        float4 s = slab[i];
#pragma unroll
        for (int k = 1; k < S; ++k) {
            const float4 v = slab[k * n4 + i];
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
        const int n = (int)((i * 4) % N);
        const float4 o = make_float4(fmaxf(s.x + bias[n], 0.f), fmaxf(s.y + bias[n + 1], 0.f),
                                     fmaxf(s.z + bias[n + 2], 0.f), fmaxf(s.w + bias[n + 3], 0.f));
        y[i] = o;
        m = fmaxf(fmaxf(o.x, o.y), fmaxf(o.z, o.w));
    }
    amax_record(am, m);
}

// the same reduce with the actor head fused (ppox_skinny_linear's arithmetic on the finished row,
// bitwise the same logits): one wave per row, lane l owns columns 4l .. 4l + 3 and 256 + 4l .. of
// the 512 (the skinny kernel's k order), the NO dot products wave-reduced in its butterfly order
template <int S, int NO>
__global__ void __launch_bounds__(256) fc_fwd_sk_reduce_actor(const float4* __restrict__ slab, long long M,
                                                               const float* __restrict__ bias, float4* __restrict__ y,
                                                               uint32_t* __restrict__ am, const float* __restrict__ wa,
                                                               const float* __restrict__ ba, float* __restrict__ logits) {
    const int lane = threadIdx.x & 63;
    const long long b = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    float m = 0.f;
    if (b < M) {  // wave-uniform
        const long long n4 = M * 128;
        float acc[NO];
#pragma unroll
        for (int o = 0; o < NO; ++o) acc[o] = 0.f;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            const int c4 = lane + 64 * half;
            const long long i = b * 128 + c4;
            float4 s = slab[i];
#pragma unroll
            for (int k = 1; k < S; ++k) {
                const float4 v = slab[k * n4 + i];
                s.x += v.x;
                s.y += v.y;
                s.z += v.z;
                s.w += v.w;
            }
            const int n = 4 * c4;
            const float4 o = make_float4(fmaxf(s.x + bias[n], 0.f), fmaxf(s.y + bias[n + 1], 0.f),
                                         fmaxf(s.z + bias[n + 2], 0.f), fmaxf(s.w + bias[n + 3], 0.f));
            y[i] = o;
            m = fmaxf(m, fmaxf(fmaxf(o.x, o.y), fmaxf(o.z, o.w)));
#pragma unroll
            for (int a = 0; a < NO; ++a) {
                const float4 wv = reinterpret_cast<const float4*>(wa)[a * 128 + c4];
                acc[a] = fmaf(o.x, wv.x, acc[a]);
                acc[a] = fmaf(o.y, wv.y, acc[a]);
                acc[a] = fmaf(o.z, wv.z, acc[a]);
                acc[a] = fmaf(o.w, wv.w, acc[a]);
            }
        }
#pragma unroll
        for (int a = 0; a < NO; ++a)
#pragma unroll
            for (int k = 32; k > 0; k >>= 1) acc[a] += __shfl_xor(acc[a], k, 64);
        if (lane < NO) {
            float r = acc[0];
#pragma unroll
            for (int a = 1; a < NO; ++a) r = lane == a ? acc[a] : r;
            logits[b * NO + lane] = r + ba[lane];
        }
    }
    amax_record(am, m);
}

// K-splits for a batch: enough (row tile, column block, split) workgroups for two per CU, at most 8
// (the heads' 512-deep hidden layer: splits up to 256 workgroups — 2 at 2,048 rows: 9.5 + 5.9 µs for the
// GEMM + reduce vs 10.9 + 6.2 with the fc layer's 512, whose K = 3136 gains from the fourth split)
inline int fc_fwd_splits(long long batch, long long wgs = 512) {
    const long long wg = ppox::ceil_div(batch, SG_ROWS) * FcFwd::NCB;
    int s = 1;
    while (s < 8 && wg * s < wgs) s *= 2;
    return s;
}

struct ActorHead {
    const float *w, *b;
    int n;          // actions (1..8); 0: no actor head fused
    float* logits;  // rows x n
};

// K = 3136: the fc layer (reduce: + bias, ReLU, f's amax, the actor head); K = 512: the heads' hidden
// layer (the same reduce with the critic head Linear(512, 1) fused, no amax)
template <int S>
int launch_fc_sk_reduce(const Args& a, float* slab, const float* bias, float* f, const ActorHead& act, hipStream_t st,
                        const char* name);
template <int K, int S, bool AP = false>
int launch_fc_fwd_sk(const Args& a, const uint16_t* q, float* slab, const float* bias, float* f, const ActorHead& act,
                     hipStream_t st, const char* name = "ppox_nature_fc_fwd_splitk") {
    Args b = a;
    b.y = slab;
    b.amax_y = nullptr;  // partial products: f's amax is recorded by the reduce
    const int rc = launch_sgemm<Px<SgRowsSK<K, 512, S>, AP>>(b, q, ppox::ceil_div(a.batch, SG_ROWS) * FcFwd::NCB * S,
                                                             st, name);
    if (rc != PPOX_OK) return rc;
    return launch_fc_sk_reduce<S>(a, slab, bias, f, act, st, name);
}
// the S partial products in order + bias, ReLU, f's amax (a.amax_y), the fused head
template <int S>
int launch_fc_sk_reduce(const Args& a, float* slab, const float* bias, float* f, const ActorHead& act, hipStream_t st,
                        const char* name) {
    const float4* sl = reinterpret_cast<const float4*>(slab);
    float4* f4 = reinterpret_cast<float4*>(f);
    const unsigned rows4 = (unsigned)ppox::ceil_div(a.batch, 4LL);
    switch (act.n) {
#define PPOX_FSA(N)                                                                                              \
    case N:                                                                                                      \
        fc_fwd_sk_reduce_actor<S, N><<<rows4, 256, 0, st>>>(sl, a.batch, bias, f4, a.amax_y, act.w, act.b, act.logits); \
        break;
        PPOX_FSA(1) PPOX_FSA(2) PPOX_FSA(3) PPOX_FSA(4) PPOX_FSA(5) PPOX_FSA(6) PPOX_FSA(7) PPOX_FSA(8)
#undef PPOX_FSA
        default:
            fc_fwd_sk_reduce<512, S><<<ppox::ceil_div(a.batch * 512 / 4, 256), 256, 0, st>>>(sl, a.batch, bias, f4,
                                                                                             a.amax_y);
    }
    PPOX_LAUNCHED(name);
}

// ---------------------------------------------------------------------------
// Register-direct implicit GEMM (the default forward / dgrad path).
// Each wave owns 32*MT rows x all NOUT columns and is independent: no LDS, no
// barriers.  Within a 32-wide K chunk the MFMA k-slice of step kk is
// {kk, 16 + kk}: lane half h = lane >> 5 supplies k = 16h + kk, so every lane
// reads its row's 16 contiguous K values (4 x 16 B) straight into VGPRs.  B is
// packed so that load q of column tile j is one contiguous 1 KB run across the
// wave (lane L takes floats 4L..4L+3: k = 16h + 4q..4q+3 of column l32) —
// fully coalesced (rg_index).  Chunk c+1 is loaded while chunk c runs on the
// matrix cores.  Used for conv1 forward (u8 input); the f32 layers keep the
// LDS-staged igemm: their 32-row x 32-B fragment loads cost more TA cycles than
// the LDS round trip (measured: profiles/README.md).
// Rows past the end load a clamped (valid) address; their C rows are never
// stored, and a GEMM row only ever reaches its own C row.
// ---------------------------------------------------------------------------
using f32x4 = __attribute__((ext_vector_type(4))) float;

// packed-B position of natural element (k, col) of a [K][NOUT] matrix
__host__ __device__ constexpr int rg_index(int k, int col, int nout) {
    return (k >> 5) * 32 * nout + (col >> 5) * 1024 + ((k & 15) >> 2) * 256 + (((k >> 4) & 1) * 32 + (col & 31)) * 4 +
           (k & 3);
}

// conv1: u8 NCHW frames; chunk c = channel c/2, kernel rows 4(c&1)..+3; lane
// half h takes kernel rows 4(c&1)+2h, +1: two 8-byte runs = four words
template <int MT_>
struct RgFwd1 {
    using L = G1;
    static constexpr int NOUT = L::COUT, MT = MT_, ROWS = 128 * MT;
    using Raw = uint32_t[MT][4];
    struct Tile {
        unsigned m0, M;  // this wave's first row, total rows (< 2^31, host-checked)
    };
    __device__ static bool tile(const Args& a, Tile& t, int wave) {
        const long long w = xcd_remap(blockIdx.x, gridDim.x);
        t.M = (unsigned)(a.batch * L::P);
        t.m0 = (unsigned)(w * ROWS) + wave * 32 * MT;
        return t.m0 < t.M;
    }
    __device__ static int nchunk(const Tile&) { return L::K / BK; }
    __device__ static const float* bchunk(const Args& a, const Tile&, int c) { return a.wp + c * BK * NOUT; }
    struct Loader {
        const uint8_t* base[MT];
        __device__ Loader(const Args& a, const Tile& t, int lane) {
            const uint8_t* x = reinterpret_cast<const uint8_t*>(a.x);
#pragma unroll
            for (int i = 0; i < MT; ++i) {
                unsigned m = t.m0 + i * 32 + (lane & 31);
                m = m < t.M ? m : t.m0;
                const unsigned n = m / L::P, p = m - n * L::P, oy = p / L::OW, ox = p % L::OW;
                base[i] = x + u8_sample_base(a, n, (long long)L::CIN * L::IH * L::IW) +
                          (oy * L::S + (lane >> 5) * 2) * L::IW + ox * L::S;
            }
        }
        __device__ inline void load(int c, Raw& r) const {
            const int off = (c >> 1) * (L::IH * L::IW) + (c & 1) * 4 * L::IW;
#pragma unroll
            for (int i = 0; i < MT; ++i) {
                const uint8_t* p = base[i] + off;
                r[i][0] = *reinterpret_cast<const uint32_t*>(p);
                r[i][1] = *reinterpret_cast<const uint32_t*>(p + 4);
                r[i][2] = *reinterpret_cast<const uint32_t*>(p + L::IW);
                r[i][3] = *reinterpret_cast<const uint32_t*>(p + L::IW + 4);
            }
        }
        __device__ static inline float elem(const Raw& r, int i, int kk) {
            return (float)((r[i][kk >> 2] >> (8 * (kk & 3))) & 0xFFu);
        }
    };
    __device__ static void store(const Args& a, const Tile& t, int row, int co, float acc, bool) {
        const unsigned m = t.m0 + row;
        if (m >= t.M) return;
        a.y[(long long)m * L::COUT + co] = fmaxf(acc + a.bias[co], 0.f);
    }
};

template <class Prob, bool OUT_NCHW = false>
__global__ void __launch_bounds__(256, 2) rgemm_kernel(Args a) {
    constexpr int NOUT = Prob::NOUT, NT = NOUT / 32, MT = Prob::MT;
    using Ld = typename Prob::Loader;
    using Raw = typename Prob::Raw;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    typename Prob::Tile t;
    if (!Prob::tile(a, t, wave)) return;  // wave-uniform; nothing below synchronises
    const int n = Prob::nchunk(t);
    const Ld ld(a, t, lane);

    f32x16 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = zero16();

    Raw a0, a1;
    f32x4 b0[NT][4], b1[NT][4];
    auto loadB = [&](int c, f32x4 (&b)[NT][4]) {
        const f32x4* p = reinterpret_cast<const f32x4*>(Prob::bchunk(a, t, c)) + lane;
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) b[j][q] = p[j * 256 + q * 64];
    };
    auto compute = [&](const Raw& ar, const f32x4 (&b)[NT][4]) {
#pragma unroll
        for (int kk = 0; kk < 16; ++kk)
#pragma unroll
            for (int j = 0; j < NT; ++j)
#pragma unroll
                for (int i = 0; i < MT; ++i)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(Ld::elem(ar, i, kk), b[j][kk >> 2][kk & 3],
                                                                     acc[i][j], 0, 0, 0);
    };
    if (n > 0) {
        ld.load(0, a0);
        loadB(0, b0);
    }
    for (int c = 0; c < n; c += 2) {
        if (c + 1 < n) {
            ld.load(c + 1, a1);
            loadB(c + 1, b1);
        }
        compute(a0, b0);
        if (c + 2 < n) {
            ld.load(c + 2, a0);
            loadB(c + 2, b0);
        }
        if (c + 1 < n) compute(a1, b1);
    }
    // C/D map: col = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                Prob::store(a, t, i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5), j * 32 + (lane & 31),
                            acc[i][j][r], OUT_NCHW);
}

// ---------------------------------------------------------------------------
// Wgrad.  WG = (k-block of KT rows of K) x (all COUT) x (slice of output pixels).
// Per step of MS = 32 pixels: stage X[32][KT] (im2col) and G[32][COUT] in LDS,
// then D(k x co) += X^T G on the MFMA (A operand = X^T: lane i <-> k, kk <-> pixel).
// Each thread's X unit (4 consecutive k) is fixed for the whole kernel, so its
// within-sample offset is computed once; its pixels advance by MS per step with
// 32-bit (sample, pixel) counters (MS <= P, so at most one wrap) — no divisions
// of 64-bit indices in the loop.
// ---------------------------------------------------------------------------

template <class L, bool U8>
struct WgCfg {
    static constexpr int KT = (L::COUT == 32) ? 128 : 64;  // 4 tiles of 32x32 per WG
    static constexpr int KB = L::K / KT;
    // row strides: +4 floats keeps the 16-B stores aligned and conflict-free (a half-wave's
    // 32 lanes write 512 contiguous bytes) and puts the two MFMA k-halves 4 banks apart
    static constexpr int XST = KT + 4, GST = L::COUT + 4;
    static constexpr int UPR = KT / 4;         // 4-element X units per pixel
    static constexpr int XV = MS * UPR / 256;  // X units per thread per step
    static constexpr int XPS = 256 / UPR;      // pixel stride between a thread's X units
    static constexpr int GUPR = L::COUT / 4;
    static constexpr int GV = MS * GUPR / 256;
    static constexpr int GPS = 256 / GUPR;
    static_assert(MS <= L::P, "one wrap per step");
};


template <class L, bool U8>
__global__ void __launch_bounds__(256, 2) wgrad_kernel(WArgs a) {
    using C = WgCfg<L, U8>;
    constexpr int KT = C::KT, KB = C::KB, XST = C::XST, GST = C::GST, COUT = L::COUT;
    constexpr int XV = C::XV, GV = C::GV, UPR = C::UPR, GUPR = C::GUPR;
    __shared__ __attribute__((aligned(16))) float Xs[2][MS * XST];
    __shared__ __attribute__((aligned(16))) float Gs[2][MS * GST];
    // XCD-aware block -> (split, kb): the KB k-blocks of a split share blockIdx % 8
    const int b = blockIdx.x, xcd = b & 7, q = b >> 3;
    const int kb = q % KB, split = (q / KB) * 8 + xcd;
    const unsigned M = (unsigned)(a.batch * L::P);
    const unsigned long long mb64 = (unsigned long long)split * (unsigned long long)a.px_per_split;
    const unsigned mbeg = mb64 < M ? (unsigned)mb64 : M;
    const unsigned mend = (unsigned)min((unsigned long long)M, (unsigned long long)mbeg + a.px_per_split);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int kt = (COUT == 32) ? wave : (wave >> 1), ct = (COUT == 32) ? 0 : (wave & 1);
    f32x16 acc = zero16();

    // ---- fixed per-thread X unit ----
    const int u = threadIdx.x % UPR, px0 = threadIdx.x / UPR;
    const int k = kb * KT + u * 4;
    unsigned koff;
    if constexpr (U8) {
        koff = ((k >> 6) * L::IH + ((k >> 3) & 7)) * L::IW + (k & 7);  // (ci, ky, kx) in a NCHW frame stack
    } else {
        const int tap = k / L::CIN;
        koff = ((tap / L::KW) * L::IW + (tap % L::KW)) * L::CIN + (k % L::CIN);  // (ky, kx, ci) NHWC
    }
    // per X slot: its sample's base (bytes for u8, elements for f32) and its pixel in
    // that sample; both advance by MS pixels per step (at most one wrap: MS <= P)
    constexpr unsigned long long SAMPLE_F32 = (unsigned long long)L::IH * L::IW * L::CIN;
    const unsigned long long sstride = U8 ? (unsigned long long)a.sample_stride : SAMPLE_F32;
    unsigned long long sb[XV];
    unsigned xp[XV];
#pragma unroll
    for (int i = 0; i < XV; ++i) {
        const unsigned m = mbeg + px0 + i * C::XPS;
        const unsigned n = m / L::P;
        xp[i] = m - n * L::P;
        sb[i] = n * sstride;
    }
    const unsigned xn0 = mbeg / L::P, xp0 = mbeg - xn0 * L::P;  // a pixel that always exists
    const unsigned long long sb0 = xn0 * sstride;
    const int c4 = threadIdx.x % GUPR, gpx0 = threadIdx.x / GUPR;
    const uint8_t* xu8 = reinterpret_cast<const uint8_t*>(a.x);
    const float* xf = reinterpret_cast<const float*>(a.x);

    float4 xr[XV];
    uint32_t xw[XV];
    float4 gr[GV];
    float bsum0 = 0.f, bsum1 = 0.f, bsum2 = 0.f, bsum3 = 0.f;

    // FULL: every pixel of the step is inside the slice (all steps but possibly the
    // last of the last slice — splits are whole steps long); otherwise pixels past
    // the end read the slice's first pixel and are zeroed by a select
    auto load = [&](unsigned ms, auto full_tag) {
        constexpr bool FULL = decltype(full_tag)::value;
#pragma unroll
        for (int i = 0; i < XV; ++i) {
            bool ok = true;
            unsigned long long sbi = sb[i];
            unsigned pp = xp[i];
            if constexpr (!FULL) {
                ok = ms + px0 + i * C::XPS < mend;
                sbi = ok ? sbi : sb0;
                pp = ok ? pp : xp0;
            }
            const unsigned oy = pp / L::OW, ox = pp - oy * L::OW;
            if constexpr (U8) {
                const uint32_t v =
                    *reinterpret_cast<const uint32_t*>(xu8 + sbi + (oy * L::S * L::IW + ox * L::S + koff));
                xw[i] = ok ? v : 0u;
            } else {
                const float4 v = *reinterpret_cast<const float4*>(
                    xf + sbi + ((oy * L::S) * L::IW + ox * L::S) * L::CIN + koff);
                xr[i] = ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
            }
            xp[i] += MS;  // advance to the next step's pixel
            if (xp[i] >= (unsigned)L::P) {
                xp[i] -= L::P;
                sb[i] += sstride;
            }
        }
#pragma unroll
        for (int j = 0; j < GV; ++j) {
            const unsigned m = ms + gpx0 + j * C::GPS;
            bool ok = true;
            if constexpr (!FULL) ok = m < mend;
            const float4 v = *reinterpret_cast<const float4*>(a.g + (ok ? m : mbeg) * COUT + c4 * 4);
            gr[j] = ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto load_step = [&](unsigned ms) {
        if (ms + MS <= mend)
            load(ms, std::true_type{});
        else
            load(ms, std::false_type{});
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < XV; ++i) {
            float4* d = reinterpret_cast<float4*>(Xs[buf] + (px0 + i * C::XPS) * XST + u * 4);
            if constexpr (U8) {
                *d = make_float4((float)(xw[i] & 0xFFu), (float)((xw[i] >> 8) & 0xFFu), (float)((xw[i] >> 16) & 0xFFu),
                                 (float)(xw[i] >> 24));
            } else {
                *d = xr[i];
            }
        }
#pragma unroll
        for (int j = 0; j < GV; ++j) {
            *reinterpret_cast<float4*>(Gs[buf] + (gpx0 + j * C::GPS) * GST + c4 * 4) = gr[j];
            bsum0 += gr[j].x;
            bsum1 += gr[j].y;
            bsum2 += gr[j].z;
            bsum3 += gr[j].w;
        }
    };

    const unsigned nsteps = mend > mbeg ? (mend - mbeg + MS - 1) / MS : 0;
    if (nsteps > 0) {
        load_step(mbeg);
        store(0);
    }
    __syncthreads();
    const float* Xbase = &Xs[0][0] + (lane >> 5) * XST + kt * 32 + (lane & 31);
    const float* Gbase = &Gs[0][0] + (lane >> 5) * GST + ct * 32 + (lane & 31);
    for (unsigned s = 0; s < nsteps; ++s) {
        const int cur = (int)(s & 1);
        if (s + 1 < nsteps) load_step(mbeg + (s + 1) * MS);
        const float* X = Xbase + cur * (MS * XST);
        const float* G = Gbase + cur * (MS * GST);
#pragma unroll
        for (int kk = 0; kk < MS / 2; ++kk)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(X[kk * 2 * XST], G[kk * 2 * GST], acc, 0, 0, 0);
        if (s + 1 < nsteps) store(cur ^ 1);
        __syncthreads();
    }
    // partial slab [split][K][COUT]: row (k) = kb*KT + kt*32 + C-row, col (co) = ct*32 + (lane & 31)
    float* slab = a.slab + (long long)split * L::K * COUT;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int kr = kb * KT + kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        slab[kr * COUT + ct * 32 + (lane & 31)] = acc[r];
    }
    if (kb == 0) {
        // bias grad partial: column sums of this split's G rows (each thread owns columns c4*4..+3)
        constexpr int GROUPS = 256 / GUPR;
        __shared__ float bred[GROUPS * COUT];
        bred[gpx0 * COUT + c4 * 4 + 0] = bsum0;
        bred[gpx0 * COUT + c4 * 4 + 1] = bsum1;
        bred[gpx0 * COUT + c4 * 4 + 2] = bsum2;
        bred[gpx0 * COUT + c4 * 4 + 3] = bsum3;
        __syncthreads();
        if (threadIdx.x < COUT) {
            float t = 0.f;
            for (int g = 0; g < GROUPS; ++g) t += bred[g * COUT + threadIdx.x];
            a.bslab[(long long)split * COUT + threadIdx.x] = t;
        }
    }
}

// sum the slabs, scatter to PyTorch [co][ci][ky][kx] (+ bias).  A block owns 4·E
// consecutive outputs (E float4 lanes of every slab row) x RG split groups; thread (e, g)
// sums splits g, g+RG, g+2RG, ... in order, then the RG group sums are combined by a
// fixed pairwise tree — one order per output, so the result is deterministic.  E x RG: 32 x 8 for the
// f32 kernels' <= 512 splits; for the split kernels' up to 2048, 32 x 32, or 8 x 128 when
// the layer has few outputs (conv1: 8,224 -> 257 blocks instead of 65, a fuller chip).
template <class L, bool NHWC_ORDER, int RED_E, int RG>
__global__ void __launch_bounds__(RED_E * RG) wgrad_reduce(const float* __restrict__ slab,
                                                         const float* __restrict__ bslab, int splits,
                                                         float* __restrict__ dw, float* __restrict__ db) {
    __shared__ float4 part[RG][RED_E];
    constexpr int KC = L::K * L::COUT;
    static_assert(KC % 4 == 0 && L::COUT % 4 == 0, "wgrad_reduce: float4 lanes");
    const int e = threadIdx.x % RED_E, grp = threadIdx.x / RED_E;
    const int i = (blockIdx.x * RED_E + e) * 4;  // first of this lane's four outputs
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    auto add = [](float4& a, const float4 b) {
        a.x += b.x;
        a.y += b.y;
        a.z += b.z;
        a.w += b.w;
    };
    // (unrolled: a lane's loads of several splits issue together; the adds keep split order)
    if (i < KC) {
#pragma unroll 8
        for (int sp = grp; sp < splits; sp += RG) add(s, *reinterpret_cast<const float4*>(slab + (long long)sp * KC + i));
    } else if (i < KC + L::COUT) {
#pragma unroll 8
        for (int sp = grp; sp < splits; sp += RG)
            add(s, *reinterpret_cast<const float4*>(bslab + (long long)sp * L::COUT + (i - KC)));
    }
    // the RG group sums combined by a fixed pairwise tree (deterministic, and its rounding
    // error grows with log2(RG) rather than RG)
    part[grp][e] = s;
    __syncthreads();
#pragma unroll
    for (int h = RG / 2; h >= 1; h >>= 1) {
        if (grp < h) add(part[grp][e], part[grp + h][e]);
        __syncthreads();
    }
    if (grp != 0) return;
    const float4 t = part[0][e];
    const float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int ic = i + c;
        if (ic < KC) {
            const int k = ic / L::COUT, co = ic % L::COUT;
            int ci, ky, kx;
            if (NHWC_ORDER) {
                ci = k % L::CIN;
                const int tap = k / L::CIN;
                ky = tap / L::KW;
                kx = tap % L::KW;
            } else {
                kx = k % L::KW;
                ky = (k / L::KW) % L::KH;
                ci = k / (L::KW * L::KH);
            }
            dw[((co * L::CIN + ci) * L::KH + ky) * L::KW + kx] = tv[c];
        } else if (ic < KC + L::COUT) {
            db[ic - KC] = tv[c];
        }
    }
}

// ---------------------------------------------------------------------------
// Wgrad, split-f16.  Same decomposition as wgrad_kernel (WG = k-block of KT rows x
// all COUT x a slice of output pixels; partial slabs reduced by wgrad_reduce), on
// v_mfma_f32_32x32x16_f16.  Per step of MS = 32 pixels the X (im2col) and G tiles
// are staged in LDS as f16 planes, row-major [pixel][k] / [pixel][co] (each f32
// value split once per workgroup into its two planes; conv1's u8 frames are
// one exact plane), and the MFMA fragments — 8 consecutive pixels of one k (A) or
// one co (B) per lane — come straight out of LDS with the transposing read
// ds_read_b64_tr_b16 (two per fragment).  32-byte chunks of a row are XOR-swizzled
// (tr_swz) so each 32-lane half's 4 rows x 2 chunks hit 8 distinct bank groups.
// conv1: 3 MFMAs per tile and k-step (x*g0, x*g1, x*g2, all exact); f32 layers: the
// six products of mfma_split6.  Loads of step s+1 fly under the MFMAs of step s.
// ---------------------------------------------------------------------------
template <class L, bool U8, int KT_>
struct WsCfg {
    static constexpr int KT = KT_, KB = L::K / KT, COUT = L::COUT;
    static constexpr int XP = U8 ? 1 : NPL;                      // X planes
    static constexpr int NKT = KT / 32, NCT = COUT / 32, TPW = NKT * NCT / 4;
    // wave grid: WC waves along co (WCT co-tiles each) x 4/WC along k (WKT k-tiles each)
    static constexpr int WCT = TPW % NCT == 0 ? NCT : (NCT % TPW == 0 ? TPW : 1);
    static constexpr int WC = NCT / WCT, WKT = NKT / (4 / WC);
    static constexpr int XR = KT * 2, GR = COUT * 2;             // LDS row bytes
    static constexpr int XPB = MS * XR, GPB = MS * GR;           // LDS plane bytes
    static constexpr int STAGE = XP * XPB + NPL * GPB;
    // staging: 8 threads per pixel row; a thread stages XU units of 8 consecutive k and GW
    // consecutive co of one pixel, so its addresses come from one (sample, pixel) pair
    static constexpr int UPX = KT / 8, XU = UPX / 8, GW = COUT / 8;
    static_assert(KB * KT == L::K && (NKT * NCT) % 4 == 0 && XU * 8 == UPX && (GW == 4 || GW == 8), "wgrad split shape");
    static_assert(WKT * WCT == TPW && 4 % WC == 0 && NKT % (4 / WC) == 0, "wave tiling");
};

// XOR on the 32-byte chunk index of row px (rows of ROWB bytes): the transposed reads
// of a 32-lane half (rows px..px+3, chunks 2t and 2t+1) then cover all 64 banks once
template <int ROWB>
__device__ inline int tr_swz(int px) {
    constexpr int m = (ROWB / 32) & 7;
    static_assert(m == 0 || m == 4 || m == 2, "tr_swz: row stride");
    if constexpr (m == 0) return 2 * (px & 3);
    else if constexpr (m == 4) return 2 * ((px >> 1) & 1);
    else return 0;
}

typedef short v4s16 __attribute__((ext_vector_type(4)));
__device__ inline uint2 lds_tr16(const uint8_t* p) {
    const v4s16 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s16*)p);
    return __builtin_bit_cast(uint2, r);
}

__device__ float kZeroG[64] = {};  // the G row of a pixel past a split's end (global AS: no flat loads)

// CB > 1: G rows hold CB blocks of COUT columns (row stride CB * COUT) and each
// workgroup owns one block — the fc layer's weight gradient (K = the 512 outputs,
// G = the NHWC conv3 activations, one 64-channel pixel per block); its grid is any
// number of (split, column-block, k-block) items, k-block fastest within an XCD.
// XPL / GPL (round 4): X / G are PX planes (conv_common.h; a.xexp / a.gexp): each unit's 8 values
// are read as their two 16-B plane runs and stored to LDS as they are (no split in registers)
template <class L, bool U8, int KT, bool ROWS, int CB = 1, bool XPL = false, bool GPL = false>
__global__ void __launch_bounds__(256, 2) wgrad_split_kernel(WArgs a) {
    using C = WsCfg<L, U8, KT>;
    static_assert(!(XPL && U8) && (!GPL || C::GW == 8), "PX operands: f32 X, 8 G values per thread");
    constexpr int COUT = L::COUT, XP = C::XP, XR = C::XR, GR = C::GR, XU = C::XU;
    constexpr int WKT = C::WKT, WCT = C::WCT, GS = CB * COUT;
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * C::STAGE];
    int kb, split, cb;
    if constexpr (CB == 1) {
        const int b = blockIdx.x, xcd = b & 7, q = b >> 3;
        kb = q % C::KB;
        split = (q / C::KB) * 8 + xcd;
        cb = 0;
    } else {
        // k-block fastest: the KB workgroups that read one G column block (CB > 1: a pixel of
        // the fc layer's h3) run together on one XCD and share it through its L2 (column-block
        // fastest re-streamed every block from HBM once per k-block: 3.5x the algorithmic bytes)
        const long long w = xcd_remap(blockIdx.x, gridDim.x);
        kb = (int)(w % C::KB);
        cb = (int)((w / C::KB) % CB);
        split = (int)(w / (CB * C::KB));
    }
    const unsigned M = (unsigned)(a.batch * L::P);
    const unsigned long long mb64 = (unsigned long long)split * (unsigned long long)a.px_per_split;
    const unsigned mbeg = mb64 < M ? (unsigned)mb64 : M;
    const unsigned mend = (unsigned)min((unsigned long long)M, (unsigned long long)mbeg + a.px_per_split);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kt0 = (wave / C::WC) * WKT, ct0 = (wave % C::WC) * WCT;

    f32x16 hi[WKT][WCT], lo[WKT][WCT];
#pragma unroll
    for (int i = 0; i < WKT; ++i)
#pragma unroll
        for (int j = 0; j < WCT; ++j) hi[i][j] = lo[i][j] = zero16();

    constexpr unsigned long long SAMPLE_F32 = (unsigned long long)L::IH * L::IW * L::CIN;
    const uint8_t* xu8 = reinterpret_cast<const uint8_t*>(a.x);
    const float* xf = reinterpret_cast<const float*>(a.x);
    constexpr int GW = C::GW;
    // raw global data of one step; the pipeline holds two (steps s+1 and s+2 during step s)
    struct Raw {
        uint32_t xw[XU][2];
        float4 xr[XU][2];
        float4 gr[2];
    };
    // one step's f16 planes in registers (split under the MFMAs of the step before)
    struct Planes {
        u32x4 x[XU][NPL];
        u32x4 g[NPL];
        uint2 g4[NPL];
    };
    // operand scales from the amax slots (uint8 X: exact at scale 1); the slab is unscaled
    const int ex = U8 ? 0 : (XPL ? *a.xexp : split_scale_exp(amax_read(a.amax_x)));
    const int eg = GPL ? *a.gexp : split_scale_exp(amax_read(a.amax_g));
    const float sx = exp2i(ex), sg = exp2i(eg), uo = exp2i(-ex) * exp2i(-eg);
    const float ub = GPL ? exp2i(-eg) : 1.f;  // GPL: the bias sums add the scaled values
    Raw raw[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {  // defined values: the last step splits a set it never stores
#pragma unroll
        for (int i = 0; i < XU; ++i) {
            raw[t].xw[i][0] = raw[t].xw[i][1] = 0u;
            raw[t].xr[i][0] = raw[t].xr[i][1] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        raw[t].gr[0] = raw[t].gr[1] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float bsum[GW];
#pragma unroll
    for (int e = 0; e < GW; ++e) bsum[e] = 0.f;
    // this thread's pixel row and units; the pixel advances by MS per step (at most one
    // wrap into the next sample: MS <= P), so no 64-bit index is divided in the loop
    // unit i of the thread is j = 8i + (tid & 7): the 8 threads of a pixel row write 128
    // contiguous bytes per store instruction (bank-conflict-free)
    const int pxl = tid >> 3, ju = tid & 7, gco = (tid & 7) * GW;
    const unsigned long long sstride = U8 ? (unsigned long long)a.sample_stride : SAMPLE_F32;
    // byte (u8) / float offset of sample n: through the rollout rows when a.idx is set (u8
    // only); the next sample's base is fetched one wrap ahead, so the idx load's latency
    // hides under the steps in between
    auto sbase = [&](unsigned n) -> unsigned long long {
        if constexpr (ROWS) {
            const unsigned nc = n < (unsigned)a.batch ? n : (unsigned)a.batch - 1;
            const long long i = a.idx[nc];
            return (unsigned long long)(((i % a.T) * a.Nenv + i / a.T) * (long long)(L::CIN * L::IH * L::IW));
        }
        return n * sstride;
    };
    unsigned xp, mcur = mbeg + pxl, ncur;
    unsigned long long sb, sbn;
    {
        const unsigned m = mcur < M ? mcur : mbeg;
        ncur = m / L::P;
        xp = m - ncur * L::P;
        sb = sbase(ncur);
        sbn = sbase(ncur + 1);
    }
    // a pixel that always exists (an empty split, mbeg == M, still issues its loads)
    const unsigned m0 = mbeg < M ? mbeg : M - 1;
    const unsigned xp0 = m0 - (m0 / L::P) * L::P;
    const unsigned long long sb00 = sbase(m0 / L::P);
    int koff[XU];
#pragma unroll
    for (int i = 0; i < XU; ++i) {
        const int k = kb * KT + 8 * (8 * i + ju);
        if constexpr (U8) {
            koff[i] = ((k >> 6) * L::IH + ((k >> 3) & 7)) * L::IW;
        } else {
            const int tap = k / L::CIN;
            koff[i] = ((tap / L::KW) * L::IW + tap % L::KW) * L::CIN + k % L::CIN;
        }
    }

    // loads of one step (steps are loaded in order; the state above advances).  Branch-free,
    // so the loads, the split of the step before and the MFMAs share one basic block: a pixel
    // past the split's end loads a valid pixel's X (finite) and a zero G row (kZeroG), so its
    // products vanish
    auto load = [&](Raw& r) {
        const bool ok = mcur < mend;
        const unsigned p = ok ? xp : xp0;
        const unsigned long long s0 = ok ? sb : sb00;
        const unsigned oy = p / L::OW, ox = p - oy * L::OW;
        if constexpr (U8) {
            const uint8_t* s = xu8 + s0 + oy * L::S * L::IW + ox * L::S;
#pragma unroll
            for (int i = 0; i < XU; ++i) {
                r.xw[i][0] = *reinterpret_cast<const uint32_t*>(s + koff[i]);
                r.xw[i][1] = *reinterpret_cast<const uint32_t*>(s + koff[i] + 4);
            }
        } else if constexpr (XPL) {
            // the unit's 8 channels lie in one 32-group: its high plane run, and 64 B on its low one
            const char* s = reinterpret_cast<const char*>(xf) + 4 * (s0 + (oy * L::S * L::IW + ox * L::S) * L::CIN);
#pragma unroll
            for (int i = 0; i < XU; ++i) {
                const char* q = s + 4 * (koff[i] & ~31) + 2 * (koff[i] & 31);
                r.xr[i][0] = *reinterpret_cast<const float4*>(q);
                r.xr[i][1] = *reinterpret_cast<const float4*>(q + 64);
            }
        } else {
            const float* s = xf + s0 + (oy * L::S * L::IW + ox * L::S) * L::CIN;
#pragma unroll
            for (int i = 0; i < XU; ++i) {
                r.xr[i][0] = *reinterpret_cast<const float4*>(s + koff[i]);
                r.xr[i][1] = *reinterpret_cast<const float4*>(s + koff[i] + 4);
            }
        }
        if constexpr (GPL) {
            const unsigned long long ge = (unsigned long long)mcur * GS + cb * COUT + gco;  // gco % 8 == 0
            const char* q = ok ? reinterpret_cast<const char*>(a.g) + 4 * (ge & ~31ULL) + 2 * (ge & 31)
                               : reinterpret_cast<const char*>(kZeroG) + 4 * (gco & ~31) + 2 * (gco & 31);
            r.gr[0] = *reinterpret_cast<const float4*>(q);
            r.gr[1] = *reinterpret_cast<const float4*>(q + 64);
        } else {
            const float* sg = ok ? a.g + (unsigned long long)mcur * GS + cb * COUT + gco : kZeroG + gco;
            r.gr[0] = *reinterpret_cast<const float4*>(sg);
            if constexpr (GW == 8) r.gr[1] = *reinterpret_cast<const float4*>(sg + 4);
        }
        mcur += MS;
        if constexpr (L::P == 1) {  // one pixel per sample (the fc layer): sample = pixel
            sb = (unsigned long long)mcur * sstride;
            return;
        }
        xp += MS;
        const bool wrap = xp >= (unsigned)L::P;
        xp = wrap ? xp - L::P : xp;
        if constexpr (ROWS) {
            if (wrap) {  // rollout rows: the next sample's base was fetched one wrap ahead
                ++ncur;
                sb = sbn;
                sbn = sbase(ncur + 1);
            }
        } else {
            sb = wrap ? sb + sstride : sb;
        }
    };
    auto to_planes = [&](const Raw& r, Planes& p) {
#pragma unroll
        for (int i = 0; i < XU; ++i) {
            if constexpr (U8) {
                p.x[i][0] = u8x8_to_f16(r.xw[i][0], r.xw[i][1]);
            } else if constexpr (XPL) {
                p.x[i][0] = __builtin_bit_cast(u32x4, r.xr[i][0]);
                p.x[i][1] = __builtin_bit_cast(u32x4, r.xr[i][1]);
            } else {
                split8h(r.xr[i][0], r.xr[i][1], sx, p.x[i][0], p.x[i][1]);
            }
        }
        if constexpr (GPL) {
            p.g[0] = __builtin_bit_cast(u32x4, r.gr[0]);
            p.g[1] = __builtin_bit_cast(u32x4, r.gr[1]);
        } else if constexpr (GW == 8) {
            split8h(r.gr[0], r.gr[1], sg, p.g[0], p.g[1]);
        } else {
            split4h(r.gr[0], sg, p.g4[0], p.g4[1]);
        }
    };
    auto store = [&](const Planes& p, const Raw& r, int buf) {
        uint8_t* base = lds + buf * C::STAGE;
#pragma unroll
        for (int i = 0; i < XU; ++i) {
            const int j = 8 * i + ju;
            const int off = pxl * XR + (((j >> 1) ^ tr_swz<XR>(pxl)) << 5) + ((j & 1) << 4);
#pragma unroll
            for (int q = 0; q < XP; ++q) *reinterpret_cast<u32x4*>(base + q * C::XPB + off) = p.x[i][q];
        }
        uint8_t* gb = base + XP * C::XPB;
        const int goff = pxl * GR + (((gco >> 4) ^ tr_swz<GR>(pxl)) << 5) + (gco & 15) * 2;
#pragma unroll
        for (int q = 0; q < NPL; ++q) {
            if constexpr (GW == 8)
                *reinterpret_cast<u32x4*>(gb + q * C::GPB + goff) = p.g[q];
            else
                *reinterpret_cast<uint2*>(gb + q * C::GPB + goff) = p.g4[q];
        }
        if constexpr (GPL) {
            if constexpr (CB == 1) {  // the bias gradient (the fc layer has none here): hi + lo, scaled
                const u32x4 hw = p.g[0], lw = p.g[1];
#pragma unroll
                for (int e = 0; e < 8; ++e) bsum[e] += px_value(hw[e >> 1], lw[e >> 1], e & 1);
            }
        } else {
            bsum[0] += r.gr[0].x;
            bsum[1] += r.gr[0].y;
            bsum[2] += r.gr[0].z;
            bsum[3] += r.gr[0].w;
            if constexpr (GW == 8) {
                bsum[4] += r.gr[1].x;
                bsum[5] += r.gr[1].y;
                bsum[6] += r.gr[1].z;
                bsum[7] += r.gr[1].w;
            }
        }
    };
    // per-lane transposed-read offsets (T10): lane 4qq+pp of each 16-lane group supplies
    // row qq, columns 4pp..4pp+3 of its 4-row x 16-column block; the block's rows are
    // pixels 16ks + 8h + 4r + qq, its columns chunk 2t + g16 of the row
    const int g16 = (lane >> 4) & 1, h = lane >> 5, qq = (lane >> 2) & 3, pp = lane & 3;
    const int rowx = (8 * h + qq) * XR + pp * 8, rowg = (8 * h + qq) * GR + pp * 8;
    const int swx = tr_swz<XR>(qq), swg = tr_swz<GR>(qq);
    auto frag = [&](const uint8_t* plane, int rowoff, int rowb, int chunk, int ks) {
        const uint8_t* p = plane + rowoff + 16 * ks * rowb + (chunk << 5);
        const uint2 r0 = lds_tr16(p), r1 = lds_tr16(p + 4 * rowb);
        u32x4 f;
        f[0] = r0.x;
        f[1] = r0.y;
        f[2] = r1.x;
        f[3] = r1.y;
        return f;
    };
    auto compute = [&](int buf) {
        const uint8_t* base = lds + buf * C::STAGE;
        const uint8_t* gb = base + XP * C::XPB;
#pragma unroll
        for (int ks = 0; ks < MS / 16; ++ks) {
            u32x4 bq[WCT][NPL];
#pragma unroll
            for (int j = 0; j < WCT; ++j)
#pragma unroll
                for (int p = 0; p < NPL; ++p)
                    bq[j][p] = frag(gb + p * C::GPB, rowg, GR, (2 * (ct0 + j) + g16) ^ swg, ks);
#pragma unroll
            for (int i = 0; i < WKT; ++i) {
                u32x4 aq[NPL];
#pragma unroll
                for (int p = 0; p < XP; ++p) aq[p] = frag(base + p * C::XPB, rowx, XR, (2 * (kt0 + i) + g16) ^ swx, ks);
#pragma unroll
                for (int j = 0; j < WCT; ++j) {
                    if constexpr (U8) {
                        hi[i][j] = mfma_f16(aq[0], bq[j][0], hi[i][j]);
                        lo[i][j] = mfma_f16(aq[0], bq[j][1], lo[i][j]);
                    } else {
                        mfma_split3(aq, bq[j], hi[i][j], lo[i][j]);
                    }
                }
            }
        }
    };

    // two-deep pipeline, one basic block per step: step s+1's raw registers (loaded during
    // step s-1) are split into planes, step s+2's loads are issued into the set just freed,
    // the compiler interleaves the split's VALU work with step s's fragment reads and MFMAs,
    // and the planes go to the other LDS buffer after them.  Raw sets and buffers alternate,
    // so both are static.  (Measured: 5-10 % faster than one-deep staging after the MFMAs;
    // forcing the interleave with sched_group_barrier was slower than the compiler's.)
    const unsigned nsteps = mend > mbeg ? (mend - mbeg + MS - 1) / MS : 0;
    load(raw[0]);
    load(raw[1]);
    if (nsteps > 0) {
        Planes p;
        to_planes(raw[0], p);
        store(p, raw[0], 0);
    }
    __syncthreads();
    auto step = [&](unsigned s, auto cur_tag) {
        constexpr int CUR = decltype(cur_tag)::value;  // LDS buffer and raw set of step s
        Planes p;
        to_planes(raw[CUR ^ 1], p);
        load(raw[CUR]);
        compute(CUR);
        // unconditional (one basic block): past the last step the set holds a zero-G step,
        // written to a buffer nothing reads again (bsum adds zeros)
        store(p, raw[CUR ^ 1], CUR ^ 1);
        __syncthreads();
    };
    for (unsigned s = 0; s < nsteps; s += 2) {
        step(s, std::integral_constant<int, 0>{});
        if (s + 1 < nsteps) step(s + 1, std::integral_constant<int, 1>{});
    }
    float* slab = a.slab + (long long)split * L::K * GS + cb * COUT;
#pragma unroll
    for (int i = 0; i < WKT; ++i)
#pragma unroll
        for (int j = 0; j < WCT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int kr = kb * KT + (kt0 + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                slab[kr * GS + (ct0 + j) * 32 + (lane & 31)] = (hi[i][j][r] + lo[i][j][r]) * uo;
            }
    if (CB == 1 && kb == 0) {
        // bias grad partial: column sums of this split's G rows, combined in a fixed order
        float* bred = reinterpret_cast<float*>(lds);  // the loop ended on a barrier
#pragma unroll
        for (int e = 0; e < GW; ++e) bred[pxl * COUT + gco + e] = bsum[e];
        __syncthreads();
        if (tid < COUT) {
            float t = 0.f;
            for (int g = 0; g < MS; ++g) t += bred[g * COUT + tid];
            a.bslab[(long long)split * COUT + tid] = t * ub;
        }
    }
}

// ---------------------------------------------------------------------------
// conv2 weight gradient from H1P planes, direct (no im2col):
//   dW[tap][ci][co] = sum over samples n and output pixels p = (oy, ox) of
//                     h1[n][2 oy + ky][2 ox + kx][ci] * g2[n][p][co]       (+ db[co] = sum g2)
// One 512-thread workgroup per CU walks its own run of samples.  Per sample the whole H1P image
// (20 x 20 x 32, both f16 planes: 51 KB) is DMA'd into LDS and the sample's 81 G rows (f32) are
// split there into two f16 planes: every h1 and g2 byte is read from HBM once (the im2col form,
// wgrad_split_kernel, re-fetched h1 ~3.2x through L2 and split every value once per k-block).
// The reduction runs over the sample's 81 pixels in 6 k-steps of 16 (G rows 81..95 are zero):
// wave w owns taps 2w, 2w + 1 x all 64 output channels (4 tiles, 12 MFMAs per k-step).  The A
// fragment rows are h1 pixels (2 oy + ky, 2 ox + kx), read with the transposing LDS read: the
// image is stored column-parity split (slot = y * 20 + (x & 1) * 10 + (x >> 1), 64 B per slot and
// plane), so consecutive output pixels of one tap are consecutive slots (conflict-free reads) and
// a tap is one uniform slot offset.  G rows are 128 B per plane with 32-B chunks XOR-swizzled
// (tr_swz<128>).  Double-buffered: sample s + 1's DMAs and G loads fly under sample s's MFMAs.
// Partial slabs per workgroup, summed in a fixed order by wgrad_reduce (deterministic).
// LDS: G planes of both buffers first (so every B read's offset is an immediate), then the H
// images: 2 x 24 KB + 2 x 50 KB = 148 KB.
// ---------------------------------------------------------------------------
constexpr int W2P_GP = 96 * 128;                 // one G plane: 96 rows x 64 co x f16
constexpr int W2P_GB = 2 * W2P_GP;               // both G planes of one buffer
constexpr int W2P_HP = 400 * 64;                 // one H1P plane image: 400 slots x 32 ci x f16
constexpr int W2P_HB = 2 * W2P_HP;               // both planes of one buffer
constexpr int W2P_H0 = 2 * W2P_GB;               // the H images follow both buffers' G planes
constexpr int W2P_LDS = 2 * W2P_GB + 2 * W2P_HB;  // 151,552 B
constexpr int W2P_NDMA = 7;                      // 1-KB DMAs per wave and sample (50 per sample)
constexpr int W2P_SAMPLE = 400 * 128;            // H1P bytes per sample
constexpr int W2P_G4 = 81 * 64 / 4;              // float4 of G per sample (1296)
static_assert(W2P_LDS <= 160 * 1024, "wgrad2 planes: LDS");
static_assert(8 * W2P_NDMA >= 2 * W2P_HP / 1024 && 2 * W2P_HP % 1024 == 0, "wgrad2 planes: DMA split");

struct W2PArgs {
    const uint16_t* h1p;     // H1P [batch][400][32 hi | 32 lo]
    const int* h1_exp;       // h1 * 2^E = hi + lo
    const float* g;          // g2 [batch][81][64] f32 NHWC (ReLU mask applied), or its PX planes (g_exp)
    const uint32_t* amax_g;  // g2's amax slots (f32 g2)
    const int* g_exp = nullptr;  // PX g2: the planes' exponent
    float* slab;             // [gridDim.x][512][64]
    float* bslab;            // [gridDim.x][64]
    long long batch;
    int per;                 // samples per workgroup (every workgroup has at least one)
};

typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));
// transposing LDS read in inline asm: hipcc would otherwise wait for the in-flight LDS-DMA of the
// next sample (vmcnt(0)) before every read, exposing the prefetch
__device__ inline u32x2v w2p_tr(uint32_t addr) {
    u32x2v r;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr));
    return r;
}
template <int OFF>
__device__ inline u32x2v w2p_tr_o(uint32_t addr) {
    u32x2v r;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
    return r;
}
// one k-step's 16 fragment halves landed (tied, so the MFMAs use the post-wait values)
__device__ inline void w2p_lgkm_wait(u32x2v (&x)[16]) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),
                   "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]),
                   "+v"(x[15]));
}
__device__ inline int w2p_tapoff(int t) {  // uniform slot offset of tap t = ky * 4 + kx
    const int ky = t >> 2, kx = t & 3;
    return 20 * ky + 10 * (kx & 1) + (kx >> 1);
}

// GPL: g2 arrives as its PX planes (round 5: the conv3 dgrad's planes output) — copied to LDS as they lie
// (no split), the bias partials summed from the planes
template <bool GPL>
__global__ void __launch_bounds__(512, 1) wgrad2_planes_kernel(W2PArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[W2P_LDS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const long long s0 = (long long)blockIdx.x * a.per;
    const long long s1 = min(a.batch, s0 + (long long)a.per);
    const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)lds);
    // operand scales: G by its tensor's amax (PX: its planes' exponent), h1 by its H1P exponent; the
    // slab is unscaled
    const int eg = GPL ? *a.g_exp : split_scale_exp(amax_read(a.amax_g)), ex = *a.h1_exp;
    const float sg = exp2i(eg), uo = exp2i(-eg) * exp2i(-ex);

    // H1P DMA sources of this wave's pieces (byte offsets within a sample): DMA i (0..49) fills
    // LDS bytes [1024 i, 1024 i + 1024) of the image (plane i / 25); lane l's 16 B are piece
    // (l & 3) of slot (1024 (i % 25) + 16 l) / 64.  DMAs past the 50th re-copy the 50th.
    uint32_t hsrc[W2P_NDMA];
#pragma unroll
    for (int j = 0; j < W2P_NDMA; ++j) {
        int i = wave * W2P_NDMA + j;
        i = i < 49 ? i : 49;
        const int P = i / 25, within = (i % 25) * 1024 + lane * 16;
        const int slot = within >> 6, piece = (within >> 4) & 3;
        const int y = slot / 20, xs = slot % 20, x = xs < 10 ? 2 * xs : 2 * (xs - 10) + 1;
        hsrc[j] = (uint32_t)((y * 20 + x) * 128 + P * 64 + piece * 16);
    }
    auto dma_h = [&](long long n, int buf) {
        const char* sb = reinterpret_cast<const char*>(a.h1p) + n * W2P_SAMPLE;  // uniform 64-bit sample base
#pragma unroll
        for (int j = 0; j < W2P_NDMA; ++j) {
            int i = wave * W2P_NDMA + j;
            i = i < 49 ? i : 49;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(sb + hsrc[j]),
                (__attribute__((address_space(3))) void*)(lds + W2P_H0 + buf * W2P_HB + i * 1024), 16, 0, 0);
        }
    };
    // G: float4 q = tid + 512 r of the sample's 1296 (row q >> 4, channels 4 (q & 15) ..); the third
    // only for tid < 272 (others re-load the last float4 and store nothing)
    const int gc4 = tid & 15;
    float4 graw[3];
    auto load_g = [&](long long n) {
        const float4* src = reinterpret_cast<const float4*>(a.g) + n * W2P_G4;
        graw[0] = src[tid];
        graw[1] = src[tid + 512];
        graw[2] = src[tid < W2P_G4 - 1024 ? tid + 1024 : W2P_G4 - 1];
    };
    // bias partials: f32 g2 — the thread's 4 channels (gc4); planes — the 8 channels of its 16-B piece gc4
    // of one plane (summed as values of that plane: hi and lo partials added at the end)
    float bsum[GPL ? 8 : 4] = {};
    auto store_g = [&](int buf, bool add_bias) {
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            if (GPL && (r < 2 || tid < W2P_G4 - 1024)) {
                // piece gc4 of a 256-B pixel: plane P = (gc4 >> 2) & 1, channels c0 .. c0 + 7
                const int row = (tid + 512 * r) >> 4, P = (gc4 >> 2) & 1, c0 = 32 * (gc4 >> 3) + 8 * (gc4 & 3);
                const int chunk = c0 >> 4;
                const int off = buf * W2P_GB + P * W2P_GP + row * 128 + ((chunk ^ (2 * ((row >> 1) & 1))) << 5) +
                                (c0 & 15) * 2;
                *reinterpret_cast<float4*>(lds + off) = graw[r];
                if (add_bias) {
                    const f16x8 hv = __builtin_bit_cast(f16x8, graw[r]);
#pragma unroll
                    for (int e = 0; e < 8; ++e) bsum[e] += (float)hv[e];
                }
            } else if (!GPL && (r < 2 || tid < W2P_G4 - 1024)) {
                const int row = (tid + 512 * r) >> 4, chunk = gc4 >> 2;
                const int off = buf * W2P_GB + row * 128 + ((chunk ^ (2 * ((row >> 1) & 1))) << 5) + (gc4 & 3) * 8;
                uint2 hv, lv;
                split4h(graw[r], sg, hv, lv);
                *reinterpret_cast<uint2*>(lds + off) = hv;
                *reinterpret_cast<uint2*>(lds + off + W2P_GP) = lv;
                if (add_bias) {
                    bsum[0] += graw[r].x;
                    bsum[1] += graw[r].y;
                    bsum[2] += graw[r].z;
                    bsum[3] += graw[r].w;
                }
            }
        }
    };
    // zero G rows 81..95 of both buffers and planes once (the loads never write them)
    if (tid < 480) {
        const int pl = tid / 120, o = (tid % 120) * 16;
        *reinterpret_cast<u32x4*>(lds + pl * W2P_GP + 81 * 128 + o) = u32x4{0u, 0u, 0u, 0u};
    }

    // fragment addresses: lane (h, g16, qq, pp) supplies row qq (+ 4 for the second read) of the
    // 8-row group h of k-step ks, 8 B at column chunk g16
    const int h = lane >> 5, g16 = (lane >> 4) & 1, qq = (lane >> 2) & 3, pp = lane & 3;
    uint32_t aaddr[6][2];
#pragma unroll
    for (int ks = 0; ks < 6; ++ks)
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            int p = 16 * ks + 8 * h + 4 * r + qq;
            p = p < 81 ? p : 80;  // rows past the 81 pixels: any valid slot (their G rows are zero)
            aaddr[ks][r] = lds0 + W2P_H0 + (uint32_t)((40 * (p / 9) + p % 9) * 64 + g16 * 32 + pp * 8);
        }
    const uint32_t toff[2] = {(uint32_t)w2p_tapoff(2 * wave) * 64u, (uint32_t)w2p_tapoff(2 * wave + 1) * 64u};
    const int swz = 2 * ((qq >> 1) & 1);
    const uint32_t baddr[2] = {lds0 + (uint32_t)((8 * h + qq) * 128 + (((0 + g16) ^ swz) << 5) + pp * 8),
                               lds0 + (uint32_t)((8 * h + qq) * 128 + (((2 + g16) ^ swz) << 5) + pp * 8)};

    f32x16 hi[2][2], lo[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) hi[i][j] = lo[i][j] = zero16();

    auto compute = [&](auto BUF) {
        constexpr int buf = decltype(BUF)::value;
#pragma unroll
        for (int ks = 0; ks < 6; ++ks) {
            u32x2v v[16];  // [i or j][plane][r]: A halves 0..7, B halves 8..15
            // the k-step's two row addresses, laundered so the compiler does not hoist all 96
            // (k-step, row, tap, plane, buffer) sums out of the sample loop into registers
            uint32_t ab[2] = {aaddr[ks][0], aaddr[ks][1]};
            asm volatile("" : "+v"(ab[0]), "+v"(ab[1]));
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int P = 0; P < 2; ++P)
#pragma unroll
                    for (int r = 0; r < 2; ++r)
                        v[(i * 2 + P) * 2 + r] = w2p_tr(ab[r] + (toff[i] + (uint32_t)(buf * W2P_HB + P * W2P_HP)));
            // B: co-tile j, plane P, rows +0 / +4 of the k-step (offsets are immediates)
            constexpr int B0 = buf * W2P_GB;
            auto bread = [&](auto KS) {
                constexpr int o = B0 + decltype(KS)::value * 2048;
                v[8] = w2p_tr_o<o>(baddr[0]);
                v[9] = w2p_tr_o<o + 512>(baddr[0]);
                v[10] = w2p_tr_o<o + W2P_GP>(baddr[0]);
                v[11] = w2p_tr_o<o + W2P_GP + 512>(baddr[0]);
                v[12] = w2p_tr_o<o>(baddr[1]);
                v[13] = w2p_tr_o<o + 512>(baddr[1]);
                v[14] = w2p_tr_o<o + W2P_GP>(baddr[1]);
                v[15] = w2p_tr_o<o + W2P_GP + 512>(baddr[1]);
            };
            switch (ks) {  // ks is a constant of the unrolled loop
                case 0: bread(std::integral_constant<int, 0>{}); break;
                case 1: bread(std::integral_constant<int, 1>{}); break;
                case 2: bread(std::integral_constant<int, 2>{}); break;
                case 3: bread(std::integral_constant<int, 3>{}); break;
                case 4: bread(std::integral_constant<int, 4>{}); break;
                default: bread(std::integral_constant<int, 5>{}); break;
            }
            w2p_lgkm_wait(v);
            u32x4 af[2][NPL], bf[2][NPL];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int P = 0; P < 2; ++P) {
                    const u32x2v x0 = v[(i * 2 + P) * 2], x1 = v[(i * 2 + P) * 2 + 1];
                    const u32x2v y0 = v[8 + (i * 2 + P) * 2], y1 = v[8 + (i * 2 + P) * 2 + 1];
                    af[i][P] = u32x4{x0.x, x0.y, x1.x, x1.y};
                    bf[i][P] = u32x4{y0.x, y0.y, y1.x, y1.y};
                }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) mfma_split3(af[i], bf[j], hi[i][j], lo[i][j]);
        }
    };
    auto barrier = [] { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory"); };

    dma_h(s0, 0);
    load_g(s0);
    store_g(0, true);
    barrier();
    // one step: sample s + 1 (clamped: past the last sample a dummy copy of s into the idle
    // buffer, no bias) issued, sample s computed, s + 1's G split into the other buffer
    auto step = [&](long long s, auto BUF) {
        constexpr int buf = decltype(BUF)::value;
        const bool nxt = s + 1 < s1;
        const long long sn = nxt ? s + 1 : s;
        dma_h(sn, buf ^ 1);
        load_g(sn);
        compute(BUF);
        store_g(buf ^ 1, nxt);
        barrier();
    };
#pragma unroll 1
    for (long long s = s0; s < s1; s += 2) {
        step(s, std::integral_constant<int, 0>{});
        if (s + 1 < s1) step(s + 1, std::integral_constant<int, 1>{});
    }
    float* slab = a.slab + (long long)blockIdx.x * (G2::K * G2::COUT);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int k = (2 * wave + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                slab[k * G2::COUT + j * 32 + (lane & 31)] = (hi[i][j][r] + lo[i][j][r]) * uo;
            }
    // bias partial: threads with the same gc4 hold the same channels; summed in thread order
    float* red = reinterpret_cast<float*>(lds);  // the loop ended on a barrier
    constexpr int NB = GPL ? 8 : 4;
#pragma unroll
    for (int e = 0; e < NB; ++e) red[tid * NB + e] = bsum[e];
    __syncthreads();
    if (tid < G2::COUT) {
        float t = 0.f;
        if constexpr (GPL) {  // channel tid: the high plane's piece, then the low plane's (4 pieces on)
            const int ph = 8 * (tid >> 5) + ((tid & 31) >> 3), e = tid & 7;
            float th = 0.f, tl = 0.f;
            for (int k = 0; k < 32; ++k) th += red[(ph + 16 * k) * 8 + e];
            for (int k = 0; k < 32; ++k) tl += red[(ph + 4 + 16 * k) * 8 + e];
            t = (th + tl) * exp2i(-eg);
        } else {
            const int c4 = tid >> 2, e = tid & 3;
            for (int k = 0; k < 32; ++k) t += red[(c4 + 16 * k) * 4 + e];
        }
        a.bslab[(long long)blockIdx.x * G2::COUT + tid] = t;
    }
}

// ---------------------------------------------------------------------------
// conv1 weight gradient, direct (no im2col; round 3):
//   dW1[co][ci][ky][kx] = sum over samples n and output pixels (oy, ox) of
//                         x[n][ci][4 oy + ky][4 ox + kx] * g1[n][oy][ox][co]   (+ db1[co] = sum g1)
// One 512-thread workgroup per CU walks its own run of samples in units of half a sample: 10 output
// rows, whose input rows 40 hh .. 40 hh + 43 of the 4 channels are 14.8 KB of frame bytes and whose
// 200 g1 rows are 25.6 KB — every frame and g1 byte is read from HBM once (the im2col form,
// wgrad_split_kernel, re-read each frame byte ~3.6x through L2: 8x8 windows at stride 4, and ran
// latency-bound at small batches).  A unit's frame rows go global -> registers -> LDS phase-split:
// byte x of a row is stored at phase x & 3, position x >> 2, so the 8 output pixels (4 ox + kx) of
// one tap are 8 consecutive bytes of one phase row, from position ox + (kx >> 2) (an 8-B and a
// 4-B read, shifted by v_alignbyte).  Its g1 rows are split into two f16 planes in LDS (split-f16,
// the scale from g1's amax slots), 24 slots per output row (ox 20..23 hold zero rows, so the
// k-steps of 16 pixels never straddle a row).  MFMA D[k][co] += X[k][px] G[px][co], k = 64 ci +
// 8 ky + kx: eight tiles of 32 k; wave w owns tiles 2 (w & 3) and 2 (w & 3) + 1 (input channel
// w & 3) on the k-steps of parity w >> 2, two exact products per tile (x * g_hi, x * g_lo: frames
// are exact in f16) in separate accumulators.  Double-buffered: unit u + 1's loads fly under unit
// u's MFMAs.  Each workgroup writes two partial slabs (its two k-step parities), summed with the
// others in a fixed order by wgrad_reduce (deterministic).  LDS: 2 x (23.4 + 30 KB) = 107 KB.
// ---------------------------------------------------------------------------
constexpr int W1F_ROWS = 44;                   // input rows of a unit (per channel)
constexpr int W1F_PR = 32;                     // bytes per phase row (positions 0..20 real; reads reach 27)
constexpr int W1F_YS = 4 * W1F_PR + 8;         // bytes per (ci, y): four phase rows + 8 (spreads the banks)
constexpr int W1F_PH = 4 * W1F_ROWS * W1F_YS;  // phase image of a unit: 23,936 B
constexpr int W1F_GP = 240 * 64;               // one G plane: 10 rows x 24 slots x 32 co x f16
constexpr int W1F_BUF = W1F_PH + 2 * W1F_GP;   // one buffer: 54,656 B
constexpr int W1F_LDS = 2 * W1F_BUF;           // 109,312 B
constexpr int W1F_XU = 4 * W1F_ROWS * 6;       // frame pieces of a unit: (ci, y, 16-B group) = 1056
constexpr int W1F_G4 = 200 * 8;                // float4 of g1 per unit: 1600
constexpr int W1F_SAMPLE = 4 * 84 * 84;        // frame bytes per sample
constexpr int W1F_DEPTH = 2;  // units of loads in flight (register sets)
constexpr int W1F_FLUSH = 8;  // units per partial sum (4 samples: ~960 pixels per accumulation chain and parity)
static_assert(W1F_DEPTH == 2 || W1F_DEPTH == 3, "wgrad1 frames: two or three register sets");
static_assert(W1F_LDS <= 160 * 1024 && W1F_PH % 16 == 0 && W1F_YS % 8 == 0, "wgrad1 frames: LDS layout");
static_assert(W1F_XU <= 3 * 512 && W1F_G4 <= 4 * 512, "wgrad1 frames: loads per thread");

struct W1FArgs {
    const uint8_t* x;          // frames (u8), sample n at n * sample_stride, or rollout row idx[n]
    long long sample_stride;
    const long long* idx;      // optional env-major rollout rows of the step-major (T, Nenv, 4, 84, 84) frames
    long long T, Nenv;
    const float* g;            // g1 [batch][400][32] f32 NHWC (ReLU mask applied)
    const uint32_t* amax_g;    // g1's amax slots
    float* slab;               // [2 gridDim.x][256][32]
    float* bslab;              // [2 gridDim.x][32]
    long long batch;
    int per;                   // samples per workgroup (every workgroup has at least one)
};

typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

template <bool IDX>
__global__ void __launch_bounds__(512, 1) wgrad1_frames_kernel(W1FArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[W1F_LDS];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const long long n0 = (long long)blockIdx.x * a.per;
    const long long n1 = min(a.batch, n0 + (long long)a.per);
    const int nunits = (int)(2 * (n1 - n0));
    const int eg = split_scale_exp(amax_read(a.amax_g));
    const float sg = exp2i(eg), uo = exp2i(-eg);

    // frame base of a sample; through idx the next sample's row is fetched one sample ahead
    // (host-checked T * Nenv < 2^31: 32-bit row arithmetic)
    const uint32_t T32 = (uint32_t)a.T, N32 = (uint32_t)a.Nenv;
    auto row_base = [&](long long i) -> long long {
        const uint32_t i32 = (uint32_t)i, q = i32 / T32;
        return (long long)((i32 - q * T32) * N32 + q) * (long long)W1F_SAMPLE;
    };
    long long base = IDX ? row_base(a.idx[n0]) : n0 * a.sample_stride;
    long long pref = IDX ? a.idx[n0 + 1 < n1 ? n0 + 1 : n0] : 0;

    // this thread's loads of a unit: frame pieces q = tid + 512 j (ci, y, 16-B group), g1 float4s
    // q = tid + 512 j (pixel q >> 3, channels 4 (q & 7) ..); past the ends a clamped piece is loaded
    // and not stored.  W1F_DEPTH register sets: unit v's in set v % W1F_DEPTH, loaded that many units ahead
    struct Raw {
        u32x4 x[3];
        float4 g[4];
    };
    Raw raw[W1F_DEPTH];
    auto load = [&](Raw& r, long long b, long long n, int hh) {
        u32x4 (&xr)[3] = r.x;
        float4 (&gr)[4] = r.g;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            int q = tid + 512 * j;
            q = q < W1F_XU ? q : W1F_XU - 1;
            const int ci = q / (W1F_ROWS * 6), rem = q - ci * (W1F_ROWS * 6), y = rem / 6, jg = rem - y * 6;
            const long long off = b + ci * (84 * 84) + (40 * hh + y) * 84 + (jg < 5 ? 16 * jg : 68);
            const u32x4a4 v = *reinterpret_cast<const u32x4a4*>(a.x + off);
            xr[j] = u32x4{v.x, v.y, v.z, v.w};
        }
        const float4* gs = reinterpret_cast<const float4*>(a.g + (n * 400 + hh * 200) * 32);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int q = tid + 512 * j;
            gr[j] = gs[q < W1F_G4 ? q : W1F_G4 - 1];
        }
    };
    float bsum[4] = {0.f, 0.f, 0.f, 0.f};
    auto store = [&](const Raw& r, int buf, bool add_bias) {
        const u32x4 (&xr)[3] = r.x;
        const float4 (&gr)[4] = r.g;
        uint8_t* B = lds + buf * W1F_BUF;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int q = tid + 512 * j;
            if (q < W1F_XU) {
                const int ci = q / (W1F_ROWS * 6), rem = q - ci * (W1F_ROWS * 6), y = rem / 6, jg = rem - y * 6;
                // dwords d0..d3 = positions 4 jg .. 4 jg + 3 (jg = 5: only position 20, the load's last dword)
                const bool last = jg == 5;
                const uint32_t d0 = last ? xr[j][3] : xr[j][0], d1 = last ? 0u : xr[j][1];
                const uint32_t d2 = last ? 0u : xr[j][2], d3 = last ? 0u : xr[j][3];
                // 4 x 4 byte transpose: phase r's dword = byte r of d0..d3
                const uint32_t e01 = __builtin_amdgcn_perm(d1, d0, 0x06020400u), o01 = __builtin_amdgcn_perm(d1, d0, 0x07030501u);
                const uint32_t e23 = __builtin_amdgcn_perm(d3, d2, 0x06020400u), o23 = __builtin_amdgcn_perm(d3, d2, 0x07030501u);
                uint8_t* dst = B + (ci * W1F_ROWS + y) * W1F_YS + 4 * jg;
                *reinterpret_cast<uint32_t*>(dst + 0 * W1F_PR) = __builtin_amdgcn_perm(e23, e01, 0x05040100u);
                *reinterpret_cast<uint32_t*>(dst + 1 * W1F_PR) = __builtin_amdgcn_perm(o23, o01, 0x05040100u);
                *reinterpret_cast<uint32_t*>(dst + 2 * W1F_PR) = __builtin_amdgcn_perm(e23, e01, 0x07060302u);
                *reinterpret_cast<uint32_t*>(dst + 3 * W1F_PR) = __builtin_amdgcn_perm(o23, o01, 0x07060302u);
            }
        }
        uint8_t* G = B + W1F_PH;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int q = tid + 512 * j;
            if (q < W1F_G4) {
                const int px = q >> 3, slot = (px / 20) * 24 + px % 20;
                uint2 hv, lv;
                split4h(gr[j], sg, hv, lv);
                *reinterpret_cast<uint2*>(G + slot * 64 + (q & 7) * 8) = hv;
                *reinterpret_cast<uint2*>(G + W1F_GP + slot * 64 + (q & 7) * 8) = lv;
                if (add_bias) {
                    bsum[0] += gr[j].x;
                    bsum[1] += gr[j].y;
                    bsum[2] += gr[j].z;
                    bsum[3] += gr[j].w;
                }
            }
        }
    };
    // zero G rows of the pad slots (ox 20..23) of both buffers and planes once: 640 x 16 B
    for (int i = tid; i < 640; i += 512) {
        const int bp = i / 160, w = i % 160, row = w / 16, c = w % 16;  // (buffer, plane), output row, 16 B
        *reinterpret_cast<u32x4*>(lds + (bp >> 1) * W1F_BUF + W1F_PH + (bp & 1) * W1F_GP + (row * 24 + 20) * 64 + c * 16) =
            u32x4{0u, 0u, 0u, 0u};
    }

    // A: lane (m, h) of tile 2 tp + tt holds k = 64 tp + 32 tt + m: ky = 4 tt + (m >> 3), kx = m & 7
    const int tp = wave & 3, par = wave >> 2, m = lane & 31, h = lane >> 5;
    const int kx = m & 7, sh = kx >> 2;
    int abase[2];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) abase[tt] = (tp * W1F_ROWS + 4 * tt + (m >> 3)) * W1F_YS + (kx & 3) * W1F_PR;
    // B: the transposed-read lane offsets of wgrad_split_kernel (64-B rows, no swizzle)
    const int g16 = (lane >> 4) & 1, qq = (lane >> 2) & 3, pp = lane & 3;
    const int rowg = (8 * h + qq) * 64 + pp * 8 + (g16 << 5);

    // hi / lo: the running products of W1F_FLUSH units, then added into tot and restarted, so no
    // f32 accumulation chain grows past ~1,000 pixels however many samples the workgroup walks
    f32x16 hi[2], lo[2], tot[2];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) hi[tt] = lo[tt] = tot[tt] = zero16();

    auto compute = [&](int buf) {
        const uint8_t* B = lds + buf * W1F_BUF;
        const uint8_t* G = B + W1F_PH;
#pragma unroll
        for (int ks2 = 0; ks2 < 8; ++ks2) {
            const int ks = 2 * ks2 + par;  // this wave's k-steps (15 per unit: parity 1 has seven)
            if (ks < 15) {
                const int gi = 2 * ks + h, goff = (gi / 3) * 4 * W1F_YS + 8 * (gi % 3);
                u32x4 af[2];
#pragma unroll
                for (int tt = 0; tt < 2; ++tt) {
                    const uint8_t* p = B + abase[tt] + goff;
                    const uint2 v = *reinterpret_cast<const uint2*>(p);
                    const uint32_t w2 = *reinterpret_cast<const uint32_t*>(p + 8);
                    af[tt] = u8x8_to_f16(__builtin_amdgcn_alignbyte(v.y, v.x, sh), __builtin_amdgcn_alignbyte(w2, v.y, sh));
                }
                u32x4 bq[2];
#pragma unroll
                for (int P = 0; P < 2; ++P) {
                    const uint8_t* p = G + P * W1F_GP + rowg + 16 * ks * 64;
                    const uint2 r0 = lds_tr16(p), r1 = lds_tr16(p + 4 * 64);
                    bq[P] = u32x4{r0.x, r0.y, r1.x, r1.y};
                }
#pragma unroll
                for (int tt = 0; tt < 2; ++tt) {
                    hi[tt] = mfma_f16(af[tt], bq[0], hi[tt]);
                    lo[tt] = mfma_f16(af[tt], bq[1], lo[tt]);
                }
            }
        }
    };

    // unit v's loads into set v & 1 (past the last unit: the last again, stored to the idle buffer
    // without its bias); a new sample's frame base from the idx value prefetched a sample ahead
    // branch-free (selects, and the idx load issued for every unit): a load under a branch makes
    // hipcc's waits at the join drain every load in flight, the next units' prefetch included
    auto issue = [&](int v, auto SET) {
        const int vc = v < nunits ? v : nunits - 1;
        const long long nv = n0 + (vc >> 1);
        const bool fresh = (v & 1) == 0 && v < nunits && v > 0;
        if constexpr (IDX) {
            // base from the idx value loaded at the previous unit (the next sample's), then the
            // value for the sample after this one (the same load for both halves of a sample)
            base = fresh ? row_base(pref) : base;
            pref = a.idx[nv + 1 < n1 ? nv + 1 : n1 - 1];
        } else {
            base = fresh ? nv * a.sample_stride : base;
        }
        load(raw[decltype(SET)::value], base, nv, vc & 1);
    };
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    using S2 = std::integral_constant<int, 2>;
    issue(0, S0{});
    issue(1, S1{});
    if constexpr (W1F_DEPTH == 3) issue(2, S2{});
    store(raw[0], 0, true);
    __syncthreads();
    // step u (set SET = u % W1F_DEPTH): unit u + W1F_DEPTH's loads into the set unit u held, unit u
    // computed (LDS buffer u & 1), unit u + 1 (loaded earlier) split into the other buffer
    auto step = [&](int u, auto SET) {
        constexpr int set = decltype(SET)::value, nset = (set + 1) % W1F_DEPTH;
        issue(u + W1F_DEPTH, SET);
        compute(u & 1);
        if ((u + 1) % W1F_FLUSH == 0 || u + 1 == nunits) {
#pragma unroll
            for (int tt = 0; tt < 2; ++tt) {
#pragma unroll
                for (int q = 0; q < 16; ++q) tot[tt][q] += hi[tt][q] + lo[tt][q];
                hi[tt] = lo[tt] = zero16();
            }
        }
        store(raw[nset], (u + 1) & 1, u + 1 < nunits);
        __syncthreads();
    };
#pragma unroll 1
    for (int u = 0; u < nunits; u += W1F_DEPTH) {
        step(u, S0{});
        if (u + 1 < nunits) step(u + 1, S1{});
        if constexpr (W1F_DEPTH == 3)
            if (u + 2 < nunits) step(u + 2, S2{});
    }

    const int split = 2 * blockIdx.x + par;
    float* slab = a.slab + (long long)split * (G1::K * G1::COUT);
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int k = 64 * tp + 32 * tt + (r & 3) + 8 * (r >> 2) + 4 * h;
            slab[k * G1::COUT + m] = tot[tt][r] * uo;
        }
    // bias partial: threads with the same tid & 7 hold the same four channels; summed in thread order
    float* red = reinterpret_cast<float*>(lds);  // the loop ended on a barrier
#pragma unroll
    for (int e = 0; e < 4; ++e) red[tid * 4 + e] = bsum[e];
    __syncthreads();
    if (tid < G1::COUT) {
        const int c4 = tid >> 2, e = tid & 3;
        float t = 0.f;
        for (int k = 0; k < 64; ++k) t += red[(c4 + 8 * k) * 4 + e];
        a.bslab[(long long)2 * blockIdx.x * G1::COUT + tid] = t;
        a.bslab[(long long)(2 * blockIdx.x + 1) * G1::COUT + tid] = 0.f;
    }
}

// conv3 output grad: NCHW (Flatten order) -> NHWC, times the ReLU mask of h3 (NCHW)
__global__ void __launch_bounds__(256) nchw_to_nhwc_mask(const float* __restrict__ g, const float* __restrict__ h,
                                                         long long batch, float* __restrict__ out) {
    __shared__ float t[64 * 50];
    const long long n = blockIdx.x;
    const float* gs = g + n * 3136;
    const float* hs = h + n * 3136;
    for (int i = threadIdx.x; i < 3136; i += 256) {
        const int c = i / 49, p = i % 49;
        t[c * 50 + p] = hs[i] > 0.f ? gs[i] : 0.f;
    }
    __syncthreads();
    float* o = out + n * 3136;
    for (int i = threadIdx.x; i < 3136; i += 256) {
        const int p = i / 64, c = i % 64;
        o[i] = t[c * 50 + p];
    }
}

// ---------------------------------------------------------------------------
// weight packing (once per optimizer step)
// ---------------------------------------------------------------------------
// RG: rgemm layout (rg_index); else the igemm's natural [K][NOUT]
template <bool RG>
__device__ inline int pack_pos(int k, int col, int nout, int i) {
    if constexpr (RG) return rg_index(k, col, nout);
    return i;
}
// forward: [K][COUT] in the kernel's K order
template <class L, bool NHWC_ORDER, bool RG>
__global__ void pack_fwd(const float* __restrict__ w, float* __restrict__ wp) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= L::K * L::COUT) return;
    const int k = i / L::COUT, co = i % L::COUT;
    int ci, ky, kx;
    if (NHWC_ORDER) {
        ci = k % L::CIN;
        const int tap = k / L::CIN;
        ky = tap / L::KW;
        kx = tap % L::KW;
    } else {
        kx = k % L::KW;
        ky = (k / L::KW) % L::KH;
        ci = k / (L::KW * L::KH);
    }
    wp[pack_pos<RG>(k, co, L::COUT, i)] = w[((co * L::CIN + ci) * L::KH + ky) * L::KW + kx];
}

// dgrad: [(ky, kx, co)][ci] — chunk (tap, 32 co) is a contiguous 32 x CIN block
template <class L, bool RG>
__device__ inline void pack_dgrad_elem(const float* __restrict__ w, float* __restrict__ wp, int i) {
    if (i >= L::KH * L::KW * L::COUT * L::CIN) return;
    const int ci = i % L::CIN, co = (i / L::CIN) % L::COUT, tap = i / (L::CIN * L::COUT);
    wp[pack_pos<RG>(tap * L::COUT + co, ci, L::CIN, i)] = w[((co * L::CIN + ci) * L::KH + tap / L::KW) * L::KW + tap % L::KW];
}
template <class L, bool RG>
__global__ void pack_dgrad(const float* __restrict__ w, float* __restrict__ wp) {
    pack_dgrad_elem<L, RG>(w, wp, blockIdx.x * blockDim.x + threadIdx.x);
}

template <class Prob>
int launch_igemm(const Args& a, long long blocks, hipStream_t s, const char* name) {
    if (blocks == 0) return PPOX_OK;
    igemm_kernel<Prob><<<(unsigned)blocks, 256, 0, s>>>(a);
    PPOX_LAUNCHED(name);
}

template <class Prob, bool OUT_NCHW = false>
int launch_rgemm(const Args& a, long long blocks, hipStream_t s, const char* name) {
    if (blocks == 0) return PPOX_OK;
    rgemm_kernel<Prob, OUT_NCHW><<<(unsigned)blocks, 256, 0, s>>>(a);
    PPOX_LAUNCHED(name);
}
constexpr int RG_FWD1_MT = 2;

template <class L, bool U8>
int launch_wgrad(const WArgs& wa_in, hipStream_t s) {
    WArgs wa = wa_in;
    using C = WgCfg<L, U8>;
    const long long M = wa.batch * L::P;
    const int splits = wa.splits;
    wa.px_per_split = ppox::ceil_div(ppox::ceil_div(M, splits), MS) * MS;  // whole steps
    wgrad_kernel<L, U8><<<(unsigned)(C::KB * splits), 256, 0, s>>>(wa);
    PPOX_LAUNCHED("ppox_nature_conv_wgrad");
}

template <class L, bool NHWC_ORDER>
int launch_wgrad_reduce(const float* slab, const float* bslab, int splits, float* dw, float* db, hipStream_t s) {
    ppox::ktime_mark(s);
    constexpr int N = L::K * L::COUT + L::COUT;
    if (splits >= 256 && N < 4 * 32 * 256) {  // few outputs, many splits: 8 lanes x 128 split groups
        wgrad_reduce<L, NHWC_ORDER, 8, 128><<<ppox::ceil_div(N, 32), 1024, 0, s>>>(slab, bslab, splits, dw, db);
    } else if (splits >= 256) {  // 32 split groups per element: shorter sequential chains
        wgrad_reduce<L, NHWC_ORDER, 32, 32><<<ppox::ceil_div(N, 128), 1024, 0, s>>>(slab, bslab, splits, dw, db);
    } else {
        wgrad_reduce<L, NHWC_ORDER, 32, 8><<<ppox::ceil_div(N, 128), 256, 0, s>>>(slab, bslab, splits, dw, db);
    }
    PPOX_LAUNCHED("ppox_nature_wgrad_reduce");
}


constexpr int WS_KT2 = 128;
constexpr int WS_KT3 = 64;
constexpr int WS_PX = 2048;  // split wgrad: pixels per split-K slice
constexpr int WS_FILL = 512;  // split wgrad: workgroups at least (conv1 / conv2, small batches)
// split wgrad: its own split-K count (~WS_PX pixels per split so the grid fills the chip)
template <class L, bool U8, int KT, bool XPL = false, bool GPL = false>
struct WsLaunch {
    using C = WsCfg<L, U8, KT>;
    static long long splits(long long batch) {
        const long long px = batch * L::P;
        long long s = (px + WS_PX - 1) / WS_PX;
        // small batches (the 8-GPU per-rank minibatch): enough splits for two workgroups per CU
        // where the k-blocks are few (conv1/conv2 at B = 2048: 0.082 -> 0.074 / 0.100 -> 0.078 ms;
        // conv3's nine k-blocks already give 441 workgroups, and more splits measured slower)
        if constexpr (C::KB <= 4) {
            const long long fill = (WS_FILL + C::KB - 1) / C::KB;
            s = s < fill ? fill : s;
        }
        const long long most = (px + MS - 1) / MS;  // at least one step per split
        s = s > most ? most : s;
        s = s < 8 ? 8 : (s > 2048 ? 2048 : s);
        return (s + 7) / 8 * 8;
    }
    static long long workspace_bytes(long long batch) {
        return splits(batch) * (long long)(L::K * L::COUT + L::COUT) * (long long)sizeof(float);
    }
    static int run(const void* x, long long sample_stride, const float* g, long long batch, void* ws, float* dw,
                   float* db, const uint32_t* amax_x, const uint32_t* amax_g, hipStream_t s,
                   const long long* idx = nullptr, long long T = 0, long long Nenv = 0, const int* xexp = nullptr,
                   const int* gexp = nullptr) {
        const int sp = (int)splits(batch);
        float* slab = reinterpret_cast<float*>(ws);
        WArgs wa{x, sample_stride, g, slab, slab + (long long)sp * L::K * L::COUT, batch, 0, sp, idx, T, Nenv,
                 amax_x, amax_g};
        wa.xexp = xexp;
        wa.gexp = gexp;
        const long long M = batch * L::P;
        wa.px_per_split = ppox::ceil_div(ppox::ceil_div(M, sp), MS) * MS;
        if (U8 && idx != nullptr)
            wgrad_split_kernel<L, U8, KT, U8><<<(unsigned)(C::KB * sp), 256, 0, s>>>(wa);
        else
            wgrad_split_kernel<L, U8, KT, false, 1, XPL, GPL><<<(unsigned)(C::KB * sp), 256, 0, s>>>(wa);
        PPOX_LAUNCHED_NORET("ppox_nature_conv_wgrad_split");
        return launch_wgrad_reduce<L, !U8>(slab, wa.bslab, sp, dw, db, s);
    }
};
using Ws1 = WsLaunch<G1, true, 256>;
using Ws2 = WsLaunch<G2, false, WS_KT2>;
using Ws3 = WsLaunch<G3, false, WS_KT3>;
using Ws3PP = WsLaunch<G3, false, WS_KT3, true, true>;  // PX h2 and g3
using Ws3PF = WsLaunch<G3, false, WS_KT3, true, false>;
using Ws3FP = WsLaunch<G3, false, WS_KT3, false, true>;
// Every per-optimizer-step weight packing of the training step in two launches (the
// minibatch loop is launch-bound at small per-rank batches): wmax_kernel (each weight
// tensor's amax partials, into the tails of the forms packed from it), then pack_all_kernel
// (element ranges of the jobs laid end to end, null outputs skipped; each wave derives the
// tensors' scales from the partials, and the first wave writes every form's exponent).
struct PackAll {
    const float *w1, *w2, *w3, *wfc;
    float* wpd2;                                       // f32 dgrad2 [(tap, co)][ci]
    uint16_t *q1, *q2, *q3, *qd2, *qd3, *qfcf, *qfcd;  // split planes
    const float* wh = nullptr;                         // the heads' hidden layer (512 x 512)
    uint16_t *qhf = nullptr, *qhd = nullptr;           // its forward (W^T) and dgrad (W) forms
    const float* b1 = nullptr;                         // conv1 bias (with q1: the H1P exponent)
    uint32_t* zero = nullptr;                          // words zeroed by wmax_kernel (a pass's amax table)
    long long zero_words = 0;
    const float *b2 = nullptr, *b3 = nullptr;          // conv2 / conv3 biases (with q2 / q3: the PX bounds)
    // round 6: the tensors' amax partials as the Adam step recorded them ([PA_TENSORS][AMAX_SLOTS], the weights
    // unchanged since; null: the packing's own amax pass), and the partials buffer the next Adam step records into
    // (zeroed here; nullable)
    const uint32_t* amax_in = nullptr;
    uint32_t* amax_next = nullptr;
};
constexpr long long PA_N1 = 8 * 2 * 64 * 8, PA_N2 = (long long)G2::K * G2::COUT, PA_N3 = (long long)G3::K * G3::COUT;
constexpr long long PA_NFC = (long long)FcFwd::NCB * FcFwd::K * FcFwd::NOUT;
constexpr long long PA_NFCD = (long long)FcDgrad::NCB * FcDgrad::K * FcDgrad::NOUT;
// the split-GEMM jobs run in 8-element units (pack_frag_unit); q1 and wpd2 per element
constexpr long long PU_2 = PA_N2 / 8, PU_3 = PA_N3 / 8, PU_FC = PA_NFC / 8, PU_FCD = PA_NFCD / 8;
constexpr long long PA_NH = (long long)HeadFwd::NCB * HeadFwd::K * HeadFwd::NOUT, PU_H = PA_NH / 8;
// planes (uint16) of each packed form; a buffer is planes + 2 * PACK_TAIL32 uint16
constexpr long long PL_Q1 = FWD1_PACK, PL_Q2 = NPL * PA_N2, PL_Q3 = NPL * PA_N3, PL_FCF = NPL * PA_NFC,
                    PL_FCD = NPL * PA_NFCD, PL_H = NPL * PA_NH;
static_assert(PL_FCF == PL_FCD, "fc forms: one size");

// source value (k, col) of layer L's forward [K][COUT] (NHWC K order) or dgrad [(tap, co)][ci]
// matrix, from the PyTorch [co][ci][ky][kx] weights
template <class L, bool DGRAD>
struct ConvSrc {
    const float* w;
    __device__ float operator()(int k, int col) const {
        int co, ci, tap;
        if (DGRAD) {
            ci = col;
            co = k % L::COUT;
            tap = k / L::COUT;
        } else {
            co = col;
            ci = k % L::CIN;
            tap = k / L::CIN;
        }
        return w[((co * L::CIN + ci) * L::KH + tap / L::KW) * L::KW + tap % L::KW];
    }
};
// source value (k, col) of column block cb of a GemmRows B (w[n][k] when TRANS, w[k][n] otherwise);
// PERM (the fc layer): its 3136-wide side (K of the forward, N of the dgrad) in NHWC feature order
template <class Prob, bool TRANS, bool PERM>
struct RowsSrc {
    const float* w;
    int cb;
    __device__ float operator()(int k, int col) const {
        const int n = cb * Prob::NOUT + col;
        if (n >= Prob::N) return 0.f;
        const int f = PERM ? fc_nchw_feature(TRANS ? k : n) : (TRANS ? k : n);
        return TRANS ? w[(long long)n * Prob::K + f] : w[(long long)k * Prob::N + f];
    }
};
template <class Prob, bool TRANS, bool PERM = true>
__device__ inline void pack_rows_unit(const float* w, float s, uint16_t* q, long long u) {
    constexpr long long per = (long long)Prob::K * Prob::NOUT / 8;
    const int cb = (int)(u / per);
    pack_frag_unit<Prob::NOUT>(RowsSrc<Prob, TRANS, PERM>{w, cb}, s, q + (long long)cb * Prob::K * Prob::NOUT * NPL,
                               u - cb * per);
}

// The fc forms, enumerated so that consecutive units read consecutive floats of w (the
// permutation f = p * 64 + c <- c * 49 + p otherwise turns every lane's reads into 49-float
// strides across all of W): unit u = (outer, c-group or k-group, p) with p (0..48) fastest.
//   TRANS (forward, B[k][n] = W[n][c * 49 + p], k = p * 64 + c): u = (n, g, p), values
//     c = 8g .. 8g + 7 of column n at k0 = p * 64 + 8g;
//   dgrad (B[k][n] = W[k][c * 49 + p], n = p * 64 + c): u = (kg, c, p), values k = 8kg .. 8kg + 7
//     of column n (block p, column c of the block).
template <bool TRANS>
__device__ inline void pack_fc_unit(const float* __restrict__ w, float s, uint16_t* __restrict__ q, long long u) {
    constexpr int K = TRANS ? 3136 : 512, NT = 2;
    const int p = (int)(u % 49);
    const long long r = u / 49;
    int k0, col, cb;
    float v[8];
    if constexpr (TRANS) {
        const int g = (int)(r & 7), n = (int)(r >> 3);
        const float* src = w + (long long)n * 3136 + 8 * g * 49 + p;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = src[e * 49];
        k0 = p * 64 + 8 * g, col = n & 63, cb = n >> 6;
    } else {
        const int c = (int)(r & 63), kg = (int)(r >> 6);
        const float* src = w + (long long)(8 * kg) * 3136 + c * 49 + p;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = src[(long long)e * 3136];
        k0 = 8 * kg, col = c, cb = p;
    }
    u32x4 p0, p1;
    split8h(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), s, p0, p1);
    const int cs = k0 >> 4, h = (k0 >> 3) & 1, j = col >> 5, l = h * 32 + (col & 31);
    u32x4* d = reinterpret_cast<u32x4*>(q + (long long)cb * K * 64 * NPL + ((long long)(cs * NT + j) * NPL) * 512) + l;
    d[0] = p0;
    d[64] = p1;
}

// the forms packed from weight tensor t (0: w1, 1: w2, 2: w3, 3: wfc) and their plane counts
__device__ inline void pa_forms(const PackAll& p, int t, uint16_t* (&f)[2], long long& planes) {
    switch (t) {
        case 0: f[0] = p.q1; f[1] = nullptr; planes = PL_Q1; break;
        case 1: f[0] = p.q2; f[1] = p.qd2; planes = PL_Q2; break;
        case 2: f[0] = p.q3; f[1] = p.qd3; planes = PL_Q3; break;
        case 3: f[0] = p.qfcf; f[1] = p.qfcd; planes = PL_FCF; break;
        default: f[0] = p.qhf; f[1] = p.qhd; planes = PL_H; break;
    }
}
constexpr int PA_TENSORS = 5;

// The H1P exponent of conv1's output (one workgroup): |h1| <= 255 max_c (sum_k |W1[c][k]|) +
// |b1[c]| for uint8 frames; thread t sums k-range t & 7 of channel t >> 3 in f64.  Stored in
// slot H1P_EXP_SLOT of q1's tail, read by the conv1 forward (output scale) and the H1P consumers.
// The bound carries a 2^-10 margin, so every value times 2^E stays below 2^15 (f16 max 65504).
__device__ void h1p_exp_block(const float* __restrict__ w1, const float* __restrict__ b1, uint16_t* __restrict__ q1) {
    const int t = threadIdx.x, c = t >> 3, part = t & 7;
    double sum = 0.0;
    for (int k = part * 32; k < part * 32 + 32; ++k) sum += fabs((double)w1[c * G1::K + k]);
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) sum += __shfl_xor(sum, o);
    double bound = 255.0 * sum + fabs((double)b1[c]);
#pragma unroll
    for (int o = 8; o < 64; o <<= 1) bound = fmax(bound, __shfl_xor(bound, o));
    __shared__ double red[4];
    if ((t & 63) == 0) red[t >> 6] = bound;
    __syncthreads();
    if (t == 0) {
        const double m = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
        const float mf = (float)(m * (1.0 + 1.0 / 1024.0));
        pack_tail(q1, PL_Q1)[AMAX_SLOTS + H1P_EXP_SLOT] = (uint32_t)split_scale_exp(__float_as_uint(mf));
    }
}

// The PX output bounds (round 4): column l1-norms sum_k |B[k][n]| of a packed form's matrix, their
// maximum as AMAX_SLOTS partials in the form's tail (NORM_SLOT0; every slot written) and the bias
// bound max |b| (BMAX_SLOT; NaN without a bias, so a PX output bounded without it comes out NaN).
// Job 0: q2 (conv2 forward, n = co: W2[co][:], 512 contiguous), job 1: q3 (conv3 forward, 576),
// job 2: qfcd (fc dgrad, n = a feature q: W[:][q] over the 512 outputs, 16 features per workgroup),
// job 3: qd3 (conv3 dgrad, n = ci: W3[:][ci][:][:] over the 576 (co, ky, kx); no bias: bound 0 — the PX
// g2 of round 5).  Fixed summation orders (f32; the bound's 2^-10 margin covers their rounding):
// deterministic.
constexpr int PA_NORM_JOBS = 4;
__device__ void norm_block(const PackAll& p, int job, int b) {
    __shared__ float red[256];
    const int t = threadIdx.x;
    float colmax = 0.f;
    if (job == 3) {
        if (!p.qd3) return;
        float sum = 0.f;
        if (b < 64) {  // input channel b: threads stride its 576 (co, tap) weights
            for (int k = t; k < G3::K; k += 256) sum += fabsf(p.w3[((k / 9) * 64 + b) * 9 + k % 9]);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
        if ((t & 63) == 0) red[t >> 6] = sum;
        __syncthreads();
        if (t == 0) {
            uint32_t* tail = pack_tail(p.qd3, PL_Q3);
            tail[NORM_SLOT0 + b] = __float_as_uint((red[0] + red[1]) + (red[2] + red[3]));
            if (b == 0) tail[AMAX_SLOTS + BMAX_SLOT] = 0u;
        }
        return;
    }
    if (job < 2) {
        uint16_t* q = job == 0 ? p.q2 : p.q3;
        if (!q) return;
        const float* w = job == 0 ? p.w2 : p.w3;
        const int K = job == 0 ? G2::K : G3::K;
        const float* bias = job == 0 ? p.b2 : p.b3;
        float sum = 0.f;
        if (b < 64) {  // output channel b (COUT = 64): threads stride its K weights
            for (int k = t; k < K; k += 256) sum += fabsf(w[b * K + k]);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);  // a fixed butterfly: deterministic
        if ((t & 63) == 0) red[t >> 6] = sum;
        __syncthreads();
        if (t == 0) {
            const float tot = (red[0] + red[1]) + (red[2] + red[3]);
            uint32_t* tail = pack_tail(q, job == 0 ? PL_Q2 : PL_Q3);
            tail[NORM_SLOT0 + b] = __float_as_uint(tot);
            if (b == 0) {
                float bm = bias ? 0.f : __builtin_nanf("");
                if (bias)
                    for (int i = 0; i < 64; ++i) bm = fmaxf(bm, fabsf(bias[i]));
                tail[AMAX_SLOTS + BMAX_SLOT] = __float_as_uint(bm);
            }
        }
        return;
    }
    if (!p.qfcd) return;
    // features 16 b .. 16 b + 15 (b < 196): thread (part = t >> 4, f = t & 15) sums outputs 32 part ..
    const int f = 16 * b + (t & 15), part = t >> 4;
    float sum = 0.f;
    if (f < 3136) {
#pragma unroll 8
        for (int k = 32 * part; k < 32 * part + 32; ++k) sum += fabsf(p.wfc[(long long)k * 3136 + f]);
    }
    red[t] = sum;
    __syncthreads();
    if (t < 16) {
        float tot = 0.f;
        for (int i = 0; i < 16; ++i) tot += red[16 * i + t];
        colmax = tot;
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) colmax = fmaxf(colmax, __shfl_xor(colmax, o, 16));
        if (t == 0) {
            uint32_t* tail = pack_tail(p.qfcd, PL_FCD);
            tail[NORM_SLOT0 + b] = __float_as_uint(colmax);
            if (b == 0) tail[AMAX_SLOTS + BMAX_SLOT] = 0u;  // the dgrad has no bias
        }
    }
}

// AMAX_SLOTS workgroups per weight tensor: workgroup b's max |w| over its stride into slot b of
// the tails of both forms (every slot written: no zeroing), so the packer's amax_read sees the
// tensor's max.  Then AMAX_SLOTS workgroups per PX norm job, one workgroup for the H1P exponent
// (with q1 and b1), then the workgroups zeroing p.zero (the next pass's amax table: no fill launch
// of its own)
// The packing's auxiliary workgroups (nb = 0, 1, ...): the PX norm jobs, the H1P exponent, the zeroing of p.zero
// (1,024 words per workgroup) and of p.amax_next, and — with p.amax_in — one workgroup per tensor copying the
// given amax partials into the tails of its forms (where the amax pass would have written them)
constexpr int PA_NEXT_WORDS = PA_TENSORS * AMAX_SLOTS, PA_NEXT_BLOCKS = (PA_NEXT_WORDS + 1023) / 1024;
static_assert(PA_NEXT_WORDS % 4 == 0, "amax_next: whole uint4 stores");
inline long long pack_aux_blocks(const PackAll& p) {
    return PA_NORM_JOBS * AMAX_SLOTS + 1 + ppox::ceil_div(p.zero_words, 1024LL) + (p.amax_next ? PA_NEXT_BLOCKS : 0) +
           (p.amax_in ? PA_TENSORS : 0);
}
__device__ void pack_aux_block(const PackAll& p, long long nb) {
    if (nb < PA_NORM_JOBS * AMAX_SLOTS) {
        norm_block(p, (int)(nb / AMAX_SLOTS), (int)(nb % AMAX_SLOTS));
        return;
    }
    nb -= PA_NORM_JOBS * AMAX_SLOTS;
    if (nb == 0) {
        if (p.q1 && p.b1) h1p_exp_block(p.w1, p.b1, p.q1);
        return;
    }
    nb -= 1;
    const long long zblocks = (p.zero_words + 1023) / 1024;
    if (nb < zblocks) {
        const long long i = (nb * 256 + threadIdx.x) * 4;  // this thread's four words
        if (i + 4 <= p.zero_words) {
            *reinterpret_cast<uint4*>(p.zero + i) = make_uint4(0u, 0u, 0u, 0u);
        } else {
            for (long long k = i; k < p.zero_words; ++k) p.zero[k] = 0u;  // a ragged tail
        }
        return;
    }
    nb -= zblocks;
    if (p.amax_next) {
        if (nb < PA_NEXT_BLOCKS) {
            const long long i = nb * 256 + threadIdx.x;
            if (4 * i < PA_NEXT_WORDS) reinterpret_cast<uint4*>(p.amax_next)[i] = make_uint4(0u, 0u, 0u, 0u);
            return;
        }
        nb -= PA_NEXT_BLOCKS;
    }
    if (p.amax_in && nb < PA_TENSORS) {
        uint16_t* f[2];
        long long planes;
        pa_forms(p, (int)nb, f, planes);
        const uint32_t v = p.amax_in[nb * AMAX_SLOTS + threadIdx.x];
        for (int k = 0; k < 2; ++k)
            if (f[k]) pack_tail(f[k], planes)[threadIdx.x] = v;
    }
}

__global__ void __launch_bounds__(256) wmax_kernel(PackAll p) {
    if (blockIdx.x >= PA_TENSORS * AMAX_SLOTS) {
        pack_aux_block(p, (long long)blockIdx.x - PA_TENSORS * AMAX_SLOTS);
        return;
    }
    const int t = blockIdx.x / AMAX_SLOTS, b = blockIdx.x % AMAX_SLOTS;
    uint16_t* f[2];
    long long planes;
    pa_forms(p, t, f, planes);
    if (!f[0] && !f[1]) return;
    const float4* w = reinterpret_cast<const float4*>(t == 0 ? p.w1 : t == 1 ? p.w2 : t == 2 ? p.w3 : t == 3 ? p.wfc : p.wh);
    const long long n4 =
        (t == 0 ? (long long)G1::K * G1::COUT : t == 1 ? PA_N2 : t == 2 ? PA_N3 : t == 3 ? 512LL * 3136 : PA_NH) / 4;
    float m = 0.f;
#pragma unroll 8
    for (long long i = (long long)b * 256 + threadIdx.x; i < n4; i += AMAX_SLOTS * 256) {  // (loads issue 8 at a time)
        const float4 v = w[i];
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    __shared__ uint32_t red[4];
    const uint32_t wm = wave_max_u32(__float_as_uint(m));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = wm;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t v = max(max(red[0], red[1]), max(red[2], red[3]));
        for (int k = 0; k < 2; ++k)
            if (f[k]) pack_tail(f[k], planes)[b] = v;
    }
}

__device__ uint32_t kZeroTail[AMAX_SLOTS] = {};  // the amax partials of a tensor packed into no form

// npack: the packing workgroups; with p.amax_in the auxiliary ones follow them (the amax pass's, in this launch)
__global__ void __launch_bounds__(256) pack_all_kernel(PackAll p, long long total, unsigned npack) {
    if (blockIdx.x >= npack) {
        pack_aux_block(p, (long long)(blockIdx.x - npack));
        return;
    }
    // the tensors' scales (wave-uniform), from the partials of their first packed form (or the given ones); the
    // five reads are unconditional (a tensor with no form reads zeros), so they are one round trip
    float sc[PA_TENSORS];
    uint32_t am[PA_TENSORS];
#pragma unroll
    for (int t = 0; t < PA_TENSORS; ++t) {  // all five loads before the exponent stores below
        uint16_t* f[2];
        long long planes;
        pa_forms(p, t, f, planes);
        uint16_t* src = f[0] ? f[0] : f[1];
        am[t] = amax_read(!src ? kZeroTail : p.amax_in ? p.amax_in + t * AMAX_SLOTS : pack_tail(src, planes));
    }
#pragma unroll
    for (int t = 0; t < PA_TENSORS; ++t) {
        uint16_t* f[2];
        long long planes;
        pa_forms(p, t, f, planes);
        const int e = (f[0] || f[1]) ? split_scale_exp(am[t]) : 0;
        sc[t] = exp2i(e);
        if (blockIdx.x == 0 && threadIdx.x == 0)
            for (int k = 0; k < 2; ++k)
                if (f[k]) pack_tail(f[k], planes)[AMAX_SLOTS] = (uint32_t)e;
    }
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)npack * 256) {
        long long j = i;
        if (j < PA_N1) { if (p.q1) pack_fwd1_split_elem(p.w1, sc[0], p.q1, (int)j); continue; }
        j -= PA_N1;
        if (j < PU_2) { if (p.q2) pack_frag_unit<G2::COUT>(ConvSrc<G2, false>{p.w2}, sc[1], p.q2, j); continue; }
        j -= PU_2;
        if (j < PU_3) { if (p.q3) pack_frag_unit<G3::COUT>(ConvSrc<G3, false>{p.w3}, sc[2], p.q3, j); continue; }
        j -= PU_3;
        if (j < PU_2) { if (p.qd2) pack_frag_unit<G2::CIN>(ConvSrc<G2, true>{p.w2}, sc[1], p.qd2, j); continue; }
        j -= PU_2;
        if (j < PU_3) { if (p.qd3) pack_frag_unit<G3::CIN>(ConvSrc<G3, true>{p.w3}, sc[2], p.qd3, j); continue; }
        j -= PU_3;
        if (j < PA_N2) { if (p.wpd2) pack_dgrad_elem<G2, false>(p.w2, p.wpd2, (int)j); continue; }
        j -= PA_N2;
        if (j < PU_FC) { if (p.qfcf) pack_fc_unit<true>(p.wfc, sc[3], p.qfcf, j); continue; }
        j -= PU_FC;
        if (j < PU_FCD) { if (p.qfcd) pack_fc_unit<false>(p.wfc, sc[3], p.qfcd, j); continue; }
        j -= PU_FCD;
        if (j < PU_H) { if (p.qhf) pack_rows_unit<HeadFwd, true, false>(p.wh, sc[4], p.qhf, j); continue; }
        j -= PU_H;
        if (p.qhd) pack_rows_unit<HeadDgrad, false, false>(p.wh, sc[4], p.qhd, j);
    }
}

// Host record of the packed forms whose tail holds a finite PX bias bound: q2 / q3 packed WITH
// their bias (pack_all with b2 / b3), and every fc dgrad form (no bias: its bound is 0).  A form
// packed without its bias (ppox_nature_pack_split, pack_all with a null b2 / b3) carries a NaN
// bound, so an entry point asked for a PX output (y_exp_out / g3_exp_out) refuses such a form
// instead of writing NaN activations.
std::mutex px_mu;
std::unordered_set<const void*> px_bounded;

void note_px_pack(const void* q, bool bounded) {
    if (!q) return;
    std::lock_guard<std::mutex> g(px_mu);
    if (bounded)
        px_bounded.insert(q);
    else
        px_bounded.erase(q);
}

}  // namespace

namespace ppox_conv {
bool px_bound_ok(const void* q) {
    std::lock_guard<std::mutex> g(px_mu);
    return px_bounded.count(q) != 0;
}
}  // namespace ppox_conv

namespace {
using ppox_conv::px_bound_ok;

int launch_pack_all(const PackAll& p, hipStream_t s, const char* name) {
    for (const void* q : {(const void*)p.wpd2, (const void*)p.q1, (const void*)p.q2, (const void*)p.q3,
                          (const void*)p.qd2, (const void*)p.qd3, (const void*)p.qfcf, (const void*)p.qfcd})
        PPOX_REQUIRE(!q || ppox::aligned16(q), "ppox_nature_pack: packed buffers must be 16-byte aligned");
    PPOX_REQUIRE((p.w1 || !p.q1) && (p.w2 || (!p.q2 && !p.qd2 && !p.wpd2)) && (p.w3 || (!p.q3 && !p.qd3)) &&
                     (p.wfc || (!p.qfcf && !p.qfcd)) && (p.wh || (!p.qhf && !p.qhd)),
                 "ppox_nature_pack: null weights");
    PPOX_REQUIRE((!p.qhf || ppox::aligned16(p.qhf)) && (!p.qhd || ppox::aligned16(p.qhd)),
                 "ppox_nature_pack: packed buffers must be 16-byte aligned");
    PPOX_REQUIRE(!p.zero_words || (p.zero && ppox::aligned16(p.zero)), "ppox_nature_pack_all: zero buffer");
    PPOX_REQUIRE((!p.amax_in || ppox::aligned16(p.amax_in)) && (!p.amax_next || ppox::aligned16(p.amax_next)) &&
                     (!p.amax_in || p.amax_in != p.amax_next),
                 "ppox_nature_pack_all: amax partials buffers");
    const long long aux = pack_aux_blocks(p);
    if (!p.amax_in) {  // the amax pass, then the packing
        wmax_kernel<<<(unsigned)(PA_TENSORS * AMAX_SLOTS + aux), 256, 0, s>>>(p);
        PPOX_LAUNCHED_NORET(name);
    }
    // element ranges end at the last job present (the head and fc dgrad ranges are the longest)
    const long long total = PA_N1 + 2 * PU_2 + 2 * PU_3 + PA_N2 + PU_FC +
                            (p.qhf || p.qhd ? PU_FCD + 2 * PU_H : (p.qfcd ? PU_FCD : 0));
    // every wave first reads the five tensors' 256 amax partials (5 KB): 4,096 workgroups re-read 80 MB of them
    // through L2 — a few hundred, each striding over more units, read a few MB (PPOX_PACK_BLOCKS: A/B knob)
    static const long long cap = [] {
        const char* e = ppox::ab_env("PPOX_PACK_BLOCKS");
        return e ? std::max(1LL, std::atoll(e)) : 512LL;
    }();
    const unsigned blocks = (unsigned)std::min<long long>((total + 255) / 256, cap);
    pack_all_kernel<<<blocks + (unsigned)(p.amax_in ? aux : 0), 256, 0, s>>>(p, total, blocks);
    PPOX_LAUNCHED_NORET(name);
    note_px_pack(p.q2, p.b2 != nullptr);
    note_px_pack(p.q3, p.b3 != nullptr);
    note_px_pack(p.qfcd, true);
    note_px_pack(p.qd3, true);
    return PPOX_OK;
}

}  // namespace

extern "C" int ppox_nature_pack_weights(const float* w1, const float* w2, const float* w3, float* wp1, float* wp2,
                                        float* wp3, float* wpd2, float* wpd3, void* stream) {
    // any packed buffer may be null: that packing is skipped (ops running in split math)
    PPOX_REQUIRE(w1 && w2 && w3, "ppox_nature_pack_weights: null weights");
    PPOX_REQUIRE((!wp1 || ppox::aligned16(wp1)) && (!wp2 || ppox::aligned16(wp2)) && (!wp3 || ppox::aligned16(wp3)) &&
                     (!wpd2 || ppox::aligned16(wpd2)) && (!wpd3 || ppox::aligned16(wpd3)),
                 "ppox_nature_pack_weights: packed buffers must be 16-byte aligned");
    hipStream_t s = ppox::as_stream(stream);
    if (wp1) pack_fwd<G1, false, true><<<ppox::ceil_div(G1::K * 32, 256), 256, 0, s>>>(w1, wp1);
    if (wp2) pack_fwd<G2, true, false><<<ppox::ceil_div(G2::K * 64, 256), 256, 0, s>>>(w2, wp2);
    if (wp3) pack_fwd<G3, true, false><<<ppox::ceil_div(G3::K * 64, 256), 256, 0, s>>>(w3, wp3);
    if (wpd2) pack_dgrad<G2, false><<<ppox::ceil_div(G2::K * G2::COUT, 256), 256, 0, s>>>(w2, wpd2);
    if (wpd3) pack_dgrad<G3, false><<<ppox::ceil_div(G3::K * G3::COUT, 256), 256, 0, s>>>(w3, wpd3);
    PPOX_LAUNCHED("ppox_nature_pack_weights");
}

extern "C" int ppox_nature_conv_fwd(int32_t layer, const void* x, int64_t batch, const int64_t* idx, int64_t T,
                                    int64_t N_env, int64_t x_sample_stride, const float* wp, const float* bias,
                                    float* y, void* stream) {
    if (batch == 0) return PPOX_OK;  // empty shard / minibatch: no pointers to check
    PPOX_REQUIRE(layer >= 1 && layer <= 3, "ppox_nature_conv_fwd: layer must be 1, 2 or 3");
    PPOX_REQUIRE(x && wp && bias && y && batch >= 0, "ppox_nature_conv_fwd: bad arguments");
    PPOX_REQUIRE(ppox::aligned16(wp), "ppox_nature_conv_fwd: packed weights must be 16-byte aligned");
    PPOX_REQUIRE(batch * G1::P < (1LL << 31), "ppox_nature_conv_fwd: batch too large for 32-bit row indexing");
    Args a{x, reinterpret_cast<const long long*>(idx), T, N_env, x_sample_stride, wp, bias, nullptr, y, batch};
    hipStream_t s = ppox::as_stream(stream);
    if (layer == 1) {
        PPOX_REQUIRE(!(reinterpret_cast<uintptr_t>(x) & 3) && (idx || x_sample_stride % 4 == 0),
                     "ppox_nature_conv_fwd: u8 input must be 4-byte aligned");
        if (idx) PPOX_REQUIRE(T > 0 && N_env > 0, "ppox_nature_conv_fwd: idx needs T and N_env");
        using R1 = RgFwd1<RG_FWD1_MT>;
        return launch_rgemm<R1>(a, ppox::ceil_div(batch * G1::P, R1::ROWS), s, "ppox_nature_conv_fwd");
    }
    PPOX_REQUIRE(ppox::aligned16(x) && !idx, "ppox_nature_conv_fwd: layer 2/3 input must be 16B-aligned NHWC");
    if (layer == 2) {
        using P2 = FwdNHWCProblem<G2, false, 1>;
        return launch_igemm<P2>(a, ppox::ceil_div(batch * G2::P, P2::BMR), s, "ppox_nature_conv_fwd");
    }
    using P3 = FwdNHWCProblem<G3, true, 1>;
    return launch_igemm<P3>(a, ppox::ceil_div(batch * G3::P, P3::BMR), s, "ppox_nature_conv_fwd");
}

extern "C" int ppox_nature_conv_dgrad(int32_t layer, const float* grad_out, int64_t batch, const float* wpd,
                                      const float* prev_act, float* grad_in, void* stream) {
    if (batch == 0) return PPOX_OK;  // empty shard / minibatch: no pointers to check
    PPOX_REQUIRE(layer == 2 || layer == 3, "ppox_nature_conv_dgrad: layer must be 2 or 3");
    PPOX_REQUIRE(grad_out && wpd && prev_act && grad_in && batch >= 0, "ppox_nature_conv_dgrad: bad arguments");
    PPOX_REQUIRE(ppox::aligned16(grad_out) && ppox::aligned16(wpd), "ppox_nature_conv_dgrad: 16B alignment");
    Args a{grad_out, nullptr, 0, 0, 0, wpd, nullptr, prev_act, grad_in, batch};
    hipStream_t s = ppox::as_stream(stream);
    if (layer == 2) {
        using D2 = DgradPMProblem<G2, 1>;
        return launch_igemm<D2>(a, ppox::ceil_div(batch, D2::BMR) * D2::NPOS, s, "ppox_nature_conv_dgrad");
    }
    using D3 = DgradPMProblem<G3, 1>;
    return launch_igemm<D3>(a, ppox::ceil_div(batch, D3::BMR) * D3::NPOS, s, "ppox_nature_conv_dgrad");
}

// split-K factor over pixels: ~4096 pixels per split, but enough splits that the
// grid (splits x k-blocks) fills the chip (>= ~1536 workgroups, 2 rounds of the
// ~768 resident slots) at small per-rank batches; at least 4 steps per split
extern "C" int64_t ppox_nature_wgrad_splits(int32_t layer, int64_t batch) {
    const long long P = layer == 1 ? G1::P : (layer == 2 ? G2::P : G3::P);
    const long long kb = layer == 1 ? WgCfg<G1, true>::KB : (layer == 2 ? WgCfg<G2, false>::KB : WgCfg<G3, false>::KB);
    const long long px = batch * P;
    long long s = (px + 4095) / 4096;
    const long long fill = (1536 + kb - 1) / kb, most = px / (4 * MS);
    if (s < fill) s = fill < most ? fill : most;
    s = s < 8 ? 8 : (s > 512 ? 512 : s);
    return (s + 7) / 8 * 8;
}

extern "C" int64_t ppox_nature_wgrad_workspace_bytes(int32_t layer, int64_t batch) {
    const long long splits = ppox_nature_wgrad_splits(layer, batch);
    const long long kc = layer == 1 ? G1::K * G1::COUT : (layer == 2 ? G2::K * G2::COUT : G3::K * G3::COUT);
    const long long c = layer == 1 ? G1::COUT : 64;
    return splits * (kc + c) * (long long)sizeof(float);
}

extern "C" int ppox_nature_conv_wgrad(int32_t layer, const void* x, int64_t batch, const int64_t* idx, int64_t T,
                                      int64_t N_env, int64_t x_sample_stride, const float* grad_out, void* workspace,
                                      int64_t workspace_bytes, void* stream) {
    PPOX_REQUIRE(layer >= 1 && layer <= 3, "ppox_nature_conv_wgrad: layer must be 1, 2 or 3");
    PPOX_REQUIRE(x && grad_out && workspace && batch > 0, "ppox_nature_conv_wgrad: bad arguments");
    PPOX_REQUIRE(workspace_bytes >= ppox_nature_wgrad_workspace_bytes(layer, batch),
                 "ppox_nature_conv_wgrad: workspace too small");
    PPOX_REQUIRE(ppox::aligned16(grad_out), "ppox_nature_conv_wgrad: grad_out must be 16B aligned");
    const int splits = (int)ppox_nature_wgrad_splits(layer, batch);
    const long long kc = layer == 1 ? G1::K * G1::COUT : (layer == 2 ? G2::K * G2::COUT : G3::K * G3::COUT);
    float* slab = reinterpret_cast<float*>(workspace);
    WArgs wa{x, x_sample_stride, grad_out, slab, slab + (long long)splits * kc, batch, 0, splits};
    hipStream_t s = ppox::as_stream(stream);
    PPOX_REQUIRE(!idx, "ppox_nature_conv_wgrad: gathered (idx) input not supported; gather first");
    PPOX_REQUIRE(batch * (layer == 1 ? G1::P : layer == 2 ? G2::P : G3::P) < (1LL << 31) / 64,
                 "ppox_nature_conv_wgrad: batch too large for 32-bit pixel indexing");
    if (layer == 1) {
        PPOX_REQUIRE(!(reinterpret_cast<uintptr_t>(x) & 3) && x_sample_stride % 4 == 0,
                     "ppox_nature_conv_wgrad: u8 input 4-byte aligned");
        return launch_wgrad<G1, true>(wa, s);
    }
    PPOX_REQUIRE(ppox::aligned16(x) && !idx, "ppox_nature_conv_wgrad: layer 2/3 input must be 16B-aligned NHWC");
    if (layer == 2) return launch_wgrad<G2, false>(wa, s);
    return launch_wgrad<G3, false>(wa, s);
}

extern "C" int ppox_nature_wgrad_reduce(int32_t layer, int64_t batch, const void* workspace, float* dw, float* db,
                                        void* stream) {
    PPOX_REQUIRE(layer >= 1 && layer <= 3, "ppox_nature_wgrad_reduce: layer must be 1, 2 or 3");
    PPOX_REQUIRE(workspace && dw && db && batch > 0, "ppox_nature_wgrad_reduce: bad arguments");
    const int splits = (int)ppox_nature_wgrad_splits(layer, batch);
    const long long kc = layer == 1 ? G1::K * G1::COUT : (layer == 2 ? G2::K * G2::COUT : G3::K * G3::COUT);
    const float* slab = reinterpret_cast<const float*>(workspace);
    const float* bslab = slab + (long long)splits * kc;
    hipStream_t s = ppox::as_stream(stream);
    if (layer == 1) return launch_wgrad_reduce<G1, false>(slab, bslab, splits, dw, db, s);
    if (layer == 2) return launch_wgrad_reduce<G2, true>(slab, bslab, splits, dw, db, s);
    return launch_wgrad_reduce<G3, true>(slab, bslab, splits, dw, db, s);
}


namespace {
bool wgrad1_im2col();
void w2p_grid(long long batch, int& per, long long& grid, int min_per = 1);
int w2p_min_per();
int launch_wgrad1_frames(const void* x, long long sample_stride, const long long* idx, long long T, long long Nenv,
                         const float* g, long long batch, void* ws, long long ws_bytes, float* dw, float* db,
                         const uint32_t* amax_g, hipStream_t s);
}  // namespace

extern "C" int64_t ppox_nature_wgrad_split_workspace_bytes(int32_t layer, int64_t batch) {
    if (batch <= 0) return 0;
    if (layer == 1 && !wgrad1_im2col()) {
        // the direct conv1 weight gradient: two partial slabs per workgroup, one workgroup per CU
        // (grid = min(batch, CUs): more than Ws1's 512-slab floor on a device with > 256 CUs)
        int per;
        long long grid;
        w2p_grid(batch, per, grid);
        return std::max(Ws1::workspace_bytes(batch), 2 * grid * (long long)(G1::K * G1::COUT + G1::COUT) * 4);
    }
    if (layer == 3)  // the im2col split form's slabs, or the direct form's (one per workgroup, PX operands)
        return std::max(Ws3::workspace_bytes(batch),
                        ppox_conv::dwgrad3_grid(batch) * (long long)(G3::K * G3::COUT + G3::COUT) * 4);
    return layer == 1 ? Ws1::workspace_bytes(batch) : layer == 2 ? Ws2::workspace_bytes(batch) : -1;
}

extern "C" int ppox_nature_conv_wgrad_split(int32_t layer, const void* x, int64_t batch, int64_t x_sample_stride,
                                            const float* grad_out, void* workspace, int64_t workspace_bytes, float* dw,
                                            float* db, const uint32_t* amax_x, const uint32_t* amax_g,
                                            const int* x_exp, const int* g_exp, void* stream) {
    PPOX_REQUIRE(layer >= 1 && layer <= 3, "ppox_nature_conv_wgrad_split: layer must be 1, 2 or 3");
    PPOX_REQUIRE(x && grad_out && workspace && dw && db && batch > 0, "ppox_nature_conv_wgrad_split: bad arguments");
    PPOX_REQUIRE((!x_exp && !g_exp) || layer == 3, "ppox_nature_conv_wgrad_split: PX operands are layer 3's (h2, g3)");
    PPOX_REQUIRE((amax_g || g_exp) && (layer == 1 || amax_x || x_exp) && (!amax_g || ppox::aligned16(amax_g)) &&
                     (!amax_x || ppox::aligned16(amax_x)),
                 "ppox_nature_conv_wgrad_split: amax slots of the operands (16B-aligned) required");
    PPOX_REQUIRE(workspace_bytes >= ppox_nature_wgrad_split_workspace_bytes(layer, batch),
                 "ppox_nature_conv_wgrad_split: workspace too small");
    PPOX_REQUIRE(ppox::aligned16(grad_out), "ppox_nature_conv_wgrad_split: grad_out must be 16B aligned");
    PPOX_REQUIRE((layer == 1 && !wgrad1_im2col()) ||
                     batch * (layer == 1 ? G1::P : layer == 2 ? G2::P : G3::P) < (1LL << 31) / 64,
                 "ppox_nature_conv_wgrad_split: batch too large for 32-bit pixel indexing");
    hipStream_t s = ppox::as_stream(stream);
    if (layer == 1) {
        PPOX_REQUIRE(!(reinterpret_cast<uintptr_t>(x) & 3) && x_sample_stride % 4 == 0,
                     "ppox_nature_conv_wgrad_split: u8 input 4-byte aligned");
        if (!wgrad1_im2col())
            return launch_wgrad1_frames(x, x_sample_stride, nullptr, 0, 0, grad_out, batch, workspace, workspace_bytes,
                                        dw, db, amax_g, s);
        return Ws1::run(x, x_sample_stride, grad_out, batch, workspace, dw, db, nullptr, amax_g, s);
    }
    PPOX_REQUIRE(ppox::aligned16(x), "ppox_nature_conv_wgrad_split: layer 2/3 input must be 16B-aligned NHWC");
    if (layer == 2) return Ws2::run(x, 0, grad_out, batch, workspace, dw, db, amax_x, amax_g, s);
    if (x_exp && g_exp && ppox_conv::dwgrad3_enabled(batch)) {  // the direct form (dconv.hip)
        float* slab = reinterpret_cast<float*>(workspace);
        float* bslab = slab + ppox_conv::dwgrad3_grid(batch) * (G3::K * G3::COUT);
        const int rc = ppox_conv::dwgrad3(x, grad_out, batch, x_exp, g_exp, slab, bslab, s);
        if (rc != PPOX_OK) return rc;
        return launch_wgrad_reduce<G3, true>(slab, bslab, (int)ppox_conv::dwgrad3_grid(batch), dw, db, s);
    }
    if (x_exp && g_exp) return Ws3PP::run(x, 0, grad_out, batch, workspace, dw, db, amax_x, amax_g, s, nullptr, 0, 0, x_exp, g_exp);
    if (x_exp) return Ws3PF::run(x, 0, grad_out, batch, workspace, dw, db, amax_x, amax_g, s, nullptr, 0, 0, x_exp, g_exp);
    if (g_exp) return Ws3FP::run(x, 0, grad_out, batch, workspace, dw, db, amax_x, amax_g, s, nullptr, 0, 0, x_exp, g_exp);
    return Ws3::run(x, 0, grad_out, batch, workspace, dw, db, amax_x, amax_g, s);
}

// conv1 split wgrad reading its frames straight from the rollout (sample n = env-major row
// idx[n] of the step-major (T, N_env, 4, 84, 84) buffer): the minibatch gather fused, as in
// ppox_nature_conv_fwd_split's idx form (replaces ppox_gather_rows + the strided call)
extern "C" int ppox_nature_conv_wgrad_split_idx(int32_t layer, const void* x, int64_t batch, const int64_t* idx,
                                                int64_t T, int64_t N_env, const float* grad_out, void* workspace,
                                                int64_t workspace_bytes, float* dw, float* db, const uint32_t* amax_g,
                                                void* stream) {
    PPOX_REQUIRE(layer == 1, "ppox_nature_conv_wgrad_split_idx: layer must be 1 (u8 frames)");
    PPOX_REQUIRE(x && idx && grad_out && workspace && dw && db && batch > 0 && T > 0 && N_env > 0,
                 "ppox_nature_conv_wgrad_split_idx: bad arguments");
    PPOX_REQUIRE(amax_g && ppox::aligned16(amax_g), "ppox_nature_conv_wgrad_split_idx: amax slots of G required");
    PPOX_REQUIRE(workspace_bytes >= ppox_nature_wgrad_split_workspace_bytes(layer, batch),
                 "ppox_nature_conv_wgrad_split_idx: workspace too small");
    PPOX_REQUIRE(ppox::aligned16(grad_out) && !(reinterpret_cast<uintptr_t>(x) & 3),
                 "ppox_nature_conv_wgrad_split_idx: alignment");
    if (!wgrad1_im2col())  // (the direct form indexes in 64 bits)
        return launch_wgrad1_frames(x, 0, reinterpret_cast<const long long*>(idx), T, N_env, grad_out, batch, workspace,
                                    workspace_bytes, dw, db, amax_g, ppox::as_stream(stream));
    PPOX_REQUIRE(batch * G1::P < (1LL << 31) / 64, "ppox_nature_conv_wgrad_split_idx: batch too large");
    return Ws1::run(x, 0, grad_out, batch, workspace, dw, db, nullptr, amax_g, ppox::as_stream(stream),
                    reinterpret_cast<const long long*>(idx), T, N_env);
}

extern "C" int ppox_nchw_to_nhwc_relu_grad(const float* grad, const float* act, int64_t batch, float* out,
                                           void* stream) {
    if (batch == 0) return PPOX_OK;  // empty shard / minibatch: no pointers to check
    PPOX_REQUIRE(grad && act && out && batch >= 0, "ppox_nchw_to_nhwc_relu_grad: bad arguments");
    nchw_to_nhwc_mask<<<(unsigned)batch, 256, 0, ppox::as_stream(stream)>>>(grad, act, batch, out);
    PPOX_LAUNCHED("ppox_nchw_to_nhwc_relu_grad");
}

namespace ppox_conv {
// split-f16 packing of the conv weights (called from conv_split.hip's entry point)
int pack_split(const float* w1, const float* w2, const float* w3, uint16_t* q1, uint16_t* q2, uint16_t* q3,
               uint16_t* qd2, uint16_t* qd3, hipStream_t s) {
    return launch_pack_all(PackAll{w1, w2, w3, nullptr, nullptr, q1, q2, q3, qd2, qd3, nullptr, nullptr}, s,
                           "ppox_nature_pack_split");
}

long long planes(int which) {
    switch (which) {
        case 1: return PL_Q1;
        case 2: case 12: return PL_Q2;
        case 3: case 13: return PL_Q3;
        case 4: return PL_FCF;
        default: return -1;
    }
}

int split_fwd23(int32_t layer, const void* x, int64_t batch, const uint16_t* wq, const float* bias, float* y,
                const uint32_t* amax_x, uint32_t* amax_y, uint32_t* relu_bits, const int* x_exp, int* y_exp_out,
                hipStream_t s) {
    PPOX_REQUIRE(ppox::aligned16(x), "ppox_nature_conv_fwd_split: layer 2/3 input must be 16B-aligned NHWC");
    // amax_x: the split of an f32 x and the bound of a PX output
    PPOX_REQUIRE((amax_x || (x_exp && !y_exp_out)) && (!amax_x || ppox::aligned16(amax_x)),
                 "ppox_nature_conv_fwd_split: amax slots of x required (layer 2/3)");
    PPOX_REQUIRE(!(reinterpret_cast<uintptr_t>(relu_bits) & 7), "ppox_nature_conv_fwd_split: relu_bits 8B alignment");
    PPOX_REQUIRE(!x_exp || layer == 3, "ppox_nature_conv_fwd_split: PX input (x_exp) is layer 3's (h2 planes)");
    Args a{x, nullptr, 0, 0, 0, nullptr, bias, nullptr, y, batch, amax_x, amax_y, pack_exp(wq, planes(layer))};
    a.bits_y = relu_bits;
    a.xexp = x_exp;
    a.yexp_out = y_exp_out;
    PPOX_REQUIRE(!y_exp_out || px_bound_ok(wq),
                 "ppox_nature_conv_fwd_split: a PX output needs wq packed with its bias (ppox_nature_pack_all)");
    a.ynorm = pack_norm(wq, planes(layer));
    a.ybias = pack_bmax(wq, planes(layer));
    constexpr const char* nm = "ppox_nature_conv_fwd_split";
    if (layer == 2) {
        const long long blocks = ppox::ceil_div(batch * G2::P, SG_ROWS);
        if (y_exp_out) return launch_sgemm<Px<SgFwd<G2, false>, false, true>>(a, wq, blocks, s, nm);
        return launch_sgemm<SgFwd<G2, false>>(a, wq, blocks, s, nm);
    }
    const long long blocks = ppox::ceil_div(batch * G3::P, SG_ROWS);
    if (x_exp && y_exp_out && dconv_enabled(3, batch))
        return dconv_fwd(3, x, batch, wq, bias, y, amax_x, amax_y, relu_bits, x_exp, y_exp_out, s);
    if (x_exp && y_exp_out) return launch_sgemm<Px<SgFwd<G3, false>, true, true>>(a, wq, blocks, s, nm);
    if (x_exp) return launch_sgemm<Px<SgFwd<G3, false>, true>>(a, wq, blocks, s, nm);
    if (y_exp_out) return launch_sgemm<Px<SgFwd<G3, false>, false, true>>(a, wq, blocks, s, nm);
    return launch_sgemm<SgFwd<G3, false>>(a, wq, blocks, s, nm);
}
}  // namespace ppox_conv

extern "C" int ppox_nature_conv_dgrad_split(int32_t layer, const float* grad_out, int64_t batch, const uint16_t* wqd,
                                            const float* prev_act, float* grad_in, const uint32_t* amax_g,
                                            uint32_t* amax_out, const uint32_t* relu_bits, const int* g_exp,
                                            int* y_exp_out, void* stream) {
    if (batch == 0) return PPOX_OK;  // empty shard / minibatch: no pointers to check
    PPOX_REQUIRE(layer == 2 || layer == 3, "ppox_nature_conv_dgrad_split: layer must be 2 or 3");
    PPOX_REQUIRE(grad_out && wqd && (prev_act || relu_bits) && grad_in && (amax_g || g_exp) && batch >= 0,
                 "ppox_nature_conv_dgrad_split: bad arguments");
    // relu_bits: the ReLU bitmask of the layer below (conv1's for layer 2, conv2's for layer 3)
    PPOX_REQUIRE(ppox::aligned16(grad_out) && ppox::aligned16(wqd) && (!amax_g || ppox::aligned16(amax_g)),
                 "ppox_nature_conv_dgrad_split: 16B alignment");
    Args a{grad_out, nullptr, 0, 0, 0, nullptr, nullptr, prev_act, grad_in, batch, amax_g, amax_out,
           pack_exp(wqd, ppox_conv::planes(10 + layer))};
    hipStream_t s = ppox::as_stream(stream);
    if (layer == 2 && g_exp) {  // PX g2 (the conv3 dgrad's planes output): the direct class-wise form
        PPOX_REQUIRE(relu_bits && !y_exp_out, "ppox_nature_conv_dgrad_split: a PX g2 needs conv1's ReLU bitmask "
                                              "(and writes an f32 g1)");
        return ppox_conv::ddgrad2(grad_out, batch, wqd, grad_in, relu_bits, amax_out, g_exp, a.wexp, s);
    }
    if (layer == 2) {
        PPOX_REQUIRE(!y_exp_out, "ppox_nature_conv_dgrad_split: layer 2 writes an f32 g1");
        const long long ntriples = ppox::ceil_div(batch, (long long)C2S);
        // one workgroup per CU (150 KB of LDS each), striding over the triples
        static int cus[64] = {};
        int dev = 0;
        PPOX_REQUIRE(hipGetDevice(&dev) == hipSuccess && dev < 64, "ppox_nature_conv_dgrad_split: no device");
        if (cus[dev] == 0)
            PPOX_REQUIRE(hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
                             cus[dev] > 0,
                         "ppox_nature_conv_dgrad_split: CU count");
        const long long grid = std::min<long long>(ntriples, cus[dev]);
        a.bits_mask = relu_bits;
        // PPOX_COLP_VMCNT0=1: every counted wait of the kernel as vmcnt(0) (the same result, bitwise)
        const char* safe_env = ppox::ab_env("PPOX_COLP_VMCNT0");
        const bool safe = safe_env && safe_env[0] == '1';
        const u32x4* wqv = reinterpret_cast<const u32x4*>(wqd);
        if (relu_bits && !safe)
            dgrad2_colp_kernel<true><<<(unsigned)grid, 512, 0, s>>>(a, wqv, ntriples);
        else if (relu_bits)
            dgrad2_colp_kernel<true, true><<<(unsigned)grid, 512, 0, s>>>(a, wqv, ntriples);
        else if (!safe)
            dgrad2_colp_kernel<false><<<(unsigned)grid, 512, 0, s>>>(a, wqv, ntriples);
        else
            dgrad2_colp_kernel<false, true><<<(unsigned)grid, 512, 0, s>>>(a, wqv, ntriples);
        PPOX_LAUNCHED("ppox_nature_conv_dgrad_split");
    }
    a.bits_mask = relu_bits;
    a.xexp = g_exp;  // PX g3 (the fc dgrad's planes output)
    PPOX_REQUIRE(!g_exp || relu_bits, "ppox_nature_conv_dgrad_split: a PX g3 needs conv2's ReLU bitmask");
    if (y_exp_out) {  // PX g2, bounded by amax(g3) x the dgrad matrix's column norms (no bias)
        PPOX_REQUIRE(relu_bits && amax_g && ppox::aligned16(amax_g),
                     "ppox_nature_conv_dgrad_split: a PX g2 needs conv2's ReLU bitmask and g3's amax slots");
        PPOX_REQUIRE(ppox_conv::px_bound_ok(wqd),
                     "ppox_nature_conv_dgrad_split: a PX g2 needs wqd packed by ppox_nature_pack_all");
        a.yexp_out = y_exp_out;
        a.ynorm = pack_norm(wqd, PL_Q3);
        a.ybias = pack_bmax(wqd, PL_Q3);
        if (g_exp && ppox_conv::ddgrad3_enabled(batch))  // the direct form (dconv.hip)
            return ppox_conv::ddgrad3(grad_out, batch, wqd, grad_in, amax_g, amax_out, relu_bits, g_exp, a.wexp, a.ynorm,
                                      a.ybias, y_exp_out, s);
        const long long blocks = ppox::ceil_div(batch, SG_ROWS) * SgDgradPM<G3>::NPOS;
        if (g_exp) return launch_sgemm<Px<SgDgradPM<G3, true>, true, true>>(a, wqd, blocks, s, "ppox_nature_conv_dgrad_split");
        return launch_sgemm<Px<SgDgradPM<G3, true>, false, true>>(a, wqd, blocks, s, "ppox_nature_conv_dgrad_split");
    }
    if (g_exp)
        return launch_sgemm<Px<SgDgradPM<G3, true>, true>>(a, wqd, ppox::ceil_div(batch, SG_ROWS) * SgDgradPM<G3>::NPOS,
                                                           s, "ppox_nature_conv_dgrad_split");
    if (relu_bits)
        return launch_sgemm<SgDgradPM<G3, true>>(a, wqd, ppox::ceil_div(batch, SG_ROWS) * SgDgradPM<G3>::NPOS, s,
                                                 "ppox_nature_conv_dgrad_split");
    return launch_sgemm<SgDgradPM<G3>>(a, wqd, ppox::ceil_div(batch, SG_ROWS) * SgDgradPM<G3>::NPOS, s,
                                       "ppox_nature_conv_dgrad_split");
}

// ---- conv2 on H1P (conv1's output as f16 planes, conv_common.h) --------------------------
namespace {
int cu_count() {
    static int cus[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    if (cus[dev] == 0 && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus[dev] = 0;
    return cus[dev];
}
// wgrad2_planes_kernel: samples per workgroup and workgroups (one per CU, none empty); min_per > 1:
// at least that many samples per workgroup (fewer slabs for the reduce at small batches)
void w2p_grid(long long batch, int& per, long long& grid, int min_per) {
    const long long cus = std::max(1, cu_count());
    per = (int)ppox::ceil_div(batch, std::min(batch, cus));
    per = std::max(per, std::min(min_per, (int)std::min<long long>(batch, 1 << 20)));
    grid = ppox::ceil_div(batch, (long long)per);
}
// PPOX_W2P_MIN_PER (A/B knob, default 1): the conv2 weight gradient's samples-per-workgroup floor
int w2p_min_per() {
    static const int v = [] {
        const char* e = ppox::ab_env("PPOX_W2P_MIN_PER");
        return e ? std::max(1, std::atoi(e)) : 1;
    }();
    return v;
}

// the direct conv1 weight gradient (wgrad1_frames_kernel, one workgroup per CU) + its slab reduce;
// PPOX_WGRAD1_IM2COL=1 runs the im2col form (wgrad_split_kernel) instead
bool wgrad1_im2col() {
    static const int v = [] {
        const char* e = ppox::ab_env("PPOX_WGRAD1_IM2COL");
        return e && e[0] == '1' ? 1 : 0;
    }();
    return v != 0;
}
int launch_wgrad1_frames(const void* x, long long sample_stride, const long long* idx, long long T, long long Nenv,
                         const float* g, long long batch, void* ws, long long ws_bytes, float* dw, float* db,
                         const uint32_t* amax_g, hipStream_t s) {
    int per;
    long long grid;
    w2p_grid(batch, per, grid);
    PPOX_REQUIRE(2 * grid * (long long)(G1::K * G1::COUT + G1::COUT) * 4 <= ws_bytes,
                 "ppox_nature_conv_wgrad_split: workspace too small for the direct conv1 weight gradient");
    PPOX_REQUIRE(!idx || T * Nenv < (1LL << 31), "ppox_nature_conv_wgrad_split_idx: T * N_env must be < 2^31");
    float* slab = reinterpret_cast<float*>(ws);
    W1FArgs a{reinterpret_cast<const uint8_t*>(x), sample_stride, idx, T, Nenv, g, amax_g, slab,
              slab + 2 * grid * (G1::K * G1::COUT), batch, per};
    if (idx)
        wgrad1_frames_kernel<true><<<(unsigned)grid, 512, 0, s>>>(a);
    else
        wgrad1_frames_kernel<false><<<(unsigned)grid, 512, 0, s>>>(a);
    PPOX_LAUNCHED_NORET("ppox_nature_conv_wgrad_split");
    return launch_wgrad_reduce<G1, false>(slab, a.bslab, (int)(2 * grid), dw, db, s);
}
}  // namespace

extern "C" int ppox_nature_conv2_fwd_planes(const uint16_t* h1p, const uint16_t* q1, int64_t batch,
                                            const uint16_t* wq2, const float* bias, float* y, const uint32_t* amax_x,
                                            uint32_t* amax_y, uint32_t* relu_bits, int* y_exp_out, void* stream) {
    if (batch == 0) return PPOX_OK;
    PPOX_REQUIRE(h1p && q1 && wq2 && bias && y && batch > 0, "ppox_nature_conv2_fwd_planes: bad arguments");
    PPOX_REQUIRE(ppox::aligned16(h1p) && ppox::aligned16(wq2), "ppox_nature_conv2_fwd_planes: 16B alignment");
    PPOX_REQUIRE(!(reinterpret_cast<uintptr_t>(relu_bits) & 7), "ppox_nature_conv2_fwd_planes: relu_bits 8B alignment");
    PPOX_REQUIRE(!y_exp_out || (amax_x && ppox::aligned16(amax_x)),
                 "ppox_nature_conv2_fwd_planes: a PX output (y_exp_out) needs h1's amax slots (amax_x)");
    PPOX_REQUIRE(!y_exp_out || ppox_conv::px_bound_ok(wq2),
                 "ppox_nature_conv2_fwd_planes: a PX output needs wq2 packed with its bias (ppox_nature_pack_all)");
    Args a{h1p, nullptr, 0, 0, 0, nullptr, bias, nullptr, y, batch, amax_x, amax_y, pack_exp(wq2, PL_Q2)};
    a.bits_y = relu_bits;
    a.xexp = h1p_exp(q1, PL_Q1);
    a.yexp_out = y_exp_out;
    a.ynorm = pack_norm(wq2, PL_Q2);
    a.ybias = pack_bmax(wq2, PL_Q2);
    const long long blocks = ppox::ceil_div(batch * G2::P, SG_ROWS);
    if (y_exp_out && ppox_conv::dconv_enabled(2, batch))
        return ppox_conv::dconv_fwd(2, h1p, batch, wq2, bias, y, amax_x, amax_y, relu_bits, a.xexp, y_exp_out,
                                    ppox::as_stream(stream));
    if (y_exp_out)
        return launch_sgemm<Px<SgFwd2P, true, true>>(a, wq2, blocks, ppox::as_stream(stream), "ppox_nature_conv2_fwd_planes");
    return launch_sgemm<SgFwd2P>(a, wq2, blocks, ppox::as_stream(stream), "ppox_nature_conv2_fwd_planes");
}

extern "C" int64_t ppox_nature_conv2_wgrad_planes_workspace_bytes(int64_t batch) {
    if (batch <= 0) return 0;
    int per;
    long long grid;
    w2p_grid(batch, per, grid, w2p_min_per());
    return grid * (long long)(G2::K * G2::COUT + G2::COUT) * (long long)sizeof(float);
}

extern "C" int ppox_nature_conv2_wgrad_planes(const uint16_t* h1p, const uint16_t* q1, int64_t batch,
                                              const float* grad_out, void* workspace, int64_t workspace_bytes,
                                              float* dw, float* db, const uint32_t* amax_g, const int* g_exp,
                                              void* stream) {
    PPOX_REQUIRE(h1p && q1 && grad_out && workspace && dw && db && (amax_g || g_exp) && batch > 0,
                 "ppox_nature_conv2_wgrad_planes: bad arguments");
    PPOX_REQUIRE(ppox::aligned16(h1p) && ppox::aligned16(grad_out) && (!amax_g || ppox::aligned16(amax_g)) &&
                     ppox::aligned16(workspace),
                 "ppox_nature_conv2_wgrad_planes: 16B alignment");
    PPOX_REQUIRE(cu_count() > 0, "ppox_nature_conv2_wgrad_planes: no device");
    PPOX_REQUIRE(workspace_bytes >= ppox_nature_conv2_wgrad_planes_workspace_bytes(batch),
                 "ppox_nature_conv2_wgrad_planes: workspace too small");
    int per;
    long long grid;
    w2p_grid(batch, per, grid, w2p_min_per());
    float* slab = reinterpret_cast<float*>(workspace);
    W2PArgs wa{h1p, h1p_exp(q1, PL_Q1), grad_out, amax_g, nullptr, slab, slab + grid * (long long)(G2::K * G2::COUT),
               batch, per};
    wa.g_exp = g_exp;
    hipStream_t s = ppox::as_stream(stream);
    if (g_exp)
        wgrad2_planes_kernel<true><<<(unsigned)grid, 512, 0, s>>>(wa);
    else
        wgrad2_planes_kernel<false><<<(unsigned)grid, 512, 0, s>>>(wa);
    PPOX_LAUNCHED_NORET("ppox_nature_conv2_wgrad_planes");
    return launch_wgrad_reduce<G2, true>(slab, wa.bslab, (int)grid, dw, db, s);
}

// ---- NatureCNN fc layer (3136 -> 512) on the split-f16 GEMM -----------------------
// Weight gradient dW = df^T h3 on the split wgrad kernel: "pixels" = samples (GFc has one
// output pixel), K = the 512 outputs (X = df rows), G = the NHWC conv3 activations in 49
// blocks of 64 channels (one spatial position each, NHWC feature order f = p * 64 + c).
// Split-K partial slabs [split][512][3136] are summed in a fixed order by fc_wgrad_reduce,
// which writes dW in the Flatten order of the fc weight.
using GFc = Geo<512, 1, 1, 1, 1, 1, 64>;
constexpr int FCW_KT = 128, FCW_CB = 49;
template <int CB, int MAXS>
struct RowsWgrad {
    using C = WsCfg<GFc, false, FCW_KT>;
    static constexpr long long TILES = (long long)C::KB * CB;
    static constexpr long long SLAB = (long long)GFc::K * CB * GFc::COUT;  // floats per split
    // the split count whose (rounds of 512 workgroup slots) x (steps per split + 3 of fixed
    // prologue / epilogue cost) is least: 13 at B = 16384 (4.98 rounds), 5 at B = 2048 (fc)
    static int splits(long long batch) {
        int best = 1;
        long long best_cost = -1;
        for (int sp = 1; sp <= MAXS; ++sp) {
            const long long steps = ppox::ceil_div(ppox::ceil_div(batch, (long long)sp), (long long)MS);
            if (sp > 1 && steps < 2) break;
            const long long cost = ppox::ceil_div(TILES * sp, 512LL) * (steps + 3);
            if (best_cost < 0 || cost < best_cost) {
                best_cost = cost;
                best = sp;
            }
        }
        return best;
    }
    static long long workspace_bytes(long long batch) { return splits(batch) * SLAB * (long long)sizeof(float); }
};
using FcWgrad = RowsWgrad<FCW_CB, 16>;
using HeadWgrad = RowsWgrad<512 / 64, 128>;  // the heads' hidden layer: G = f in 8 column blocks

// slabs [splits][512][N] summed in split order; PERM: the fc's NHWC features -> Flatten order
template <int N, bool PERM>
__global__ void __launch_bounds__(256) rows_wgrad_reduce(const float* __restrict__ slab, int splits,
                                                         float* __restrict__ dw) {
    constexpr long long SL = 512LL * N;
    const long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;  // 4 slab elements (o, feature)
    if (i >= SL) return;
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
    for (int sp = 0; sp < splits; ++sp) {  // (unrolled: the splits' loads issue together)
        const float4 v = *reinterpret_cast<const float4*>(slab + sp * SL + i);
        t.x += v.x;
        t.y += v.y;
        t.z += v.z;
        t.w += v.w;
    }
    if constexpr (PERM) {
        const int o = (int)(i / N), f = (int)(i - (long long)o * N);  // N % 4 == 0: one row
        float* row = dw + (long long)o * N;
        row[fc_nchw_feature(f)] = t.x;
        row[fc_nchw_feature(f + 1)] = t.y;
        row[fc_nchw_feature(f + 2)] = t.z;
        row[fc_nchw_feature(f + 3)] = t.w;
    } else {  // dw may be a 4-B aligned view (a parameter's grad in the flat buffer)
        dw[i] = t.x;
        dw[i + 1] = t.y;
        dw[i + 2] = t.z;
        dw[i + 3] = t.w;
    }
}

// The fc layer's reduce: one workgroup per output row o.  The row's 3136 NHWC-ordered sums (same
// split order as rows_wgrad_reduce: bitwise the same values) are staged in LDS, then written in
// Flatten order q = c * 49 + p (NHWC f = p * 64 + c) as coalesced stores; the staging row is padded
// one float per 64 (f + (f >> 6) = 65 p + c), so the strided reads of consecutive q hit distinct banks.
// (rows_wgrad_reduce<3136, true> scattered every store across 49-float strides.)
__global__ void __launch_bounds__(256) fc_wgrad_reduce_perm(const float* __restrict__ slab, int splits,
                                                            float* __restrict__ dw) {
    constexpr int N = 3136, N4 = N / 4, UPT = (N4 + 255) / 256;
    constexpr long long SL = 512LL * N;
    static_assert(N == 49 * 64 && UPT == 4, "fc reduce shape");
    __shared__ float row[N + N / 64];
    const int o = blockIdx.x, t = threadIdx.x;
    const float* base = slab + (long long)o * N;
    float4 acc[UPT];
    int uo[UPT];
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
        acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        const int u = t + 256 * k;
        uo[k] = 4 * (u < N4 ? u : N4 - 1);  // clamped: loads unconditional, the extra unit not stored
    }
#pragma unroll 2
    for (int sp = 0; sp < splits; ++sp) {
        float4 v[UPT];
#pragma unroll
        for (int k = 0; k < UPT; ++k) v[k] = *reinterpret_cast<const float4*>(base + sp * SL + uo[k]);
#pragma unroll
        for (int k = 0; k < UPT; ++k) {
            acc[k].x += v[k].x;
            acc[k].y += v[k].y;
            acc[k].z += v[k].z;
            acc[k].w += v[k].w;
        }
    }
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
        if (t + 256 * k >= N4) break;
        const int f = uo[k], r = f + (f >> 6);  // the 4 features share one 64-block
        row[r] = acc[k].x;
        row[r + 1] = acc[k].y;
        row[r + 2] = acc[k].z;
        row[r + 3] = acc[k].w;
    }
    __syncthreads();
    float* out = dw + (long long)o * N;
    for (int q = t; q < N; q += 256) {
        const int c = q / 49, pp = q - 49 * c;
        out[q] = row[65 * pp + c];
    }
}

// ---------------------------------------------------------------------------
// fc weight gradient, direct (round 6; models-checkpoint.py:60 Linear(3136, 512) trained by ppo.py:241):
//   dW[o][f] = sum over rows r of df[r][o] h3[r][f]      (f = p * 64 + c, NHWC; stored in Flatten order by the reduce)
// on PX df and PX h3 (both operands as their two f16 planes, as the fc dgrad and forward read them).  The split
// wgrad form (wgrad_split_kernel<GFc>) tiles 128 outputs x one pixel (64 features) per workgroup, two per CU, and
// needs 13 split-K slabs at 16,384 rows to fill the chip: its L2 -> LDS staging is ~0.5 KB per MFMA and its slabs
// + reduce 84 MB each way (PMC 2.0x the algorithmic bytes).  Here one 256-thread workgroup per
// CU owns 256 outputs x 2 pixels (128 features) over a fifth of the rows: 50 tiles x 5 splits = 250 workgroups,
// 0.33 KB staged per MFMA, 5 slabs.
//   * per 16-row k-step the workgroup stages 24 sub-images of 16 rows x 32 columns f16 (1 KB each): df (8 output
//     groups x 2 planes) and h3 (2 pixels x 2 channel halves x 2 planes), each lane one 16-B piece by a register
//     load (row lane >> 2, piece lane & 3), stored to LDS as it lies (a sub-image = 1 KB contiguous, the
//     transposing read's layout of dwgrad3_kernel: lane (h, g16, qq, pp) reads rows 8 h + qq (+ 4) at column
//     32 g16 + 8 pp, conflict-free);
//   * wave w: outputs 128 (w & 1) .. + 127 of the workgroup's 256 (4 tiles) x pixel w >> 1 (2 tiles): 8 tiles,
//     hi / lo accumulator pairs (hA hB | hA lB + lA hB, as the split wgrad form), 24 MFMAs per k-step;
//   * two-deep register pipeline (step s + 2's loads fly while step s + 1 goes to the other LDS slot under step
//     s's MFMAs), one barrier per k-step; rows past the split read a zero df piece;
//   * partial slabs [split][512][3136] (NHWC features) summed in split order by fc_wgrad_reduce_perm.
constexpr int FWG_KS = 16, FWG_GROUPS = 25, FWG_SPLITS = 5;    // k-step rows; 2-pixel groups (the 25th: pixel 48)
constexpr int FWG_NA = 16, FWG_NB = 8, FWG_SUB = FWG_KS * 64;  // df / h3 sub-images per k-step; bytes each
constexpr int FWG_STAGE = (FWG_NA + FWG_NB) * FWG_SUB, FWG_NSLOT = 3;  // 24 KB per slot
constexpr int FWG_P = (FWG_NA + FWG_NB) / 4;                   // pieces per thread per k-step: 6 (4 df, 2 h3)
constexpr long long FWG_DFROW = 1024 * 2, FWG_H3ROW = 49 * 256;  // PX row bytes

struct FwgArgs {
    const uint8_t* df;  // PX df [batch][16 groups: 32 hi | 32 lo f16]
    const uint8_t* h3;  // PX h3 [batch][49 pixels: (hi | lo) x 2 channel halves]
    const int *df_exp, *h3_exp;
    float* slab;  // [splits][512][3136]
    long long batch, rows_per_split;
};
__device__ __attribute__((aligned(16))) uint8_t kFwgZero[64] = {};  // the df piece of a row past the split

// the accumulators live in AGPRs (16 f32x16 = all 256 of them; hipcc, left to place them, shuttled them between
// the register files and spilled): the MFMAs are inline asm, the fragments VGPRs.  PAD: 2 wait states before the
// MFMA (a fragment assembled by a VALU move must not be read as an MFMA source sooner; hipcc pads nothing in asm
// and may place the move anywhere before its use — every MFMA here is padded: an s_nop issues inside the previous
// MFMA's 32 cycles)
__device__ inline void fwg_zero(f32x16& c, const u32x4& z) {  // c = 0 x 0 + 0, defined in AGPRs
    // padded too: hipcc writes z (v_mov) right before the first of these (read unpadded, stale lanes made NaN)
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %1, %1, 0" : "=a"(c) : "v"(z));
}
template <bool PAD>
__device__ inline void fwg_mfma(f32x16& c, const u32x4& x, const u32x4& y) {
    static_assert(PAD, "fwg_mfma: every MFMA padded");
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(c) : "v"(x), "v"(y));
}

// wait for every outstanding LDS read of this wave; F's 24 registers named, so no use moves above the wait
template <class Frag>
__device__ inline void fwg_wait(Frag& F) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(F.b[0]), "+v"(F.b[1]), "+v"(F.b[2]), "+v"(F.b[3]), "+v"(F.b[4]), "+v"(F.b[5]), "+v"(F.b[6]),
                   "+v"(F.b[7]));
    asm volatile("" : "+v"(F.a0[0]), "+v"(F.a0[1]), "+v"(F.a0[2]), "+v"(F.a0[3]), "+v"(F.a0[4]), "+v"(F.a0[5]),
                      "+v"(F.a0[6]), "+v"(F.a0[7]));
    asm volatile("" : "+v"(F.a1[0]), "+v"(F.a1[1]), "+v"(F.a1[2]), "+v"(F.a1[3]), "+v"(F.a1[4]), "+v"(F.a1[5]),
                      "+v"(F.a1[6]), "+v"(F.a1[7]));
}

template <class Fn, int... I>
__device__ inline void fwg_unroll(Fn&& fn, std::integer_sequence<int, I...>) {
    (fn(std::integral_constant<int, I>{}), ...);
}
// the transposing fragment read at a compile-time offset (one base address per operand; asm so the offsets fold
// into the instruction: the compiler's own form kept a 64-bit generic address per sub-image)
template <int OFF>
__device__ inline uint2 fwg_tr(uint32_t addr) {
    uint2 r;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF) : "memory");
    return r;
}
// wait until at most N of this wave's LDS reads are outstanding; x: the registers those reads fill
template <int N, int K>
__device__ inline void fwg_lgkm(uint2 (&x)[K]) {
    static_assert(K == 8, "fwg_lgkm: 8 reads");
    asm volatile("s_waitcnt lgkmcnt(%8)"
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7])
                 : "n"(N));
}

__global__ void __launch_bounds__(256, 1) fcwg_kernel(FwgArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[FWG_NSLOT * FWG_STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // item = (split, feature group, output half), the output half fastest: the workgroups of one XCD share their
    // split's df rows (and each h3 pixel pair with its other half) through its L2
    const long long w = xcd_remap(blockIdx.x, gridDim.x);
    const int oh = (int)(w & 1), fg = (int)((w >> 1) % FWG_GROUPS), split = (int)(w / (2 * FWG_GROUPS));
    const long long r0 = (long long)split * a.rows_per_split;
    const long long r1 = min(a.batch, r0 + a.rows_per_split);
    const int nsteps = r1 > r0 ? (int)((r1 - r0 + FWG_KS - 1) / FWG_KS) : 0;
    // this thread's pieces: sub-image wave + 4 i (i < 4: df output group 8 oh + ((wave + 4 i) >> 1), plane
    // (wave + 4 i) & 1; i >= 4: h3 pixel, half, plane), row lane >> 2, 16-B piece lane & 3.  Buffer loads: 32-bit
    // offsets, and a row past the split reads past the buffer's end, which returns zeros
    const int prow = lane >> 2, pc = lane & 3;
    uint32_t aoff[4], boff[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int sub = wave + 4 * i;
        aoff[i] = (uint32_t)((8 * oh + (sub >> 1)) * 128 + (sub & 1) * 64 + pc * 16);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int sub = wave + 4 * i;  // (pixel, half, plane) = (sub >> 2, (sub >> 1) & 1, sub & 1)
        const int px = min(2 * fg + (sub >> 2), 48);
        boff[i] = (uint32_t)(px * 256 + ((sub >> 1) & 1) * 128 + (sub & 1) * 64 + pc * 16);
    }
    const auto a_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(a.df + r0 * FWG_DFROW), 0,
                                                        (int)((r1 - r0) * FWG_DFROW), 0x00020000);
    const auto b_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(a.h3 + r0 * FWG_H3ROW), 0,
                                                        (int)((r1 - r0) * FWG_H3ROW), 0x00020000);
    struct Raw {
        u32x4 v[FWG_P];
    };
    auto load = [&](Raw& raw, int step) {
        const uint32_t r = (uint32_t)(step * FWG_KS + prow);  // split-relative; past the end: zeros
        const uint32_t ra = r * (uint32_t)FWG_DFROW, rb = r * (uint32_t)FWG_H3ROW;
#pragma unroll
        for (int i = 0; i < 4; ++i) raw.v[i] = __builtin_amdgcn_raw_buffer_load_b128(a_rs, (int)(ra + aoff[i]), 0, 0);
#pragma unroll
        for (int i = 0; i < 2; ++i) raw.v[4 + i] = __builtin_amdgcn_raw_buffer_load_b128(b_rs, (int)(rb + boff[i]), 0, 0);
    };
    auto store = [&](const Raw& raw, int slot) {
        uint8_t* st = lds + slot * FWG_STAGE;
#pragma unroll
        for (int i = 0; i < FWG_P; ++i) *reinterpret_cast<u32x4*>(st + (tid + 256 * i) * 16) = raw.v[i];
    };
    // fragment reads (the transposing pattern of dwgrad3_kernel on 64-B rows): wave w reads df output groups
    // 4 (w & 1) .. + 3 of the workgroup's 8 and h3 pixel w >> 1
    const int h = lane >> 5, g16 = (lane >> 4) & 1, qq = (lane >> 2) & 3, pp = lane & 3;
    const int wo = wave & 1, wp = wave >> 1;
    const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)lds);
    const uint32_t lrow = (uint32_t)((8 * h + qq) * 64 + g16 * 32 + pp * 8);
    const uint32_t abase = lds0 + lrow + (uint32_t)(wo * 8 * FWG_SUB);
    const uint32_t bbase = lds0 + lrow + (uint32_t)((FWG_NA + wp * 4) * FWG_SUB);
    f32x16 hi[4][2], lo[4][2];
    {
        const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                fwg_zero(hi[i][j], z);
                fwg_zero(lo[i][j], z);
            }
    }
    auto cat = [](uint2 x0, uint2 x1) { return u32x4{x0.x, x0.y, x1.x, x1.y}; };
    // one k-step's fragments: h3 (j, plane, row half) and df tiles 0-1, 2-3 (tile, plane, row half)
    struct Frag {
        uint2 b[8], a0[8], a1[8];
    };
    // issue the 24 transposing reads of the k-step in LDS slot `slot` (they complete under the MFMAs of the
    // previous k-step: waited for by fwg_wait at the top of the next)
    auto issue = [&](Frag& F, int slot) {
        const uint32_t so = (uint32_t)(slot * FWG_STAGE), ab = abase + so, bb = bbase + so;
        fwg_unroll([&](auto X) {  // B: (j, P, half) = (x >> 2, (x >> 1) & 1, x & 1)
            constexpr int x = decltype(X)::value;
            F.b[x] = fwg_tr<((x >> 2) * 2 + ((x >> 1) & 1)) * FWG_SUB + (x & 1) * 256>(bb);
        }, std::make_integer_sequence<int, 8>{});
        fwg_unroll([&](auto X) {  // A tiles 0-1: (i, P, half)
            constexpr int x = decltype(X)::value;
            F.a0[x] = fwg_tr<((x >> 2) * 2 + ((x >> 1) & 1)) * FWG_SUB + (x & 1) * 256>(ab);
        }, std::make_integer_sequence<int, 8>{});
        fwg_unroll([&](auto X) {  // A tiles 2-3
            constexpr int x = decltype(X)::value;
            F.a1[x] = fwg_tr<((2 + (x >> 2)) * 2 + ((x >> 1) & 1)) * FWG_SUB + (x & 1) * 256>(ab);
        }, std::make_integer_sequence<int, 8>{});
    };
    auto mma = [&](const Frag& F) {
        const u32x4 bq[2][2] = {{cat(F.b[0], F.b[1]), cat(F.b[2], F.b[3])}, {cat(F.b[4], F.b[5]), cat(F.b[6], F.b[7])}};
        auto tile = [&](int i, const uint2 (&ra)[8], int t) {
            const u32x4 a0 = cat(ra[4 * t], ra[4 * t + 1]), a1 = cat(ra[4 * t + 2], ra[4 * t + 3]);
            // hA hB into hi, hA lB + lA hB into lo (mfma_split3)
            fwg_mfma<true>(hi[i][0], a0, bq[0][0]);
            fwg_mfma<true>(lo[i][0], a0, bq[0][1]);
            fwg_mfma<true>(lo[i][0], a1, bq[0][0]);
            fwg_mfma<true>(hi[i][1], a0, bq[1][0]);
            fwg_mfma<true>(lo[i][1], a0, bq[1][1]);
            fwg_mfma<true>(lo[i][1], a1, bq[1][0]);
        };
        tile(0, F.a0, 0);
        tile(1, F.a0, 1);
        tile(2, F.a1, 0);
        tile(3, F.a1, 1);
    };
    // three LDS slots, two register stages: at the top of k-step s, step s's fragments are in flight (issued in
    // step s - 1), step s + 1 sits in slot (s + 1) % 3, raw[s & 1] holds step s + 2.  Step s: wait for its
    // fragments, issue step s + 1's, its 24 MFMAs, store step s + 2 into slot (s + 2) % 3 (= (s - 1) % 3, whose
    // reads every wave waited for in step s - 1, before the barrier that ended it), load step s + 4, barrier
    Raw raw[2];
    load(raw[0], 0);
    load(raw[1], 1);
    store(raw[0], 0);  // (past the split: zeros, which an odd count's extra step reads)
    store(raw[1], 1);
    load(raw[0], 2);
    load(raw[1], 3);
    __syncthreads();
    Frag F[2];
    issue(F[0], 0);
    int sr = 1, sw = 2;  // slots read (step s + 1) and written (step s + 2)
    auto step = [&](int s, auto cur_tag) {
        constexpr int C = decltype(cur_tag)::value;
        fwg_wait(F[C]);
        issue(F[C ^ 1], sr);
        mma(F[C]);
        store(raw[C], sw);
        load(raw[C], s + 4);
        sr = sr == 2 ? 0 : sr + 1;
        sw = sw == 2 ? 0 : sw + 1;
        __syncthreads();
    };
    // whole pairs of k-steps (a branch inside the pair merged the two register stages' load counts, and hipcc then
    // waited for every load in flight at each store): an odd count's extra step reads rows past the split, zeros
    for (int s = 0; s < nsteps; s += 2) {
        step(s, std::integral_constant<int, 0>{});
        step(s + 1, std::integral_constant<int, 1>{});
    }
    // the last issued reads (past the end) land before the workgroup exits; >= 18 wait states between the last
    // MFMA writing an accumulator and its read; the statements name every accumulator, so no read is scheduled
    // above the nops
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 4"
                 : "+a"(hi[0][0]), "+a"(hi[0][1]), "+a"(hi[1][0]), "+a"(hi[1][1]), "+a"(hi[2][0]), "+a"(hi[2][1]),
                   "+a"(hi[3][0]), "+a"(hi[3][1])
                 :
                 : "memory");
    asm volatile(""
                 : "+a"(lo[0][0]), "+a"(lo[0][1]), "+a"(lo[1][0]), "+a"(lo[1][1]), "+a"(lo[2][0]), "+a"(lo[2][1]),
                   "+a"(lo[3][0]), "+a"(lo[3][1])
                 :
                 : "memory");
    const int px = 2 * fg + wp;
    if (px > 48) return;  // the 25th group's second pixel (wave-uniform)
    const float uo = exp2i(-*a.df_exp) * exp2i(-*a.h3_exp);
    float* slab = a.slab + ((long long)split * 512 + oh * 256 + wo * 128) * 3136 + px * 64;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int o = i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                slab[(long long)o * 3136 + j * 32 + (lane & 31)] = (hi[i][j][r] + lo[i][j][r]) * uo;
            }
}

// the direct form's split count: 5 (250 workgroups), fewer for batches below ~5 k-steps per split
inline int fcwg_splits(long long batch) {
    static const int maxs = [] {  // (A/B: PPOX_FCWG_SPLITS, 1-8)
        const char* e = ppox::ab_env("PPOX_FCWG_SPLITS");
        const int v = e ? std::atoi(e) : 0;
        return v >= 1 && v <= 8 ? v : FWG_SPLITS;
    }();
    return (int)std::max<long long>(1, std::min<long long>(maxs, ppox::ceil_div(batch, 4LL * FWG_KS)));
}

extern "C" int64_t ppox_nature_fc_wgrad_workspace_bytes(int64_t batch) {
    if (batch <= 0) return 0;
    return std::max<int64_t>(FcWgrad::workspace_bytes(batch), (int64_t)fcwg_splits(batch) * FcWgrad::SLAB * 4);
}

extern "C" int ppox_nature_fc_wgrad(const float* df, int64_t batch, const float* h3, void* workspace,
                                    int64_t workspace_bytes, float* dw, const uint32_t* amax_df,
                                    const uint32_t* amax_h3, const int* h3_exp, const int* df_exp, void* stream) {
    PPOX_REQUIRE(dw && batch >= 0, "ppox_nature_fc_wgrad: bad arguments");
    hipStream_t s = ppox::as_stream(stream);
    if (batch == 0) {  // no rows: a zero gradient
        PPOX_REQUIRE(hipMemsetAsync(dw, 0, sizeof(float) * FcWgrad::SLAB, s) == hipSuccess,
                     "ppox_nature_fc_wgrad: memset failed");
        return PPOX_OK;
    }
    PPOX_REQUIRE(df && h3 && workspace && (amax_df || df_exp) && (amax_h3 || h3_exp), "ppox_nature_fc_wgrad: bad arguments");
    PPOX_REQUIRE((!amax_df || ppox::aligned16(amax_df)) && (!amax_h3 || ppox::aligned16(amax_h3)),
                 "ppox_nature_fc_wgrad: 16B alignment");
    PPOX_REQUIRE(workspace_bytes >= FcWgrad::workspace_bytes(batch), "ppox_nature_fc_wgrad: workspace too small");
    PPOX_REQUIRE(ppox::aligned16(df) && ppox::aligned16(h3), "ppox_nature_fc_wgrad: 16B alignment");
    PPOX_REQUIRE(batch < (1LL << 31) / 64, "ppox_nature_fc_wgrad: batch too large for 32-bit row indexing");
    float* slab = reinterpret_cast<float*>(workspace);
    // PX df and PX h3 (the product's training pass): the direct form (round 6; PPOX_FCWG=0 under PPOX_AB=1: the
    // split wgrad form)
    const char* fe = ppox::ab_env("PPOX_FCWG");
    if (h3_exp && df_exp && !(fe && fe[0] == '0')) {
        const int sp = fcwg_splits(batch);
        FwgArgs fa{reinterpret_cast<const uint8_t*>(df), reinterpret_cast<const uint8_t*>(h3), df_exp, h3_exp, slab,
                   batch, (long long)ppox::ceil_div((long long)batch, (long long)sp)};
        fcwg_kernel<<<(unsigned)(2 * FWG_GROUPS * sp), 256, 0, s>>>(fa);
        PPOX_LAUNCHED_NORET("ppox_nature_fc_wgrad");
        ppox::ktime_mark(s);
        fc_wgrad_reduce_perm<<<512, 256, 0, s>>>(slab, sp, dw);
        PPOX_LAUNCHED("ppox_nature_fc_wgrad");
    }
    const int sp = FcWgrad::splits(batch);
    WArgs wa{df, 0, h3, slab, nullptr, batch, 0, sp, nullptr, 0, 0, amax_df, amax_h3};
    wa.gexp = h3_exp;  // PX h3 (the G operand of this GEMM)
    wa.xexp = df_exp;  // PX df (the X operand)
    wa.px_per_split = ppox::ceil_div(ppox::ceil_div((long long)batch, (long long)sp), (long long)MS) * MS;
    const unsigned g = (unsigned)(FcWgrad::TILES * sp);
    if (h3_exp && df_exp)
        wgrad_split_kernel<GFc, false, FCW_KT, false, FCW_CB, true, true><<<g, 256, 0, s>>>(wa);
    else if (h3_exp)
        wgrad_split_kernel<GFc, false, FCW_KT, false, FCW_CB, false, true><<<g, 256, 0, s>>>(wa);
    else if (df_exp)
        wgrad_split_kernel<GFc, false, FCW_KT, false, FCW_CB, true, false><<<g, 256, 0, s>>>(wa);
    else
        wgrad_split_kernel<GFc, false, FCW_KT, false, FCW_CB><<<g, 256, 0, s>>>(wa);
    PPOX_LAUNCHED_NORET("ppox_nature_fc_wgrad");
    ppox::ktime_mark(s);
    fc_wgrad_reduce_perm<<<512, 256, 0, s>>>(slab, sp, dw);
    PPOX_LAUNCHED("ppox_nature_fc_wgrad");
}

extern "C" int64_t ppox_nature_fc_pack_elems(void) { return PL_FCF + 2 * PACK_TAIL32; }

extern "C" int ppox_nature_fc_pack(const float* w, uint16_t* q_fwd, uint16_t* q_dgrad, void* stream) {
    PPOX_REQUIRE(w && (q_fwd || q_dgrad), "ppox_nature_fc_pack: bad arguments");
    return launch_pack_all(PackAll{nullptr, nullptr, nullptr, w, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                   q_fwd, q_dgrad},
                           ppox::as_stream(stream), "ppox_nature_fc_pack");
}

extern "C" int ppox_nature_fc_fwd(const float* h3, int64_t batch, const uint16_t* q_fwd, const float* bias, float* f,
                                  const uint32_t* amax_h3, uint32_t* amax_f, const int* h3_exp, void* stream) {
    if (batch == 0) return PPOX_OK;  // empty shard / minibatch: no pointers to check
    PPOX_REQUIRE(h3 && q_fwd && bias && f && (amax_h3 || h3_exp) && batch >= 0, "ppox_nature_fc_fwd: bad arguments");
    PPOX_REQUIRE(ppox::aligned16(h3) && ppox::aligned16(q_fwd) && (!amax_h3 || ppox::aligned16(amax_h3)),
                 "ppox_nature_fc_fwd: 16B alignment");
    Args a{h3, nullptr, 0, 0, 0, nullptr, bias, nullptr, f, batch, amax_h3, amax_f, pack_exp(q_fwd, PL_FCF)};
    a.xexp = h3_exp;  // PX h3 (the conv3 forward's planes output)
    const long long blocks = ppox::ceil_div(batch, SG_ROWS) * (512 / SG_FC_NB);
    if (h3_exp && ppox_conv::fcw_enabled(batch))  // the wide-tile form (dconv.hip)
        return ppox_conv::fcw(h3, batch, q_fwd, bias, f, amax_f, h3_exp, a.wexp, ppox::as_stream(stream));
    if (h3_exp)
        return launch_sgemm<Px<SgRows<3136, 512, FC_FWD, FC_FWD_GW, false, SG_FC_NB>, true>>(
            a, q_fwd, blocks, ppox::as_stream(stream), "ppox_nature_fc_fwd");
    return launch_sgemm<SgRows<3136, 512, FC_FWD, FC_FWD_GW, false, SG_FC_NB>>(a, q_fwd, blocks, ppox::as_stream(stream),
                                                                             "ppox_nature_fc_fwd");
}

extern "C" int64_t ppox_nature_fc_fwd_splitk_workspace_bytes(int64_t batch) {
    if (batch <= 0) return 0;
    const long long s = ppox_conv::fcw_sk_enabled(batch) ? ppox_conv::FCW_SPLITS : fc_fwd_splits(batch);
    return (int64_t)s * batch * 512 * 4;
}

extern "C" int ppox_nature_fc_fwd_splitk(const float* h3, int64_t batch, const uint16_t* q_fwd, const float* bias,
                                         void* workspace, int64_t workspace_bytes, float* f, const uint32_t* amax_h3,
                                         uint32_t* amax_f, const float* w_actor, const float* b_actor,
                                         int32_t n_actions, float* logits, const int* h3_exp, void* stream) {
    if (batch == 0) return PPOX_OK;
    PPOX_REQUIRE(h3 && q_fwd && bias && f && workspace && (amax_h3 || h3_exp) && batch > 0,
                 "ppox_nature_fc_fwd_splitk: bad arguments");
    PPOX_REQUIRE(ppox::aligned16(h3) && ppox::aligned16(q_fwd) && ppox::aligned16(f) && ppox::aligned16(workspace) &&
                     (!amax_h3 || ppox::aligned16(amax_h3)),
                 "ppox_nature_fc_fwd_splitk: 16B alignment");
    PPOX_REQUIRE(workspace_bytes >= ppox_nature_fc_fwd_splitk_workspace_bytes(batch),
                 "ppox_nature_fc_fwd_splitk: workspace too small");
    PPOX_REQUIRE(!logits || (w_actor && b_actor && n_actions >= 1 && n_actions <= 8 && ppox::aligned16(w_actor)),
                 "ppox_nature_fc_fwd_splitk: the fused actor head needs 1..8 actions and a 16B-aligned weight");
    Args a{h3, nullptr, 0, 0, 0, nullptr, bias, nullptr, f, batch, amax_h3, amax_f, pack_exp(q_fwd, PL_FCF)};
    a.xexp = h3_exp;  // PX h3
    float* slab = reinterpret_cast<float*>(workspace);
    hipStream_t st = ppox::as_stream(stream);
    const ActorHead act{w_actor, b_actor, logits ? (int)n_actions : 0, logits};
    if (h3_exp && ppox_conv::fcw_sk_enabled(batch)) {  // the wide-tile form split 8 ways (dconv.hip)
        const int rc = ppox_conv::fcw_sk(h3, batch, q_fwd, slab, h3_exp, a.wexp, st);
        if (rc != PPOX_OK) return rc;
        static_assert(ppox_conv::FCW_SPLITS == 8, "the reduce's split count");
        return launch_fc_sk_reduce<8>(a, slab, bias, f, act, st, "ppox_nature_fc_fwd_splitk");
    }
    if (h3_exp) {
        switch (fc_fwd_splits(batch)) {
            case 1: return launch_fc_fwd_sk<3136, 1, true>(a, q_fwd, slab, bias, f, act, st);
            case 2: return launch_fc_fwd_sk<3136, 2, true>(a, q_fwd, slab, bias, f, act, st);
            case 4: return launch_fc_fwd_sk<3136, 4, true>(a, q_fwd, slab, bias, f, act, st);
            default: return launch_fc_fwd_sk<3136, 8, true>(a, q_fwd, slab, bias, f, act, st);
        }
    }
    switch (fc_fwd_splits(batch)) {
        case 1: return launch_fc_fwd_sk<3136, 1>(a, q_fwd, slab, bias, f, act, st);
        case 2: return launch_fc_fwd_sk<3136, 2>(a, q_fwd, slab, bias, f, act, st);
        case 4: return launch_fc_fwd_sk<3136, 4>(a, q_fwd, slab, bias, f, act, st);
        default: return launch_fc_fwd_sk<3136, 8>(a, q_fwd, slab, bias, f, act, st);
    }
}

extern "C" int ppox_nature_fc_dgrad(const float* df, int64_t batch, const uint16_t* q_dgrad, const float* h3, float* g3,
                                    const uint32_t* amax_df, uint32_t* amax_g3, const uint32_t* relu_bits,
                                    int* g3_exp_out, const int* df_exp, void* stream) {
    if (batch == 0) return PPOX_OK;  // empty shard / minibatch: no pointers to check
    PPOX_REQUIRE(df && q_dgrad && (h3 || relu_bits) && g3 && amax_df && batch >= 0,
                 "ppox_nature_fc_dgrad: bad arguments");
    PPOX_REQUIRE(ppox::aligned16(df) && ppox::aligned16(q_dgrad) && ppox::aligned16(amax_df),
                 "ppox_nature_fc_dgrad: 16B alignment");
    Args a{df, nullptr, 0, 0, 0, nullptr, nullptr, h3, g3, batch, amax_df, amax_g3, pack_exp(q_dgrad, PL_FCD)};
    a.bits_mask = relu_bits;  // h3's ReLU bitmask from the conv3 forward (instead of h3)
    a.xexp = df_exp;          // PX df (ppox_px_split): its planes are the A rows as they lie
    const long long blocks = ppox::ceil_div(batch, SG_ROWS) * ppox::ceil_div(3136, SG_FC_NB);
    hipStream_t s = ppox::as_stream(stream);
    const char* nm = "ppox_nature_fc_dgrad";
    using Bits = SgRows<512, 3136, FC_DGRAD, FC_DGRAD_GW, true, SG_FC_NB>;
    using Acts = SgRows<512, 3136, FC_DGRAD, FC_DGRAD_GW, false, SG_FC_NB>;
    if (g3_exp_out) {  // g3 as PX planes, bounded by amax(df) * the fc weight's column norms
        PPOX_REQUIRE(relu_bits, "ppox_nature_fc_dgrad: a PX g3 needs h3's ReLU bitmask");
        PPOX_REQUIRE(ppox_conv::px_bound_ok(q_dgrad),
                     "ppox_nature_fc_dgrad: a PX g3 needs q_dgrad packed by ppox_nature_pack_all / fc_pack");
        a.yexp_out = g3_exp_out;
        a.ynorm = pack_norm(q_dgrad, PL_FCD);
        a.ybias = pack_bmax(q_dgrad, PL_FCD);
        if (df_exp && ppox_conv::dfcd_enabled(batch))
            return ppox_conv::dfcd(df, batch, q_dgrad, g3, amax_df, amax_g3, relu_bits, g3_exp_out, df_exp, a.wexp,
                                   a.ynorm, a.ybias, s);
        return df_exp ? launch_sgemm<Px<Bits, true, true>>(a, q_dgrad, blocks, s, nm)
                      : launch_sgemm<Px<Bits, false, true>>(a, q_dgrad, blocks, s, nm);
    }
    if (relu_bits)
        return df_exp ? launch_sgemm<Px<Bits, true>>(a, q_dgrad, blocks, s, nm) : launch_sgemm<Bits>(a, q_dgrad, blocks, s, nm);
    return df_exp ? launch_sgemm<Px<Acts, true>>(a, q_dgrad, blocks, s, nm) : launch_sgemm<Acts>(a, q_dgrad, blocks, s, nm);
}

extern "C" int ppox_nature_pack_all(const float* w1, const float* b1, const float* w2, const float* b2,
                                    const float* w3, const float* b3, const float* wfc, float* wpd2, uint16_t* q1,
                                    uint16_t* q2, uint16_t* q3, uint16_t* qd2, uint16_t* qd3, uint16_t* qfc_fwd,
                                    uint16_t* qfc_dgrad, const float* wh, uint16_t* qh_fwd, uint16_t* qh_dgrad,
                                    uint32_t* zero, int64_t zero_words, void* stream) {
    PPOX_REQUIRE(w1 && w2 && w3 && (wfc || (!qfc_fwd && !qfc_dgrad)), "ppox_nature_pack_all: null weights");
    PPOX_REQUIRE(!q1 || b1, "ppox_nature_pack_all: q1 needs the conv1 bias b1 (the H1P exponent)");
    PPOX_REQUIRE(zero_words >= 0 && (zero_words == 0 || zero), "ppox_nature_pack_all: zero buffer");
    PackAll p{w1, w2, w3, wfc, wpd2, q1, q2, q3, qd2, qd3, qfc_fwd, qfc_dgrad, wh, qh_fwd, qh_dgrad, b1, zero,
              zero_words};
    p.b2 = b2;
    p.b3 = b3;
    return launch_pack_all(p, ppox::as_stream(stream), "ppox_nature_pack_all");
}

extern "C" int ppox_nature_pack_all_wmax(const float* w1, const float* b1, const float* w2, const float* b2,
                                         const float* w3, const float* b3, const float* wfc, float* wpd2,
                                         uint16_t* q1, uint16_t* q2, uint16_t* q3, uint16_t* qd2, uint16_t* qd3,
                                         uint16_t* qfc_fwd, uint16_t* qfc_dgrad, const float* wh, uint16_t* qh_fwd,
                                         uint16_t* qh_dgrad, const uint32_t* amax_in, uint32_t* amax_next,
                                         uint32_t* zero, int64_t zero_words, void* stream) {
    static_assert(PPOX_WMAX_TENSORS == PA_TENSORS && PPOX_WMAX_SLOTS == AMAX_SLOTS, "ppox.h: the amax partials");
    PPOX_REQUIRE(w1 && w2 && w3 && (wfc || (!qfc_fwd && !qfc_dgrad)), "ppox_nature_pack_all_wmax: null weights");
    PPOX_REQUIRE(!q1 || b1, "ppox_nature_pack_all_wmax: q1 needs the conv1 bias b1 (the H1P exponent)");
    PPOX_REQUIRE(zero_words >= 0 && (zero_words == 0 || zero), "ppox_nature_pack_all_wmax: zero buffer");
    PackAll p{w1, w2, w3, wfc, wpd2, q1, q2, q3, qd2, qd3, qfc_fwd, qfc_dgrad, wh, qh_fwd, qh_dgrad, b1, zero,
              zero_words};
    p.b2 = b2;
    p.b3 = b3;
    p.amax_in = amax_in;
    p.amax_next = amax_next;
    return launch_pack_all(p, ppox::as_stream(stream), "ppox_nature_pack_all_wmax");
}

// ---- the heads' hidden layer Linear(512, 512) + ReLU on the split-f16 GEMM -------------
extern "C" int64_t ppox_head_hidden_pack_elems(void) { return PL_H + 2 * PACK_TAIL32; }

extern "C" int ppox_head_hidden_fwd(const float* f, int64_t rows, const uint16_t* q_fwd, const float* bias, float* e,
                                    const uint32_t* amax_f, void* stream) {
    if (rows == 0) return PPOX_OK;
    PPOX_REQUIRE(f && q_fwd && bias && e && amax_f && rows > 0, "ppox_head_hidden_fwd: bad arguments");
    PPOX_REQUIRE(ppox::aligned16(f) && ppox::aligned16(q_fwd) && ppox::aligned16(amax_f),
                 "ppox_head_hidden_fwd: 16B alignment");
    Args a{f, nullptr, 0, 0, 0, nullptr, bias, nullptr, e, rows, amax_f, nullptr, pack_exp(q_fwd, PL_H)};
    return launch_sgemm<SgRows<512, 512, FC_FWD, HEAD_GW, false, SG_FC_NB>>(
        a, q_fwd, ppox::ceil_div(rows, SG_ROWS) * (512 / SG_FC_NB), ppox::as_stream(stream), "ppox_head_hidden_fwd");
}

extern "C" int64_t ppox_head_hidden_fwd_splitk_workspace_bytes(int64_t rows) {
    return rows <= 0 ? 0 : (int64_t)fc_fwd_splits(rows, 256) * rows * 512 * 4;
}

// small batches: split over K like ppox_nature_fc_fwd_splitk (128 workgroups of 128 rows at 2,048 rows
// leave half the chip idle), the critic head v = e w_critic^T + b_critic fused into the reduce
extern "C" int ppox_head_hidden_fwd_splitk(const float* f, int64_t rows, const uint16_t* q_fwd, const float* bias,
                                           void* workspace, int64_t workspace_bytes, float* e, const uint32_t* amax_f,
                                           const float* w_critic, const float* b_critic, float* value, void* stream) {
    if (rows == 0) return PPOX_OK;
    PPOX_REQUIRE(f && q_fwd && bias && e && workspace && amax_f && rows > 0, "ppox_head_hidden_fwd_splitk: bad arguments");
    PPOX_REQUIRE(ppox::aligned16(f) && ppox::aligned16(q_fwd) && ppox::aligned16(e) && ppox::aligned16(workspace) &&
                     ppox::aligned16(amax_f),
                 "ppox_head_hidden_fwd_splitk: 16B alignment");
    PPOX_REQUIRE(workspace_bytes >= ppox_head_hidden_fwd_splitk_workspace_bytes(rows),
                 "ppox_head_hidden_fwd_splitk: workspace too small");
    PPOX_REQUIRE(!value || (w_critic && b_critic && ppox::aligned16(w_critic)),
                 "ppox_head_hidden_fwd_splitk: the fused critic head needs a 16B-aligned weight");
    Args a{f, nullptr, 0, 0, 0, nullptr, bias, nullptr, e, rows, amax_f, nullptr, pack_exp(q_fwd, PL_H)};
    float* slab = reinterpret_cast<float*>(workspace);
    hipStream_t st = ppox::as_stream(stream);
    const ActorHead crit{w_critic, b_critic, value ? 1 : 0, value};
    constexpr const char* nm = "ppox_head_hidden_fwd_splitk";
    switch (fc_fwd_splits(rows, 256)) {
        case 1: return launch_fc_fwd_sk<512, 1>(a, q_fwd, slab, bias, e, crit, st, nm);
        case 2: return launch_fc_fwd_sk<512, 2>(a, q_fwd, slab, bias, e, crit, st, nm);
        case 4: return launch_fc_fwd_sk<512, 4>(a, q_fwd, slab, bias, e, crit, st, nm);
        default: return launch_fc_fwd_sk<512, 8>(a, q_fwd, slab, bias, e, crit, st, nm);
    }
}

extern "C" int ppox_head_hidden_dgrad(const float* de, int64_t rows, const uint16_t* q_dgrad, const float* f, float* df,
                                      const uint32_t* amax_de, uint32_t* amax_df, void* stream) {
    if (rows == 0) return PPOX_OK;
    PPOX_REQUIRE(de && q_dgrad && f && df && amax_de && rows > 0, "ppox_head_hidden_dgrad: bad arguments");
    PPOX_REQUIRE(ppox::aligned16(de) && ppox::aligned16(q_dgrad) && ppox::aligned16(amax_de),
                 "ppox_head_hidden_dgrad: 16B alignment");
    Args a{de, nullptr, 0, 0, 0, nullptr, nullptr, f, df, rows, amax_de, amax_df, pack_exp(q_dgrad, PL_H)};
    return launch_sgemm<SgRows<512, 512, HEAD_DGRAD, HEAD_GW, false, SG_FC_NB>>(
        a, q_dgrad, ppox::ceil_div(rows, SG_ROWS) * (512 / SG_FC_NB), ppox::as_stream(stream), "ppox_head_hidden_dgrad");
}

// the heads' backward to the fc output in one launch (csrc/dconv.hip hbw_kernel): de = (e > 0) dv wc and
// df = (f > 0) (dout Wa + de Wh) — ppox_head_dgrad_outer + ppox_head_hidden_dgrad without de's HBM round trip
extern "C" int ppox_head_backward(const float* dout, const float* w_actor, const float* dv, const float* w_critic,
                                  const float* e, const float* f, const uint16_t* q_dgrad, int64_t rows, int64_t h,
                                  int64_t n_out, float* df, float* de, uint32_t* amax_de, uint32_t* amax_df,
                                  void* stream) {
    if (rows == 0) return PPOX_OK;
    PPOX_REQUIRE(dout && w_actor && dv && w_critic && e && f && q_dgrad && df && de && amax_de && amax_df && rows > 0,
                 "ppox_head_backward: bad arguments");
    PPOX_REQUIRE(h == 512, "ppox_head_backward: the hidden layer is 512 wide");
    PPOX_REQUIRE(ppox::aligned16(amax_de) && ppox::aligned16(amax_df), "ppox_head_backward: 16B alignment");
    return ppox_conv::head_backward(dout, w_actor, dv, w_critic, e, f, q_dgrad, pack_exp(q_dgrad, PL_H), rows,
                                    (int)n_out, df, de, amax_de, amax_df, ppox::as_stream(stream));
}

extern "C" int64_t ppox_head_hidden_wgrad_workspace_bytes(int64_t rows) {
    return rows <= 0 ? 0 : HeadWgrad::workspace_bytes(rows);
}

extern "C" int ppox_head_hidden_wgrad(const float* de, int64_t rows, const float* f, void* workspace,
                                      int64_t workspace_bytes, float* dw, const uint32_t* amax_de,
                                      const uint32_t* amax_f, void* stream) {
    PPOX_REQUIRE(dw && rows >= 0, "ppox_head_hidden_wgrad: bad arguments");
    hipStream_t s = ppox::as_stream(stream);
    if (rows == 0) {  // no rows: a zero gradient
        PPOX_REQUIRE(hipMemsetAsync(dw, 0, sizeof(float) * HeadWgrad::SLAB, s) == hipSuccess,
                     "ppox_head_hidden_wgrad: memset failed");
        return PPOX_OK;
    }
    PPOX_REQUIRE(de && f && workspace && amax_de && amax_f, "ppox_head_hidden_wgrad: bad arguments");
    PPOX_REQUIRE(workspace_bytes >= HeadWgrad::workspace_bytes(rows), "ppox_head_hidden_wgrad: workspace too small");
    PPOX_REQUIRE(ppox::aligned16(de) && ppox::aligned16(f) && ppox::aligned16(amax_de) && ppox::aligned16(amax_f),
                 "ppox_head_hidden_wgrad: 16B alignment");
    PPOX_REQUIRE(rows < (1LL << 31) / 64, "ppox_head_hidden_wgrad: too many rows for 32-bit row indexing");
    const int sp = HeadWgrad::splits(rows);
    float* slab = reinterpret_cast<float*>(workspace);
    WArgs wa{de, 0, f, slab, nullptr, rows, 0, sp, nullptr, 0, 0, amax_de, amax_f};
    wa.px_per_split = ppox::ceil_div(ppox::ceil_div((long long)rows, (long long)sp), (long long)MS) * MS;
    wgrad_split_kernel<GFc, false, FCW_KT, false, 512 / 64><<<(unsigned)(HeadWgrad::TILES * sp), 256, 0, s>>>(wa);
    PPOX_LAUNCHED_NORET("ppox_head_hidden_wgrad");
    ppox::ktime_mark(s);
    rows_wgrad_reduce<512, false><<<(unsigned)ppox::ceil_div(HeadWgrad::SLAB, 1024LL), 256, 0, s>>>(slab, sp, dw);
    PPOX_LAUNCHED("ppox_head_hidden_wgrad");
}

// ---- amax slots (split-f16 operand scales) -------------------------------------------
__global__ void __launch_bounds__(256) amax_kernel(const float4* __restrict__ x, long long n4,
                                                   uint32_t* __restrict__ am) {
    float m = 0.f;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
        const float4 v = x[i];
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    amax_record(am, m);
}

extern "C" int32_t ppox_amax_slots(void) { return AMAX_SLOTS; }

extern "C" int ppox_amax(const float* x, int64_t n, uint32_t* amax, void* stream) {
    PPOX_REQUIRE(amax && n >= 0 && n % 4 == 0 && (x || n == 0), "ppox_amax: bad arguments (n % 4 == 0)");
    PPOX_REQUIRE(ppox::aligned16(amax) && (!x || ppox::aligned16(x)), "ppox_amax: 16B alignment");
    if (n == 0) return PPOX_OK;
    const long long blocks = std::min<long long>(ppox::ceil_div(n / 4, 256LL), 1024);
    amax_kernel<<<(unsigned)blocks, 256, 0, ppox::as_stream(stream)>>>(reinterpret_cast<const float4*>(x), n / 4, amax);
    PPOX_LAUNCHED("ppox_amax");
}

// ---- PX planes of an f32 tensor whose amax is recorded (round 4: the fc layer's df) ----------
// y = the two f16 planes of x 2^E (include/ppox.h "PX"), E from x's amax slots — the scale a split
// GEMM would take for x as an f32 operand, so the planes are the split every consumer tile made
// in registers before (the fc dgrad split each df value once per 64-column tile: 49 times).
// A thread splits 4 consecutive values of a 32-group: 16 B in, 8 B to each plane out.
__global__ void __launch_bounds__(256) px_split_kernel(const float4* __restrict__ x, long long n4,
                                                       const uint32_t* __restrict__ am, uint16_t* __restrict__ y,
                                                       int* __restrict__ e_out) {
    const int e = split_scale_exp(amax_read(am));
    const float sc = exp2i(e);
    if (blockIdx.x == 0 && threadIdx.x == 0) *e_out = e;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
        uint2 h, l;
        split4h(x[i], sc, h, l);
        uint16_t* q = y + px_index(4 * i);
        *reinterpret_cast<uint2*>(q) = h;
        *reinterpret_cast<uint2*>(q + 32) = l;
    }
}

extern "C" int ppox_px_split(const float* x, int64_t n, const uint32_t* amax, uint16_t* y, int* exp_out,
                             void* stream) {
    PPOX_REQUIRE(amax && y && exp_out && n >= 0 && n % 32 == 0 && (x || n == 0),
                 "ppox_px_split: bad arguments (n % 32 == 0)");
    PPOX_REQUIRE(ppox::aligned16(amax) && ppox::aligned16(y) && (!x || ppox::aligned16(x)),
                 "ppox_px_split: 16B alignment");
    if (n == 0) return PPOX_OK;
    const long long blocks = std::min<long long>(ppox::ceil_div(n / 4, 256LL), 2048);
    px_split_kernel<<<(unsigned)blocks, 256, 0, ppox::as_stream(stream)>>>(reinterpret_cast<const float4*>(x), n / 4,
                                                                           amax, y, exp_out);
    PPOX_LAUNCHED("ppox_px_split");
}
