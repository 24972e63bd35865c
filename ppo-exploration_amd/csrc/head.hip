// NatureCNN head backward helpers (the elementwise parts of the explicit training
// backward of CnnActorCritic, models.py; .ipynb_checkpoints/models-checkpoint.py:60-87):
//   ppox_relu_backward_:    g = act > 0 ? g : 0 (in place) — nn.ReLU backward
//   ppox_outer_relu_backward: d[b][j] = dv[b] * w[j] * (act[b][j] > 0) — the grad of
//       a ReLU layer feeding a Linear(H, 1) critic (extra_layer -> critic_ext)
// One pass each, float4 lanes (HBM-bound: 12 B / element).
//   ppox_head_grads: every column-reduction parameter gradient of the heads in one pass
//       over f, e, de, df (+ the intrinsic head's): actor weight/bias (dout^T f, sum dout),
//       critic weight/bias (dv^T e, sum dv), extra-layer bias (sum de), fc bias (sum df).
//       Fixed-order two-level sums (row chunks, then chunks in order): deterministic.
#include "conv_common.h"  // common.h + the split-f16 amax helpers

namespace {

// am (nullable): the masked grad's amax slots (a split-f16 GEMM operand)
__global__ void __launch_bounds__(256) relu_bwd_kernel(float* __restrict__ g, const float* __restrict__ act,
                                                       long long n4, uint32_t* __restrict__ am) {
    float m = 0.f;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
        float4 v = reinterpret_cast<float4*>(g)[i];
        const float4 a = reinterpret_cast<const float4*>(act)[i];
        v.x = a.x > 0.f ? v.x : 0.f;
        v.y = a.y > 0.f ? v.y : 0.f;
        v.z = a.z > 0.f ? v.z : 0.f;
        v.w = a.w > 0.f ? v.w : 0.f;
        reinterpret_cast<float4*>(g)[i] = v;
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    amax_record(am, m);
}

// partial row of chunk c: [A*H actor W | A actor b | H critic W | 1 critic b | H extra b |
//                         H fc b | (intrinsic) H critic_int W | 1 critic_int b | H int_extra b]
struct HeadGrads {
    const float *f, *e, *ie, *dout, *dv, *div, *de, *die;
    float* df;
    long long B, R;  // rows, rows per chunk
    int H, A;
    int relu_df;        // df = f > 0 ? df : 0 first, written back (the fc layer's ReLU backward)
    uint32_t* amax_df;  // nullable: the masked df's amax slots
    // nullable (round 6): df's PX planes written in the same pass (ppox_px_split's split, bitwise) at the exponent
    // of its amax slots px_amax (recorded by the heads' backward), the exponent stored to *px_exp
    uint16_t* px;
    const uint32_t* px_amax;
    int* px_exp;
};
constexpr int HG_MAXA = 18, HG_MAXH = 512;  // actions (Montezuma 18), hidden width

__host__ __device__ inline long long head_grads_len(int H, int A, bool intr) {
    return (long long)A * H + A + H + 1 + 2LL * H + (intr ? 2LL * H + 1 : 0);
}

// thread t owns columns 2t, 2t + 1 (float2 loads); H even, H <= 512.  AM >= A actions and the
// intrinsic head are template parameters, so every load of a row is unconditional (the dout loads
// of actions a >= A re-read action A - 1 and are multiplied by zero into sums never stored): the
// row's loads issue together (a load under a branch costs a full memory round trip each)
template <int AM, bool INTR>
__global__ void __launch_bounds__(256) head_grads_partials(HeadGrads g, float* __restrict__ part) {
    const long long r0 = (long long)blockIdx.x * g.R, r1 = min(g.B, r0 + g.R);
    const int tid = threadIdx.x, H = g.H, A = g.A, j = 2 * tid;
    const bool col = j < H;
    float2 wa[AM], wc = {0.f, 0.f}, be = {0.f, 0.f}, bf = {0.f, 0.f}, wci = {0.f, 0.f}, bie = {0.f, 0.f};
    float ba[AM], bc = 0.f, bci = 0.f;
#pragma unroll
    for (int a = 0; a < AM; ++a) {
        wa[a] = make_float2(0.f, 0.f);
        ba[a] = 0.f;
    }
    const int jc = col ? j : 0;
    auto ld = [&](const float* p, long long b) { return *reinterpret_cast<const float2*>(p + b * H + jc); };
    float dm = 0.f;  // the masked df's largest |value| in this thread's columns
    float psc = 0.f;
    if (g.px) {  // (uniform)
        const int pe = split_scale_exp(amax_read(g.px_amax));
        psc = exp2i(pe);
        if (blockIdx.x == 0 && tid == 0) *g.px_exp = pe;
    }
#pragma unroll 4
    for (long long b = r0; b < r1; ++b) {
        const float dv = g.dv[b], div = INTR ? g.div[b] : 0.f;
        const float2 fv = ld(g.f, b), ev = ld(g.e, b), dev = ld(g.de, b);
        float2 dfv = ld(g.df, b);
        float d[AM];
#pragma unroll
        for (int a = 0; a < AM; ++a) d[a] = g.dout[b * A + (a < A ? a : A - 1)];
        float2 iev = {0.f, 0.f}, diev = {0.f, 0.f};
        if constexpr (INTR) {
            iev = ld(g.ie, b);
            diev = ld(g.die, b);
        }
        if (g.relu_df) {  // uniform
            dfv.x = fv.x > 0.f ? dfv.x : 0.f;
            dfv.y = fv.y > 0.f ? dfv.y : 0.f;
            if (col) *reinterpret_cast<float2*>(g.df + b * H + j) = dfv;
            dm = fmaxf(dm, fmaxf(fabsf(dfv.x), fabsf(dfv.y)));
        }
        if (g.px && col) {  // the pair's two high halves, then 32 halves further its two low halves
            uint32_t ph, pl;
            split2h((f32x2){dfv.x, dfv.y}, psc, ph, pl);
            uint16_t* q = g.px + px_index(b * H + j);
            *reinterpret_cast<uint32_t*>(q) = ph;
            *reinterpret_cast<uint32_t*>(q + 32) = pl;
        }
#pragma unroll
        for (int a = 0; a < AM; ++a) {
            wa[a].x = fmaf(d[a], fv.x, wa[a].x);
            wa[a].y = fmaf(d[a], fv.y, wa[a].y);
            ba[a] += d[a];
        }
        wc.x = fmaf(dv, ev.x, wc.x);
        wc.y = fmaf(dv, ev.y, wc.y);
        be.x += dev.x;
        be.y += dev.y;
        bf.x += dfv.x;
        bf.y += dfv.y;
        bc += dv;
        if constexpr (INTR) {
            wci.x = fmaf(div, iev.x, wci.x);
            wci.y = fmaf(div, iev.y, wci.y);
            bie.x += diev.x;
            bie.y += diev.y;
            bci += div;
        }
    }
    float* p = part + (long long)blockIdx.x * head_grads_len(H, A, INTR);
    const long long o = (long long)A * H + A;
    auto st = [&](long long at, float2 v) {
        p[at] = v.x;
        p[at + 1] = v.y;
    };
    if (col) {
#pragma unroll
        for (int a = 0; a < AM; ++a)
            if (a < A) st((long long)a * H + j, wa[a]);
        st(o + j, wc);
        st(o + H + 1 + j, be);
        st(o + 2 * H + 1 + j, bf);
        if (INTR) {
            st(o + 3 * H + 1 + j, wci);
            st(o + 4 * H + 2 + j, bie);
        }
    }
    if (tid == 0) {
#pragma unroll
        for (int a = 0; a < AM; ++a)
            if (a < A) p[(long long)A * H + a] = ba[a];
        p[o + H] = bc;
        if (INTR) p[o + 4 * H + 1] = bci;
    }
    if (g.relu_df) amax_record(g.amax_df, dm);
}

struct HeadGradOut {
    float *wa, *ba, *wc, *bc, *be, *bfc, *wci, *bci, *bie;
};

// 64 outputs per block; wave w sums chunks w, w + 4, ... (eight independent partial sums,
// combined in a fixed order), then the four waves' sums are combined in order: deterministic
__global__ void __launch_bounds__(256) head_grads_reduce(const float* __restrict__ part, long long nchunk, long long len,
                                                         int H, int A, HeadGradOut out) {
    __shared__ float red[4][64];
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long long i0 = (long long)blockIdx.x * 64 + l, ic = i0 < len ? i0 : len - 1;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    long long c = w;
    for (; c + 28 < nchunk; c += 32)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += part[(c + 4 * k) * len + ic];
    for (int k = 0; c < nchunk; c += 4, ++k) acc[k & 7] += part[c * len + ic];
    red[w][l] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    __syncthreads();
    if (w != 0 || i0 >= len) return;
    const float s = (red[0][l] + red[1][l]) + (red[2][l] + red[3][l]);
    const long long i = i0;
    // segment of element i (layout of head_grads_partials)
    long long o = i;
    const long long nwa = (long long)A * H;
    if (o < nwa) { out.wa[o] = s; return; }
    o -= nwa;
    if (o < A) { out.ba[o] = s; return; }
    o -= A;
    if (o < H) { out.wc[o] = s; return; }
    o -= H;
    if (o < 1) { out.bc[0] = s; return; }
    o -= 1;
    if (o < H) { out.be[o] = s; return; }
    o -= H;
    if (o < H) { out.bfc[o] = s; return; }
    o -= H;
    if (o < H) { out.wci[o] = s; return; }
    o -= H;
    if (o < 1) { out.bci[0] = s; return; }
    o -= 1;
    out.bie[o] = s;
}

// skinny linear y[b][o] = x[b] . w[o] + bias[o] for NO <= 8 outputs (actor / critic heads,
// models-checkpoint.py:60-87): one wave per row, lane l holds x[b][8l .. 8l+7] of each
// 512-wide chunk, wave-reduces the NO dot products (fixed butterfly order: deterministic)
template <int NO>
__global__ void __launch_bounds__(256) skinny_linear_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                            const float* __restrict__ bias, long long rows, int h,
                                                            float* __restrict__ y) {
    const int lane = threadIdx.x & 63;
    const long long b = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= rows) return;
    float acc[NO];
#pragma unroll
    for (int o = 0; o < NO; ++o) acc[o] = 0.f;
    for (int k = lane * 4; k < h; k += 256) {
        const float4 xv = *reinterpret_cast<const float4*>(x + b * h + k);
#pragma unroll
        for (int o = 0; o < NO; ++o) {
            const float4 wv = *reinterpret_cast<const float4*>(w + (long long)o * h + k);
            acc[o] = fmaf(xv.x, wv.x, acc[o]);
            acc[o] = fmaf(xv.y, wv.y, acc[o]);
            acc[o] = fmaf(xv.z, wv.z, acc[o]);
            acc[o] = fmaf(xv.w, wv.w, acc[o]);
        }
    }
#pragma unroll
    for (int o = 0; o < NO; ++o)
#pragma unroll
        for (int m = 32; m > 0; m >>= 1) acc[o] += __shfl_xor(acc[o], m, 64);
    if (lane < NO) {
        float r = acc[0];
#pragma unroll
        for (int o = 1; o < NO; ++o) r = lane == o ? acc[o] : r;
        y[b * NO + lane] = r + bias[lane];
    }
}

// skinny dgrad d[b][j] = sum_o g[b][o] w[o][j] (o < NO): the actor head's input grad
template <int NO>
__global__ void __launch_bounds__(256) skinny_dgrad_kernel(const float* __restrict__ g, const float* __restrict__ w,
                                                           long long rows, int h4, float* __restrict__ d) {
    const long long n4 = rows * h4;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
        const long long b = i / h4;
        const int j = (int)(i - b * h4);
        float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int o = 0; o < NO; ++o) {
            const float go = g[b * NO + o];
            const float4 wv = reinterpret_cast<const float4*>(w)[(long long)o * h4 + j];
            r.x = fmaf(go, wv.x, r.x);
            r.y = fmaf(go, wv.y, r.y);
            r.z = fmaf(go, wv.z, r.z);
            r.w = fmaf(go, wv.w, r.w);
        }
        reinterpret_cast<float4*>(d)[i] = r;
    }
}

// am (nullable): d's amax slots (the split hidden layer's dgrad / weight gradient read d)
__global__ void __launch_bounds__(256) outer_relu_kernel(const float* __restrict__ dv, const float* __restrict__ w,
                                                         const float* __restrict__ act, long long rows, int h4,
                                                         float* __restrict__ d, uint32_t* __restrict__ am) {
    const long long n4 = rows * h4;
    float m = 0.f;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
        const long long b = i / h4;
        const int j = (int)(i - b * h4);
        const float s = dv[b];
        const float4 ww = make_float4(w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]);  // w may be unaligned
        const float4 a = reinterpret_cast<const float4*>(act)[i];
        float4 o;
        o.x = a.x > 0.f ? s * ww.x : 0.f;
        o.y = a.y > 0.f ? s * ww.y : 0.f;
        o.z = a.z > 0.f ? s * ww.z : 0.f;
        o.w = a.w > 0.f ? s * ww.w : 0.f;
        reinterpret_cast<float4*>(d)[i] = o;
        m = fmaxf(m, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
    }
    amax_record(am, m);
}

// the actor head's input grad and the critic's ReLU-layer grad in one pass (skinny_dgrad_kernel and
// outer_relu_kernel, same arithmetic, bitwise the same results): df = dout wa, de = dv wc (e > 0)
template <int NO>
__global__ void __launch_bounds__(256) head_dgrad_outer_kernel(const float* __restrict__ dout, const float* __restrict__ wa,
                                                               const float* __restrict__ dv, const float* __restrict__ wc,
                                                               const float* __restrict__ e, long long rows, int h4,
                                                               float* __restrict__ df, float* __restrict__ de,
                                                               uint32_t* __restrict__ am) {
    const long long n4 = rows * h4;
    float m = 0.f;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
        const long long b = i / h4;
        const int j = (int)(i - b * h4);
        float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int o = 0; o < NO; ++o) {
            const float go = dout[b * NO + o];
            const float4 wv = reinterpret_cast<const float4*>(wa)[(long long)o * h4 + j];
            r.x = fmaf(go, wv.x, r.x);
            r.y = fmaf(go, wv.y, r.y);
            r.z = fmaf(go, wv.z, r.z);
            r.w = fmaf(go, wv.w, r.w);
        }
        reinterpret_cast<float4*>(df)[i] = r;
        const float s = dv[b];
        const float4 ww = make_float4(wc[4 * j], wc[4 * j + 1], wc[4 * j + 2], wc[4 * j + 3]);  // wc may be unaligned
        const float4 a = reinterpret_cast<const float4*>(e)[i];
        float4 o;
        o.x = a.x > 0.f ? s * ww.x : 0.f;
        o.y = a.y > 0.f ? s * ww.y : 0.f;
        o.z = a.z > 0.f ? s * ww.z : 0.f;
        o.w = a.w > 0.f ? s * ww.w : 0.f;
        reinterpret_cast<float4*>(de)[i] = o;
        m = fmaxf(m, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
    }
    amax_record(am, m);
}

unsigned grid_for(long long n4) {
    const long long g = (n4 + 255) / 256;
    return (unsigned)(g < 4096 ? (g > 0 ? g : 1) : 4096);
}

}  // namespace

extern "C" int ppox_relu_backward_(float* grad, const float* act, int64_t n, void* stream) {
    if (n == 0) return PPOX_OK;  // empty shard / minibatch: no pointers to check
    PPOX_REQUIRE(grad && act && n >= 0 && n % 4 == 0, "ppox_relu_backward_: bad arguments (n % 4 == 0)");
    PPOX_REQUIRE(ppox::aligned16(grad) && ppox::aligned16(act), "ppox_relu_backward_: 16B alignment");
    relu_bwd_kernel<<<grid_for(n / 4), 256, 0, ppox::as_stream(stream)>>>(grad, act, n / 4, nullptr);
    PPOX_LAUNCHED("ppox_relu_backward_");
}

extern "C" int ppox_relu_backward_amax_(float* grad, const float* act, int64_t n, uint32_t* amax, void* stream) {
    if (n == 0) return PPOX_OK;
    PPOX_REQUIRE(grad && act && amax && n > 0 && n % 4 == 0, "ppox_relu_backward_amax_: bad arguments (n % 4 == 0)");
    PPOX_REQUIRE(ppox::aligned16(grad) && ppox::aligned16(act) && ppox::aligned16(amax),
                 "ppox_relu_backward_amax_: 16B alignment");
    relu_bwd_kernel<<<grid_for(n / 4), 256, 0, ppox::as_stream(stream)>>>(grad, act, n / 4, amax);
    PPOX_LAUNCHED("ppox_relu_backward_amax_");
}

extern "C" int64_t ppox_head_grads_workspace_bytes(int64_t rows, int64_t h, int64_t n_actions, int32_t intrinsic) {
    if (rows < 0 || h <= 0 || h > HG_MAXH || h % 2 || n_actions <= 0 || n_actions > HG_MAXA) return -1;
    const long long R = std::max<long long>(8, (rows + 511) / 512), nchunk = std::max<long long>(1, (rows + R - 1) / R);
    return nchunk * head_grads_len((int)h, (int)n_actions, intrinsic != 0) * (long long)sizeof(float);
}

extern "C" int ppox_head_grads(const float* f, const float* e, const float* dout, const float* dv, const float* de,
                               const float* df, const float* ie, const float* div, const float* die, int64_t rows,
                               int64_t h, int64_t n_actions, void* workspace, float* w_actor, float* b_actor,
                               float* w_critic, float* b_critic, float* b_extra, float* b_fc, float* w_critic_int,
                               float* b_critic_int, float* b_int_extra, int32_t relu_df, uint32_t* amax_df,
                               uint16_t* df_planes, const uint32_t* df_planes_amax, int32_t* df_planes_exp,
                               void* stream) {
    PPOX_REQUIRE(f && e && dout && dv && de && df && workspace && rows >= 0, "ppox_head_grads: null input");
    PPOX_REQUIRE(!amax_df || (relu_df && ppox::aligned16(amax_df)), "ppox_head_grads: amax_df needs relu_df (16B)");
    PPOX_REQUIRE(h > 0 && h <= HG_MAXH && h % 2 == 0 && n_actions > 0 && n_actions <= HG_MAXA,
                 "ppox_head_grads: h must be even and <= 512, n_actions <= 18");
    PPOX_REQUIRE(ppox::aligned16(f) && ppox::aligned16(e) && ppox::aligned16(de) && ppox::aligned16(df),
                 "ppox_head_grads: 16B alignment");
    PPOX_REQUIRE(w_actor && b_actor && w_critic && b_critic && b_extra && b_fc, "ppox_head_grads: null output");
    const bool intr = ie != nullptr;
    PPOX_REQUIRE(!intr || (div && die && w_critic_int && b_critic_int && b_int_extra),
                 "ppox_head_grads: intrinsic head needs div, die and its three outputs");
    PPOX_REQUIRE(!df_planes || (!relu_df && h % 32 == 0 && df_planes_amax && df_planes_exp &&
                                ppox::aligned16(df_planes) && ppox::aligned16(df_planes_amax)),
                 "ppox_head_grads: df planes need relu_df == 0 (df final), h % 32 == 0, the amax slots and the "
                 "exponent output (16B aligned)");
    const long long R = std::max<long long>(8, (rows + 511) / 512), nchunk = std::max<long long>(1, (rows + R - 1) / R);
    const long long len = head_grads_len((int)h, (int)n_actions, intr);
    hipStream_t s = ppox::as_stream(stream);
    float* part = reinterpret_cast<float*>(workspace);
    HeadGrads g{f, e, ie, dout, dv, div, de, die, const_cast<float*>(df), rows, R, (int)h, (int)n_actions,
                relu_df != 0, amax_df, df_planes, df_planes_amax, df_planes_exp};
    if (n_actions <= 4) {
        if (intr) head_grads_partials<4, true><<<(unsigned)nchunk, 256, 0, s>>>(g, part);
        else head_grads_partials<4, false><<<(unsigned)nchunk, 256, 0, s>>>(g, part);
    } else {
        if (intr) head_grads_partials<HG_MAXA, true><<<(unsigned)nchunk, 256, 0, s>>>(g, part);
        else head_grads_partials<HG_MAXA, false><<<(unsigned)nchunk, 256, 0, s>>>(g, part);
    }
    PPOX_LAUNCHED_NORET("ppox_head_grads");
    HeadGradOut o{w_actor, b_actor, w_critic, b_critic, b_extra, b_fc, w_critic_int, b_critic_int, b_int_extra};
    head_grads_reduce<<<(unsigned)((len + 63) / 64), 256, 0, s>>>(part, nchunk, len, (int)h, (int)n_actions, o);
    PPOX_LAUNCHED("ppox_head_grads");
}

#define PPOX_SKINNY_CASES(M) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8)

extern "C" int ppox_skinny_linear(const float* x, const float* w, const float* bias, int64_t rows, int64_t h,
                                  int64_t n_out, float* y, void* stream) {
    if (rows == 0) return PPOX_OK;  // empty shard / minibatch: no pointers to check
    PPOX_REQUIRE(x && w && bias && y && rows >= 0 && h > 0 && h % 4 == 0 && n_out >= 1 && n_out <= 8,
                 "ppox_skinny_linear: n_out must be 1..8, h a multiple of 4");
    PPOX_REQUIRE(ppox::aligned16(x) && ppox::aligned16(w), "ppox_skinny_linear: 16B alignment");
    const unsigned blocks = (unsigned)((rows + 3) / 4);
    hipStream_t s = ppox::as_stream(stream);
    switch (n_out) {
#define PPOX_SL(N) \
    case N: skinny_linear_kernel<N><<<blocks, 256, 0, s>>>(x, w, bias, rows, (int)h, y); break;
        PPOX_SKINNY_CASES(PPOX_SL)
#undef PPOX_SL
    }
    PPOX_LAUNCHED("ppox_skinny_linear");
}

extern "C" int ppox_skinny_dgrad(const float* g, const float* w, int64_t rows, int64_t h, int64_t n_out, float* d,
                                 void* stream) {
    if (rows == 0) return PPOX_OK;  // empty shard / minibatch: no pointers to check
    PPOX_REQUIRE(g && w && d && rows >= 0 && h > 0 && h % 4 == 0 && n_out >= 1 && n_out <= 8,
                 "ppox_skinny_dgrad: n_out must be 1..8, h a multiple of 4");
    PPOX_REQUIRE(ppox::aligned16(w) && ppox::aligned16(d), "ppox_skinny_dgrad: 16B alignment");
    hipStream_t s = ppox::as_stream(stream);
    switch (n_out) {
#define PPOX_SD(N) \
    case N: skinny_dgrad_kernel<N><<<grid_for(rows * h / 4), 256, 0, s>>>(g, w, rows, (int)(h / 4), d); break;
        PPOX_SKINNY_CASES(PPOX_SD)
#undef PPOX_SD
    }
    PPOX_LAUNCHED("ppox_skinny_dgrad");
}

extern "C" int ppox_outer_relu_backward(const float* dv, const float* w, const float* act, int64_t rows, int64_t h,
                                        float* out, uint32_t* amax, void* stream) {
    if (rows == 0) return PPOX_OK;  // empty shard / minibatch: no pointers to check
    PPOX_REQUIRE(dv && w && act && out && rows >= 0 && h > 0 && h % 4 == 0, "ppox_outer_relu_backward: bad arguments");
    PPOX_REQUIRE(ppox::aligned16(act) && ppox::aligned16(out) && (!amax || ppox::aligned16(amax)),
                 "ppox_outer_relu_backward: 16B alignment");
    outer_relu_kernel<<<grid_for(rows * h / 4), 256, 0, ppox::as_stream(stream)>>>(dv, w, act, rows, (int)(h / 4), out,
                                                                                 amax);
    PPOX_LAUNCHED("ppox_outer_relu_backward");
}

extern "C" int ppox_head_dgrad_outer(const float* dout, const float* w_actor, const float* dv, const float* w_critic,
                                     const float* e, int64_t rows, int64_t h, int64_t n_out, float* df, float* de,
                                     uint32_t* amax_de, void* stream) {
    if (rows == 0) return PPOX_OK;  // empty shard / minibatch: no pointers to check
    PPOX_REQUIRE(dout && w_actor && dv && w_critic && e && df && de && rows >= 0 && h > 0 && h % 4 == 0 && n_out >= 1 &&
                     n_out <= 8,
                 "ppox_head_dgrad_outer: n_out must be 1..8, h a multiple of 4");
    PPOX_REQUIRE(ppox::aligned16(w_actor) && ppox::aligned16(e) && ppox::aligned16(df) && ppox::aligned16(de) &&
                     (!amax_de || ppox::aligned16(amax_de)),
                 "ppox_head_dgrad_outer: 16B alignment");
    hipStream_t s = ppox::as_stream(stream);
    const unsigned g = grid_for(rows * h / 4);
    switch (n_out) {
#define PPOX_HDO(N) \
    case N: head_dgrad_outer_kernel<N><<<g, 256, 0, s>>>(dout, w_actor, dv, w_critic, e, rows, (int)(h / 4), df, de, amax_de); break;
        PPOX_SKINNY_CASES(PPOX_HDO)
#undef PPOX_HDO
    }
    PPOX_LAUNCHED("ppox_head_dgrad_outer");
}
