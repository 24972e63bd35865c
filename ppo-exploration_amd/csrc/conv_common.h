// Definitions shared by the NatureCNN conv translation units (conv.hip: f32 MFMA
// kernels; conv_split.hip: bf16-split MFMA kernels).  Not part of the ABI.
#pragma once
#include "common.h"

namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;

template <int CIN_, int IH_, int IW_, int KH_, int KW_, int S_, int COUT_>
struct Geo {
    static constexpr int CIN = CIN_, IH = IH_, IW = IW_, KH = KH_, KW = KW_, S = S_, COUT = COUT_;
    static constexpr int OH = (IH - KH) / S + 1, OW = (IW - KW) / S + 1, P = OH * OW;
    static constexpr int K = CIN * KH * KW;
};
using G1 = Geo<4, 84, 84, 8, 8, 4, 32>;
using G2 = Geo<32, 20, 20, 4, 4, 2, 64>;
using G3 = Geo<64, 9, 9, 3, 3, 1, 64>;

struct Args {
    const void* x;            // forward input / dgrad: output grad G (NHWC)
    const long long* idx;     // conv1 forward/wgrad: optional env-major rollout rows
    long long T, Nenv;        // rollout dims for idx
    long long sample_stride;  // conv1 input: bytes between samples (idx == nullptr)
    const float* wp;          // packed weights [K][N]
    const float* bias;        // forward bias
    const float* mask;        // dgrad: previous activation (ReLU mask source)
    float* y;                 // output
    long long batch;
};

__device__ inline f32x16 zero16() {
    f32x16 z;
#pragma unroll
    for (int i = 0; i < 16; ++i) z[i] = 0.f;
    return z;
}

__device__ inline long long u8_sample_base(const Args& a, long long n, long long sample_bytes) {
    if (a.idx) {
        const long long i = a.idx[n];
        return ((i % a.T) * a.Nenv + i / a.T) * sample_bytes;
    }
    return n * a.sample_stride;
}

__device__ inline long long xcd_remap(long long b, long long nwg) {
    const long long q = nwg / 8, r = nwg % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// first tap index k with k == i (mod S), S*o + k == i for some 0 <= o < O, and its count
template <int S, int O, int KN>
__device__ inline void tap_range(int i, int& k0, int& cnt) {
    int lo = i - S * (O - 1);
    lo = lo < 0 ? 0 : lo;
    k0 = lo + ((i - lo) % S);
    const int hi = i < KN - 1 ? i : KN - 1;
    cnt = hi >= k0 ? (hi - k0) / S + 1 : 0;
}

// ---- split-bf16 helpers (conv_split.hip and the split kernels of conv.hip) ----
using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
using u32x4 = __attribute__((ext_vector_type(4))) uint32_t;

__device__ inline f32x16 mfma_bf16(const u32x4& a, const u32x4& b, const f32x16& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
}

// two f32 whose low 16 bits are zero (exact bf16 values) -> packed bf16x2 (e0 low)
__device__ inline uint32_t pack_hi(float e0, float e1) {
    return __builtin_amdgcn_perm(__float_as_uint(e1), __float_as_uint(e0), 0x07060302);
}

// eight uint8 (two words) -> a bf16x8 fragment (exact: 0..255 have <= 8 significant bits)
__device__ inline u32x4 u8x8_to_bf16(uint32_t w0, uint32_t w1) {
    u32x4 r;
    r[0] = pack_hi((float)(w0 & 0xFFu), (float)((w0 >> 8) & 0xFFu));
    r[1] = pack_hi((float)((w0 >> 16) & 0xFFu), (float)(w0 >> 24));
    r[2] = pack_hi((float)(w1 & 0xFFu), (float)((w1 >> 8) & 0xFFu));
    r[3] = pack_hi((float)((w1 >> 16) & 0xFFu), (float)(w1 >> 24));
    return r;
}

// exact three-way truncation split of one f32 (host+device; used by the packers)
__host__ __device__ inline void split3(float a, uint16_t& p0, uint16_t& p1, uint16_t& p2) {
    const uint32_t u = __builtin_bit_cast(uint32_t, a);
    const float a0 = __builtin_bit_cast(float, u & 0xFFFF0000u);
    const float r1 = a - a0;
    const uint32_t v = __builtin_bit_cast(uint32_t, r1);
    const float a1 = __builtin_bit_cast(float, v & 0xFFFF0000u);
    const float r2 = r1 - a1;
    p0 = (uint16_t)(u >> 16);
    p1 = (uint16_t)(v >> 16);
    p2 = (uint16_t)(__builtin_bit_cast(uint32_t, r2) >> 16);
}

// eight f32 -> their three exact bf16 planes as MFMA fragments (element e of the
// fragment = value e): a = a0 + a1 + a2 bitwise (see conv_split.hip)
__device__ inline void split8(const float4& v0, const float4& v1, u32x4& p0, u32x4& p1, u32x4& p2) {
    const float x[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    uint32_t h0[8], h1[8], h2[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const uint32_t u0 = __float_as_uint(x[e]) & 0xFFFF0000u;
        const float r1 = x[e] - __uint_as_float(u0);
        const uint32_t u1 = __float_as_uint(r1) & 0xFFFF0000u;
        const float r2 = r1 - __uint_as_float(u1);
        h0[e] = u0;
        h1[e] = u1;
        h2[e] = __float_as_uint(r2);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        p0[q] = __builtin_amdgcn_perm(h0[2 * q + 1], h0[2 * q], 0x07060302);
        p1[q] = __builtin_amdgcn_perm(h1[2 * q + 1], h1[2 * q], 0x07060302);
        p2[q] = __builtin_amdgcn_perm(h2[2 * q + 1], h2[2 * q], 0x07060302);
    }
}

// four f32 -> three exact bf16 planes, two bf16x2 words each
__device__ inline void split4(const float4& v, uint2& p0, uint2& p1, uint2& p2) {
    const float x[4] = {v.x, v.y, v.z, v.w};
    uint32_t h0[4], h1[4], h2[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const uint32_t u0 = __float_as_uint(x[e]) & 0xFFFF0000u;
        const float r1 = x[e] - __uint_as_float(u0);
        const uint32_t u1 = __float_as_uint(r1) & 0xFFFF0000u;
        h0[e] = u0;
        h1[e] = u1;
        h2[e] = __float_as_uint(r1 - __uint_as_float(u1));
    }
    p0 = make_uint2(__builtin_amdgcn_perm(h0[1], h0[0], 0x07060302), __builtin_amdgcn_perm(h0[3], h0[2], 0x07060302));
    p1 = make_uint2(__builtin_amdgcn_perm(h1[1], h1[0], 0x07060302), __builtin_amdgcn_perm(h1[3], h1[2], 0x07060302));
    p2 = make_uint2(__builtin_amdgcn_perm(h2[1], h2[0], 0x07060302), __builtin_amdgcn_perm(h2[3], h2[2], 0x07060302));
}

// a*b on split operands: the six products a_i*b_j with i + j <= 2; a0*b0 into hi,
// the rest into lo (both f32 accumulators; the result is hi + lo)
__device__ inline void mfma_split6(const u32x4 (&a)[3], const u32x4 (&b)[3], f32x16& hi, f32x16& lo) {
    hi = mfma_bf16(a[0], b[0], hi);
    lo = mfma_bf16(a[0], b[1], lo);
    lo = mfma_bf16(a[1], b[0], lo);
    lo = mfma_bf16(a[0], b[2], lo);
    lo = mfma_bf16(a[1], b[1], lo);
    lo = mfma_bf16(a[2], b[0], lo);
}

__host__ __device__ constexpr int fwd1_split_index(int c, int s, int p, int lane, int e) {
    return (((c * 2 + s) * 3 + p) * 64 + lane) * 8 + e;
}

// one element of the conv1 forward split packing (8 chunks x 2 steps x 64 lanes x 8)
__device__ inline void pack_fwd1_split_elem(const float* __restrict__ w, uint16_t* __restrict__ q, int t) {
    if (t >= 8 * 2 * 64 * 8) return;
    const int e = t & 7, lane = (t >> 3) & 63, s = (t >> 9) & 1, c = t >> 10;
    const int h = lane >> 5, co = lane & 31;
    const int k = (c >> 1) * 64 + (4 * (c & 1) + 2 * h + s) * 8 + e;  // natural (ci, ky, kx)
    uint16_t p0, p1, p2;
    split3(w[co * G1::K + k], p0, p1, p2);
    q[fwd1_split_index(c, s, 0, lane, e)] = p0;
    q[fwd1_split_index(c, s, 1, lane, e)] = p1;
    q[fwd1_split_index(c, s, 2, lane, e)] = p2;
}

constexpr int MS = 32;

struct WArgs {
    const void* x;        // layer input (u8 frames for conv1, NHWC f32 otherwise)
    long long sample_stride;  // conv1: bytes between samples
    const float* g;       // output grad, NHWC (batch, OH, OW, COUT), ReLU mask already applied
    float* slab;          // [splits][K][COUT]
    float* bslab;         // [splits][COUT]
    long long batch;
    long long px_per_split;
    int splits;
    // conv1 (u8) only: optional env-major rollout rows — sample n is row idx[n] of the
    // step-major (T, Nenv, ...) frame buffer x (the minibatch gather fused into the load)
    const long long* idx = nullptr;
    long long T = 0, Nenv = 0;
};

}  // namespace

namespace ppox_conv {
int split_pack23(const float* w2, const float* w3, uint16_t* q2, uint16_t* q3, uint16_t* qd2, uint16_t* qd3,
                 hipStream_t s);
int split_fwd23(int32_t layer, const void* x, int64_t batch, const uint16_t* wq, const float* bias, float* y,
                hipStream_t s);
}  // namespace ppox_conv
