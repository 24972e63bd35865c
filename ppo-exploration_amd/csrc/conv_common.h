// Definitions shared by the NatureCNN conv translation units (conv.hip: f32 MFMA and
// split-f16 kernels; conv_split.hip: the conv1 split forward) and the ICM kernels (the
// split-bf16 helpers).  Not part of the ABI.
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
    // split-f16 kernels: the A operand's amax slots (null: uint8 frames, exact at scale 1),
    // the output's amax slots (null: not recorded) and the packed B's scale exponent
    const uint32_t* amax_x = nullptr;
    uint32_t* amax_y = nullptr;
    const int* wexp = nullptr;
    // ReLU bitmasks (bit c of word p * (C / 32) + c / 32: channel c of pixel p > 0): written by the
    // split forwards (bits_y), read by the split dgrads instead of the f32 mask (bits_mask)
    uint32_t* bits_y = nullptr;
    const uint32_t* bits_mask = nullptr;
    // H1P operands (conv1's output as two f16 planes, h1 * 2^E = hi + lo): the exponent E of the
    // input (xexp: the split conv2 forward reads H1P) or of the output (yexp: the conv1 forward
    // writes it)
    const int* xexp = nullptr;
    const int* yexp = nullptr;
    // planes outputs of the sg2 producers (round 4: h2, h3, g3 — "PX", the H1P form generalised):
    // the output is written as two f16 planes at the exponent bound_exp() derives from the input's
    // amax (amax_x), the weights' norm slots (ynorm: 256 partial maxima of the weight matrix's
    // column l1-norms, pack tail) and the bias bound (ybias, nullable); the kernel stores it to
    // *yexp_out for the consumers
    int* yexp_out = nullptr;
    const uint32_t* ynorm = nullptr;
    const uint32_t* ybias = nullptr;
};

// H1P (conv1's output, the split conv2 operand): per pixel 32 hi then 32 lo f16 (128 B, the size
// of its f32 NHWC form); its exponent E (h1 * 2^E = hi + lo) lives in slot H1P_EXP_SLOT of the
// conv1 forward pack's tail, derived once per optimizer step from the bound
// |h1| <= 255 * max_c sum_k |W1[c][k]| + |b1[c]| (uint8 frames), so the conv1 forward can split
// its output in its epilogue without knowing the output's max
constexpr int H1P_EXP_SLOT = 1;  // + AMAX_SLOTS: after the weights' own exponent (h1p_exp below)

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

// ---- split-bf16 helpers (icm.hip: the ICM state encoder) ----
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

// ---- split-f16 ("f16x2") helpers: the NatureCNN conv / fc kernels ----------------------
// An f32 operand x of a GEMM is scaled by a power of two s (per tensor, from its running
// absolute maximum: max|x| s in [2^14, 2^15)) and split by round-to-nearest into two fp16
// planes:  h = rn16(x s),  l = rn16(x s - h)  (x s - h is exact in f32).  h + l carries 22+
// significant bits (|x s - h - l| <= 2^-24 |x s| while l is a normal fp16, i.e. for every
// |x| >= max|x| 2^-17; below that the error is an absolute 2^-25 / s, 2^-39 of the tensor's
// max).  A product is  hA hB + (hA lB + lA hB)  [+ lA lB <= 2^-22 |ab| dropped]: three
// v_mfma_f32_32x32x16_f16 (each product exact in f32), against six bf16 products for the
// same accuracy.  The accumulated result is unscaled by 1 / (sA sB) (exact: powers of two).
// uint8 frames (0..255) are exact in ONE fp16 plane (scale 1): conv1 needs two products.
using f16x8 = __attribute__((ext_vector_type(8))) _Float16;
using f16x2 = __attribute__((ext_vector_type(2))) _Float16;
using f32x2 = __attribute__((ext_vector_type(2))) float;
constexpr int NPL = 2;  // planes of a split f32 operand

__device__ inline f32x16 mfma_f16(const u32x4& a, const u32x4& b, const f32x16& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                  0);
}

// a*b on f16x2 operands: hA hB into hi, hA lB + lA hB into lo
__device__ inline void mfma_split3(const u32x4 (&a)[2], const u32x4 (&b)[2], f32x16& hi, f32x16& lo) {
    hi = mfma_f16(a[0], b[0], hi);
    lo = mfma_f16(a[0], b[1], lo);
    lo = mfma_f16(a[1], b[0], lo);
}

// Per-tensor absolute maxima ("amax"): AMAX_SLOTS uint32 (the f32 bits of max|x|: for
// non-negative floats uint order is float order), producers atomicMax one slot per wave
// (spread so no address takes more than a few thousand atomics), consumers reduce all
// slots.  The owner zeroes a tensor's slots before the kernel that produces it.
constexpr int AMAX_SLOTS = 256;

__device__ inline uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}
// every lane: max over the tensor's slots (one 16-B load per lane)
__device__ inline uint32_t amax_read(const uint32_t* __restrict__ am) {
    const uint4 v = reinterpret_cast<const uint4*>(am)[threadIdx.x & 63];
    return __builtin_amdgcn_readfirstlane(wave_max_u32(max(max(v.x, v.y), max(v.z, v.w))));
}
// this wave's maximum of |values| into slot (global wave index) mod AMAX_SLOTS; am may be null
__device__ inline void amax_record(uint32_t* __restrict__ am, float m) {
    if (!am) return;
    const uint32_t w = wave_max_u32(__float_as_uint(fabsf(m)));
    if ((threadIdx.x & 63) == 0) {
        const unsigned wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        atomicMax(am + (wid & (AMAX_SLOTS - 1)), w);
    }
}
// scale exponent of a tensor from its amax bits: max|x| 2^E in [2^14, 2^15) (E in [-113, 126];
// an all-zero or tiny tensor takes 2^126, an inf / nan one 2^-113 and stays non-finite)
__host__ __device__ inline int split_scale_exp(uint32_t amax_bits) {
    int e = (int)(amax_bits >> 23);
    e = e < 15 ? 15 : (e > 254 ? 254 : e);
    return 141 - e;
}
__host__ __device__ inline float exp2i(int e) { return __builtin_bit_cast(float, (uint32_t)(e + 127) << 23); }

// two f32 values times s -> their f16 high and low planes, packed f16x2 words (x.x low).  The
// scale is one v_pk_mul_f32 per pair; the residual x s - h is one v_fma_mix_f32 per value (h read
// as f16 straight from the packed word, times -1, plus x s: exact, so its rounding is none) —
// hipcc would emit a convert and a subtract
__device__ inline void split2h(f32x2 x, float s, uint32_t& h, uint32_t& l) {
    const f32x2 v = x * (f32x2){s, s};
    h = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2));
    float r0, r1;
    asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r0) : "v"(h), "v"(v.x));
    asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r1) : "v"(h), "v"(v.y));
    l = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){r0, r1}, f16x2));
}
// eight f32 times s -> their two f16 planes as MFMA fragments (element e = value e)
__device__ inline void split8h(const float4& v0, const float4& v1, float s, u32x4& p0, u32x4& p1) {
    uint32_t h[4], l[4];
    split2h((f32x2){v0.x, v0.y}, s, h[0], l[0]);
    split2h((f32x2){v0.z, v0.w}, s, h[1], l[1]);
    split2h((f32x2){v1.x, v1.y}, s, h[2], l[2]);
    split2h((f32x2){v1.z, v1.w}, s, h[3], l[3]);
    p0 = u32x4{h[0], h[1], h[2], h[3]};
    p1 = u32x4{l[0], l[1], l[2], l[3]};
}
// four f32 times s -> two f16 planes, two f16x2 words each
__device__ inline void split4h(const float4& v, float s, uint2& p0, uint2& p1) {
    split2h((f32x2){v.x, v.y}, s, p0.x, p1.x);
    split2h((f32x2){v.z, v.w}, s, p0.y, p1.y);
}
// ---- PX: f32 activations / gradients stored as their two f16 planes ---------------------
// A tensor of f32 layout (NHWC rows, channel runs of 32 aligned to 32 elements) is stored in the
// same bytes as, per 32-element group, the 32 high f16 then the 32 low f16 of its values times
// 2^E: element e's high half at uint16 index 2 (e & ~31) + (e & 31), its low half 32 further.  A
// 32-k chunk of an f32 GEMM operand row is then its two planes as they lie (conv1's H1P output is
// the first such tensor).  E comes from a bound on the values, so the producer can split in its
// epilogue: |y| <= amax(x) * max_n sum_k |W[k][n]| + max |b| (a ReLU or mask never increases it);
// the 2^-10 margin covers the f32 roundings of the kernel and of the bound itself.  A bound above
// the true amax only lowers the low plane's subnormal floor (absolute error 2^-25 2^-E per value).
__device__ inline int bound_exp(uint32_t amax_x, uint32_t norm, uint32_t bmax) {
    const float b = __uint_as_float(amax_x) * __uint_as_float(norm) + __uint_as_float(bmax);
    return split_scale_exp(__float_as_uint(b * (1.f + 1.f / 1024.f)));
}
// uint16 index of the high half of element e (its low half: + 32)
__host__ __device__ inline long long px_index(long long e) { return 2 * (e & ~31LL) + (e & 31); }
// one value v of a column pair (col, col ^ 1) held by lanes L, L ^ 1 (same row), scaled by s = 2^E:
// the 4-B word lane L stores after one DPP swap — the even lane the pair's two high halves, the odd
// lane their two low halves (at px_index(e_even) and px_index(e_even) + 32): as many 4-B stores as
// the f32 form.  Every lane of the wave must execute it (the swap reads the partner lane).
__device__ inline uint32_t px_pair_word(float v, float s, bool odd) {
    // the partner's value (quad_perm [1,0,3,2]), then the pair (even column first) split at once:
    // one packed scale, one packed convert per plane and one v_fma_mix per residual (split2h)
    const float pv = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
    uint32_t h, l;
    split2h(odd ? (f32x2){pv, v} : (f32x2){v, pv}, s, h, l);
    return odd ? l : h;
}
// the f32 value hi + lo (exact) of half H (0: low, 1: high) of a high-plane word and a low-plane word
__device__ inline float px_value(uint32_t hw, uint32_t lw, int H) {
    float r;
    if (H)
        asm("v_fma_mix_f32 %0, %1, 1.0, %2 op_sel:[1,0,1] op_sel_hi:[1,0,1]" : "=v"(r) : "v"(hw), "v"(lw));
    else
        asm("v_fma_mix_f32 %0, %1, 1.0, %2 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(hw), "v"(lw));
    return r;
}
// one f32 (scaled) -> its two f16 planes (the weight packers)
__device__ inline void split1h(float v, uint16_t& h, uint16_t& l) {
    const _Float16 hv = (_Float16)v;
    h = __builtin_bit_cast(uint16_t, hv);
    l = __builtin_bit_cast(uint16_t, (_Float16)(v - (float)hv));
}
// eight uint8 (two words) -> an f16x8 fragment, exact: f16 bits 0x64bb are 1024 + b, so one
// v_perm_b32 (bytes b, 0x64 of the constant word, b', 0x64) and one packed subtract per pair
__device__ inline u32x4 u8x8_to_f16(uint32_t w0, uint32_t w1) {
    const f16x2 k1024 = {(_Float16)1024.f, (_Float16)1024.f};
    const uint32_t q[4] = {__builtin_amdgcn_perm(0x64646464u, w0, 0x04010400), __builtin_amdgcn_perm(0x64646464u, w0, 0x04030402),
                           __builtin_amdgcn_perm(0x64646464u, w1, 0x04010400), __builtin_amdgcn_perm(0x64646464u, w1, 0x04030402)};
    u32x4 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(f16x2, q[i]) - k1024);
    return r;
}
// Tail of a packed buffer of `planes` uint16: PACK_TAIL32 uint32 — [0, AMAX_SLOTS) the amax
// partials of the source weights (written by wmax_kernel, read by the packer), then the scale
// exponent E the planes were packed with (read by the GEMM kernels).
constexpr int PACK_TAIL32 = 2 * AMAX_SLOTS + 8;
// tail slots after the exponent (AMAX_SLOTS): the H1P exponent (q1), the bias bound max |b| (q2, q3:
// float bits) and, from NORM_SLOT0, 256 partial maxima of the packed matrix's column l1-norms
// sum_k |B[k][n]| (float bits; q2, q3, qfcd: the PX output bounds, written by wmax_kernel)
constexpr int BMAX_SLOT = 2, NORM_SLOT0 = AMAX_SLOTS + 8;
__host__ __device__ inline uint32_t* pack_tail(uint16_t* q, long long planes) {
    return reinterpret_cast<uint32_t*>(q + planes);
}
__host__ __device__ inline const int* pack_exp(const uint16_t* q, long long planes) {
    return reinterpret_cast<const int*>(q + planes) + AMAX_SLOTS;
}
__host__ __device__ inline const uint32_t* pack_norm(const uint16_t* q, long long planes) {
    return reinterpret_cast<const uint32_t*>(q + planes) + NORM_SLOT0;
}
__host__ __device__ inline const uint32_t* pack_bmax(const uint16_t* q, long long planes) {
    return reinterpret_cast<const uint32_t*>(q + planes) + AMAX_SLOTS + BMAX_SLOT;
}
// the H1P exponent stored in the conv1 forward pack's tail (Args::xexp / yexp)
__host__ __device__ inline const int* h1p_exp(const uint16_t* q1, long long planes_q1) {
    return reinterpret_cast<const int*>(q1 + planes_q1) + AMAX_SLOTS + H1P_EXP_SLOT;
}


__host__ __device__ constexpr int fwd1_split_index(int c, int s, int p, int lane, int e) {
    return (((c * 2 + s) * NPL + p) * 64 + lane) * 8 + e;
}
constexpr int FWD1_PACK = 8 * 2 * NPL * 64 * 8;  // uint16 planes of the conv1 forward packing

// one element of the conv1 forward split packing (8 chunks x 2 steps x 64 lanes x 8), the
// weights times s
__device__ inline void pack_fwd1_split_elem(const float* __restrict__ w, float s, uint16_t* __restrict__ q, int t) {
    if (t >= 8 * 2 * 64 * 8) return;
    const int e = t & 7, lane = (t >> 3) & 63, st = (t >> 9) & 1, c = t >> 10;
    const int h = lane >> 5, co = lane & 31;
    const int k = (c >> 1) * 64 + (4 * (c & 1) + 2 * h + st) * 8 + e;  // natural (ci, ky, kx)
    uint16_t p0, p1;
    split1h(w[co * G1::K + k] * s, p0, p1);
    q[fwd1_split_index(c, st, 0, lane, e)] = p0;
    q[fwd1_split_index(c, st, 1, lane, e)] = p1;
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
    // split-f16: amax slots of X (null: uint8 frames) and of G
    const uint32_t* amax_x = nullptr;
    const uint32_t* amax_g = nullptr;
    // PX operands (f16 planes, conv_common.h): their exponents (the kernels' XPL / GPL forms)
    const int* xexp = nullptr;
    const int* gexp = nullptr;
};

}  // namespace

namespace ppox_conv {
int pack_split(const float* w1, const float* w2, const float* w3, uint16_t* q1, uint16_t* q2, uint16_t* q3,
               uint16_t* qd2, uint16_t* qd3, hipStream_t s);
long long planes(int which);  // uint16 planes of a split-packed form (1, 2, 3, 12, 13; 4 = fc)
int split_fwd23(int32_t layer, const void* x, int64_t batch, const uint16_t* wq, const float* bias, float* y,
                const uint32_t* amax_x, uint32_t* amax_y, uint32_t* relu_bits, const int* x_exp, int* y_exp_out,
                hipStream_t s);
// conv2 / conv3 forwards on planes (H1P / h2 -> h2 / h3 planes), the direct form (dconv.hip)
int dconv_fwd(int layer, const void* x, int64_t batch, const uint16_t* wq, const float* bias, float* y,
              const uint32_t* amax_x, uint32_t* amax_y, uint32_t* relu_bits, const int* x_exp, int* y_exp_out,
              hipStream_t s);
bool dconv_enabled(int layer, long long batch);
// the conv2 dgrad on PX g2 -> f32 g1 (conv1's ReLU bitmask applied), the direct class-wise form (dconv.hip)
int ddgrad2(const void* g2p, int64_t batch, const uint16_t* wqd2, float* g1, const uint32_t* relu_bits,
            uint32_t* amax_g1, const int* g_exp, const int* wexp, hipStream_t s);
// the fc dgrad on df planes -> g3 planes, the direct form (dconv.hip)
bool dfcd_enabled(long long batch);
int dfcd(const void* dfp, int64_t batch, const uint16_t* wq, float* g3, const uint32_t* amax_df, uint32_t* amax_g3,
         const uint32_t* relu_bits, int* g3_exp_out, const int* df_exp, const int* wexp, const uint32_t* ynorm,
         const uint32_t* ybias, hipStream_t s);
// ... split 8 ways over K into a slab [8][batch][512] (batches below fcw_enabled's)
bool fcw_sk_enabled(long long batch);
int fcw_sk(const void* h3p, int64_t batch, const uint16_t* q_fwd, float* slab, const int* h3_exp, const int* wexp,
           hipStream_t s);
constexpr int FCW_SPLITS = 8;
// the heads' backward to the fc output in one launch (dconv.hip hbw_kernel)
int head_backward(const float* dout, const float* wa, const float* dv, const float* wc, const float* e, const float* f,
                  const uint16_t* qhd, const int* wexp, int64_t rows, int n_out, float* df, float* de,
                  uint32_t* amax_de, uint32_t* amax_df, hipStream_t s);
// the fc forward on PX h3 in 256 x 128 tiles (dconv.hip)
bool fcw_enabled(long long batch);
int fcw(const void* h3p, int64_t batch, const uint16_t* q_fwd, const float* bias, float* f, uint32_t* amax_f,
        const int* h3_exp, const int* wexp, hipStream_t s);
// the conv3 dgrad on PX g3 -> PX g2 (conv2's ReLU bitmask applied), the direct form (dconv.hip)
bool ddgrad3_enabled(long long batch);
int ddgrad3(const void* g3p, int64_t batch, const uint16_t* wqd3, void* g2p, const uint32_t* amax_g3,
            uint32_t* amax_g2, const uint32_t* relu_bits, const int* g_exp, const int* wexp, const uint32_t* ynorm,
            const uint32_t* ybias, int* y_exp_out, hipStream_t s);
// the conv3 weight gradient on PX h2 and PX g3, the direct form (dconv.hip): per-workgroup partial slabs
// [grid][576][64] and bias slabs [grid][64], summed by the caller's wgrad_reduce; grid = dwgrad3_grid(batch)
bool dwgrad3_enabled(long long batch);
long long dwgrad3_grid(long long batch);
int dwgrad3(const void* h2p, const void* g3p, int64_t batch, const int* h_exp, const int* g_exp, float* slab,
            float* bslab, hipStream_t s);
}  // namespace ppox_conv
