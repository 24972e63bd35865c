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
};

}  // namespace
