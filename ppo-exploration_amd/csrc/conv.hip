// K6 — NatureCNN convolutions as implicit GEMMs on the fp32 matrix cores
// (v_mfma_f32_32x32x2_f32: exact f32 FMAs, the gfx950 fp32 matrix rate,
// 157 TF/s dense).  Replaces torch.nn.Conv2d + ReLU of
// .ipynb_checkpoints/models-checkpoint.py:52-58 (conv1 4->32 k8 s4,
// conv2 32->64 k4 s2, conv3 64->64 k3 s1 on 84x84x4 frames).
//
// GEMM view of one layer: M = batch*OH*OW output pixels, N = COUT, K = CIN*KH*KW.
//   A[m][k]  im2col of the input, gathered on the fly (never materialised)
//   B[k][co] weights, pre-packed once per optimizer step into the kernel's K order
// One 256-thread workgroup owns BM = 128 output pixels x all COUT channels; each
// wave 32 pixels x COUT (COUT/32 MFMA tiles).  K is walked in BK = 32 chunks,
// register-staged and double-buffered in LDS (one barrier per chunk), so the
// global gathers of chunk c+1 fly under the MFMAs of chunk c.
// Epilogue fuses + bias and ReLU and writes NHWC (conv1, conv2 — the next
// layer's gather reads 128-B channel rows) or NCHW (conv3 — the reference's
// Flatten order feeding Linear(3136, 512)).
//
// Input layouts: conv1 reads the uint8 frame stack (N, 4, 84, 84) directly (the
// reference's torch.FloatTensor(obs) conversion is fused: u8 -> f32 is exact),
// through an env-major index list when given (the minibatch gather is fused too).
#include "common.h"

namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;

constexpr int BM = 128;
constexpr int BK = 32;
constexpr int AST = BK + 1;  // padded LDS row stride (floats): conflict-free column reads

struct ConvArgs {
    const void* x;          // input activations
    const long long* idx;   // optional env-major row indices (conv1 only): sample b = rollout row idx[b]
    long long T, Nenv;      // rollout dims for idx mapping
    long long x_sample_stride;  // elements between samples when idx == nullptr
    const float* wp;        // packed weights [K][COUT]
    const float* bias;      // [COUT]
    float* y;               // output
    long long batch;        // samples
};

template <int CIN_, int IH_, int IW_, int KH_, int KW_, int S_, int COUT_, bool IN_U8_NCHW, bool OUT_NCHW>
struct Layer {
    static constexpr int CIN = CIN_, IH = IH_, IW = IW_, KH = KH_, KW = KW_, S = S_, COUT = COUT_;
    static constexpr bool OUT_NCHW_ = OUT_NCHW;
    static constexpr int OH = (IH - KH) / S + 1;
    static constexpr int OW = (IW - KW) / S + 1;
    static constexpr int P = OH * OW;
    static constexpr int K = CIN * KH * KW;
    static constexpr int NCHUNK = K / BK;
    static constexpr int NT = COUT / 32;
    static_assert(K % BK == 0, "K must be a multiple of BK");
    static_assert(COUT % 32 == 0, "COUT must be a multiple of 32");
};

// ---- A staging: global -> registers -> LDS -----------------------------------
// f32 NHWC input: K order (ky, kx, ci); a chunk is 32 consecutive channels of one
// (ky, kx) tap, i.e. one 128-byte row segment per output pixel.
template <class L>
struct StageF32 {
    float4 r[4];
    __device__ inline void load(const ConvArgs& a, long long m0, long long M, int chunk) {
        constexpr int CPT = L::CIN / BK;  // chunks per tap
        const int tap = chunk / CPT, ci0 = (chunk % CPT) * BK;
        const int ky = tap / L::KW, kx = tap % L::KW;
        const float* x = reinterpret_cast<const float*>(a.x);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int w = i * 256 + threadIdx.x;
            const int row = w >> 3, q = w & 7;
            const long long m = m0 + row;
            if (m < M) {
                const long long n = m / L::P;
                const int p = (int)(m - n * L::P);
                const int oy = p / L::OW, ox = p % L::OW;
                const float* src = x + ((n * L::IH + (oy * L::S + ky)) * L::IW + (ox * L::S + kx)) * L::CIN + ci0;
                r[i] = reinterpret_cast<const float4*>(src)[q];
            } else {
                r[i] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
    }
    __device__ inline void store(float* As) const {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int w = i * 256 + threadIdx.x;
            const int row = w >> 3, q = w & 7;
            float* d = As + row * AST + q * 4;
            d[0] = r[i].x;
            d[1] = r[i].y;
            d[2] = r[i].z;
            d[3] = r[i].w;
        }
    }
};

// u8 NCHW frame input (conv1): K order (ci, ky, kx) = the weight's own order; a
// chunk is one channel x 4 kernel rows x 8 columns: 4 runs of 8 bytes per pixel.
template <class L>
struct StageU8 {
    uint32_t r[4];
    __device__ inline void load(const ConvArgs& a, long long m0, long long M, int chunk) {
        const int ci = chunk / (L::KH / 4), ky0 = (chunk % (L::KH / 4)) * 4;
        const uint8_t* x = reinterpret_cast<const uint8_t*>(a.x);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int w = i * 256 + threadIdx.x;
            const int row = w >> 3, seg = (w & 7) >> 1, half = w & 1;
            const long long m = m0 + row;
            if (m < M) {
                const long long n = m / L::P;
                const int p = (int)(m - n * L::P);
                const int oy = p / L::OW, ox = p % L::OW;
                long long base;
                if (a.idx) {
                    const long long i_env = a.idx[n];
                    base = ((i_env % a.T) * a.Nenv + i_env / a.T) * (long long)(L::CIN * L::IH * L::IW);
                } else {
                    base = n * a.x_sample_stride;
                }
                const uint8_t* src = x + base + (ci * L::IH + oy * L::S + ky0 + seg) * L::IW + ox * L::S + half * 4;
                r[i] = *reinterpret_cast<const uint32_t*>(src);
            } else {
                r[i] = 0u;
            }
        }
    }
    __device__ inline void store(float* As) const {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int w = i * 256 + threadIdx.x;
            const int row = w >> 3, seg = (w & 7) >> 1, half = w & 1;
            float* d = As + row * AST + seg * 8 + half * 4;
            d[0] = (float)(r[i] & 0xFFu);
            d[1] = (float)((r[i] >> 8) & 0xFFu);
            d[2] = (float)((r[i] >> 16) & 0xFFu);
            d[3] = (float)(r[i] >> 24);
        }
    }
};

template <class L>
struct StageB {
    static constexpr int V = BK * L::COUT / 4 / 256;  // float4 per thread
    float4 r[V];
    __device__ inline void load(const float* wp, int chunk) {
        const float4* src = reinterpret_cast<const float4*>(wp + (long long)chunk * BK * L::COUT);
#pragma unroll
        for (int i = 0; i < V; ++i) r[i] = src[i * 256 + threadIdx.x];
    }
    __device__ inline void store(float* Bs) const {
#pragma unroll
        for (int i = 0; i < V; ++i) reinterpret_cast<float4*>(Bs)[i * 256 + threadIdx.x] = r[i];
    }
};

template <class L, class SA>
__global__ void __launch_bounds__(256, 2) conv_fwd_kernel(ConvArgs a) {
    __shared__ float As[2][BM * AST];
    __shared__ __attribute__((aligned(16))) float Bs[2][BK * L::COUT];
    const long long M = a.batch * L::P;
    const long long m0 = (long long)blockIdx.x * BM;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;

    f32x16 acc[L::NT];
#pragma unroll
    for (int j = 0; j < L::NT; ++j) acc[j] = f32x16{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

    SA sa;
    StageB<L> sb;
    sa.load(a, m0, M, 0);
    sb.load(a.wp, 0);
    sa.store(As[0]);
    sb.store(Bs[0]);
    __syncthreads();

    const int arow = wave * 32 + (lane & 31);
    const int khalf = lane >> 5;
    for (int c = 0; c < L::NCHUNK; ++c) {
        const int cur = c & 1;
        if (c + 1 < L::NCHUNK) {
            sa.load(a, m0, M, c + 1);
            sb.load(a.wp, c + 1);
        }
        const float* A = As[cur] + arow * AST + khalf;
        const float* B = Bs[cur] + khalf * L::COUT + (lane & 31);
#pragma unroll
        for (int kk = 0; kk < BK / 2; ++kk) {
            const float av = A[kk * 2];
#pragma unroll
            for (int j = 0; j < L::NT; ++j) {
                const float bv = B[kk * 2 * L::COUT + j * 32];
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[j], 0, 0, 0);
            }
        }
        if (c + 1 < L::NCHUNK) {
            sa.store(As[cur ^ 1]);
            sb.store(Bs[cur ^ 1]);
        }
        __syncthreads();
    }

    // epilogue: bias + ReLU, C/D map col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
    for (int j = 0; j < L::NT; ++j) {
        const int co = j * 32 + (lane & 31);
        const float b = a.bias[co];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            const long long m = m0 + row;
            if (m < M) {
                const float v = fmaxf(acc[j][r] + b, 0.f);
                if constexpr (L::OUT_NCHW_) {
                    const long long n = m / L::P;
                    const int p = (int)(m - n * L::P);
                    a.y[(n * L::COUT + co) * L::P + p] = v;
                } else {
                    a.y[m * L::COUT + co] = v;
                }
            }
        }
    }
}

// pack PyTorch weights [COUT][CIN][KH][KW] into [K][COUT] in the kernel's K order
template <int CIN, int KH, int KW, int COUT, bool NHWC_ORDER>
__global__ void pack_kernel(const float* __restrict__ w, float* __restrict__ wp) {
    constexpr int K = CIN * KH * KW;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= K * COUT) return;
    const int k = i / COUT, co = i % COUT;
    int ci, ky, kx;
    if (NHWC_ORDER) {
        ci = k % CIN;
        const int tap = k / CIN;
        ky = tap / KW;
        kx = tap % KW;
    } else {
        kx = k % KW;
        ky = (k / KW) % KH;
        ci = k / (KW * KH);
    }
    wp[i] = w[((co * CIN + ci) * KH + ky) * KW + kx];
}

}  // namespace

namespace {
using Conv1 = Layer<4, 84, 84, 8, 8, 4, 32, true, false>;   // -> (B, 20, 20, 32) NHWC
using Conv2 = Layer<32, 20, 20, 4, 4, 2, 64, false, false>;  // -> (B, 9, 9, 64) NHWC
using Conv3 = Layer<64, 9, 9, 3, 3, 1, 64, false, true>;     // -> (B, 64, 7, 7) NCHW
}  // namespace

extern "C" int ppox_nature_pack_weights(const float* w1, const float* w2, const float* w3, float* wp1, float* wp2,
                                        float* wp3, void* stream) {
    PPOX_REQUIRE(w1 && w2 && w3 && wp1 && wp2 && wp3, "ppox_nature_pack_weights: null pointer");
    PPOX_REQUIRE(ppox::aligned16(wp1) && ppox::aligned16(wp2) && ppox::aligned16(wp3),
                 "ppox_nature_pack_weights: packed buffers must be 16-byte aligned");
    hipStream_t s = ppox::as_stream(stream);
    pack_kernel<4, 8, 8, 32, false><<<ppox::ceil_div(256 * 32, 256), 256, 0, s>>>(w1, wp1);
    pack_kernel<32, 4, 4, 64, true><<<ppox::ceil_div(512 * 64, 256), 256, 0, s>>>(w2, wp2);
    pack_kernel<64, 3, 3, 64, true><<<ppox::ceil_div(576 * 64, 256), 256, 0, s>>>(w3, wp3);
    PPOX_LAUNCHED("ppox_nature_pack_weights");
}

extern "C" int ppox_nature_conv_fwd(int32_t layer, const void* x, int64_t batch, const int64_t* idx, int64_t T,
                                    int64_t N_env, int64_t x_sample_stride, const float* wp, const float* bias,
                                    float* y, void* stream) {
    PPOX_REQUIRE(layer >= 1 && layer <= 3, "ppox_nature_conv_fwd: layer must be 1, 2 or 3");
    PPOX_REQUIRE(x && wp && bias && y && batch >= 0, "ppox_nature_conv_fwd: bad arguments");
    PPOX_REQUIRE(ppox::aligned16(wp), "ppox_nature_conv_fwd: packed weights must be 16-byte aligned");
    if (batch == 0) return PPOX_OK;
    ConvArgs a{x, reinterpret_cast<const long long*>(idx), T, N_env, x_sample_stride, wp, bias, y, batch};
    hipStream_t s = ppox::as_stream(stream);
    if (layer == 1) {
        PPOX_REQUIRE(!(reinterpret_cast<uintptr_t>(x) & 3) && (idx || x_sample_stride % 4 == 0),
                     "ppox_nature_conv_fwd: u8 input must be 4-byte aligned");
        if (idx) PPOX_REQUIRE(T > 0 && N_env > 0, "ppox_nature_conv_fwd: idx needs T and N_env");
        const long long M = batch * Conv1::P;
        conv_fwd_kernel<Conv1, StageU8<Conv1>><<<ppox::ceil_div(M, BM), 256, 0, s>>>(a);
    } else if (layer == 2) {
        PPOX_REQUIRE(ppox::aligned16(x) && !idx, "ppox_nature_conv_fwd: layer 2 input must be 16B aligned NHWC");
        const long long M = batch * Conv2::P;
        conv_fwd_kernel<Conv2, StageF32<Conv2>><<<ppox::ceil_div(M, BM), 256, 0, s>>>(a);
    } else {
        PPOX_REQUIRE(ppox::aligned16(x) && !idx, "ppox_nature_conv_fwd: layer 3 input must be 16B aligned NHWC");
        const long long M = batch * Conv3::P;
        conv_fwd_kernel<Conv3, StageF32<Conv3>><<<ppox::ceil_div(M, BM), 256, 0, s>>>(a);
    }
    PPOX_LAUNCHED("ppox_nature_conv_fwd");
}
