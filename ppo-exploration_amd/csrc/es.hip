// ES-NSRA population evaluation and update (evolution_strategies.py:137-246, the
// reference's EvolutionStrategy: perturb -> evaluate each perturbation's episode
// return -> rank-free normalised-reward ES gradient, plus the novelty term).
//
// ppox_es_noise      eps[p][j] ~ N(0,1) f64 (Philox counter (j/2, GLOBAL member, gen, tag),
//                    Box-Muller on two 53-bit uniforms) — shard-invariant; the reference
//                    draws np.random.randn per member and layer (:176-186)
// ppox_es_env_noise  the synthetic env's shared per-step noise table xi[t][i]
// ppox_es_evaluate   one WAVE per member: theta = w + sigma*eps_p lives in registers (lane
//                    l holds weight column l of each layer: W0[:, l], W1[:, l], W2[l, :]),
//                    the member's whole episode (T steps of arctan-MLP policy + tanh head,
//                    evolution_strategies.py:50-63, and the env step) runs inside the
//                    kernel; small vectors (state, hidden activations, action) are
//                    exchanged through the wave's LDS slot.  -> fitness (episode return),
//                    behaviour characterisation (final state[0:2], the qpos[0:2] analogue
//                    of get_behavior_char :248-271)
// ppox_es_update     delta[j] = sum_p c[p] eps[p][j]  (the P^T r GEMV of :237-242 with
//                    c folding the reward / novelty mix), fixed-order two-pass reduction
// Everything is float64, as the reference's numpy program.
#include <algorithm>
#include <cmath>

#include "common.h"
#include "philox.h"

namespace {

constexpr uint32_t ENV_B_TAG = 0xB0B0B0B0u, ENV_NOISE_TAG = 0xE0E0E0E0u, EPS_TAG = 0xE5E5E5E5u;
constexpr int HMAX = 64;

__device__ inline double u53(uint32_t hi, uint32_t lo) {
    return ((double)(hi >> 5) * 67108864.0 + (double)(lo >> 6)) * 0x1.0p-53;
}

__global__ void __launch_bounds__(256) es_noise_kernel(long long P, long long n, long long member0, uint32_t gen,
                                                       uint32_t k0, uint32_t k1, double* __restrict__ eps) {
    const long long q2 = (n + 1) / 2;
    const long long total = P * q2;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const long long p = i / q2, q = i - p * q2;
        const ppox::u32x4 w =
            ppox::philox4x32_10(ppox::u32x4{(uint32_t)q, (uint32_t)(member0 + p), gen, EPS_TAG}, k0, k1);
        const double u1 = u53(w.x, w.y) + 0x1.0p-53;  // (0, 1]
        const double u2 = u53(w.z, w.w);
        const double r = sqrt(-2.0 * log(u1));
        const double th = 2.0 * M_PI * u2;
        double* e = eps + p * n + 2 * q;
        e[0] = r * cos(th);
        if (2 * q + 1 < n) e[1] = r * sin(th);
    }
}

__global__ void __launch_bounds__(256) es_env_noise_kernel(int T, int D, uint32_t k0, uint32_t k1,
                                                           double* __restrict__ xi) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= T * D) return;
    const int t = i / D, d = i - t * D;
    const ppox::u32x4 w = ppox::philox4x32_10(ppox::u32x4{(uint32_t)d, (uint32_t)t, ENV_NOISE_TAG, 0u}, k0, k1);
    xi[i] = (double)ppox::u01(w.x) - 0.5;
}

// order this wave's LDS accesses (all exchanges here are within one wave)
__device__ inline void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ inline double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// sizes: D (obs) <= DM, H1, H2 <= 64, A <= AM; weights w: W0 [D][H1], W1 [H1][H2], W2 [H2][A]
// (numpy row-major, concatenated), eps likewise per member (nullable: evaluate w itself)
template <int DM, int AM>
__global__ void __launch_bounds__(256) es_eval_kernel(const double* __restrict__ w, const double* __restrict__ eps,
                                                      double sigma, long long P, int D, int H1, int H2, int A, int T,
                                                      uint32_t k0, uint32_t k1, const double* __restrict__ xi,
                                                      double* __restrict__ fitness, double* __restrict__ bc) {
    __shared__ double sh[4][HMAX + DM + AM];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long p = (long long)blockIdx.x * 4 + wv;
    if (p >= P) return;  // wave-uniform; only wave-local LDS below
    double* hs = sh[wv];         // hidden activation exchange
    double* ss = sh[wv] + HMAX;  // state
    double* as = ss + DM;        // action
    const long long n = (long long)D * H1 + (long long)H1 * H2 + (long long)H2 * A;
    const double* ep = eps ? eps + p * n : nullptr;
    auto theta = [&](long long j) { return ep ? w[j] + sigma * ep[j] : w[j]; };
    // this lane's weight columns (zero beyond the layer sizes)
    double w0[DM], w1[HMAX], w2[AM];
#pragma unroll
    for (int i = 0; i < DM; ++i) w0[i] = (i < D && lane < H1) ? theta((long long)i * H1 + lane) : 0.0;
#pragma unroll
    for (int k = 0; k < HMAX; ++k)
        w1[k] = (k < H1 && lane < H2) ? theta((long long)D * H1 + (long long)k * H2 + lane) : 0.0;
#pragma unroll
    for (int j = 0; j < AM; ++j)
        w2[j] = (j < A && lane < H2) ? theta((long long)D * H1 + (long long)H1 * H2 + (long long)lane * A + j) : 0.0;
    // env matrix row of this lane's state component
    double brow[AM];
#pragma unroll
    for (int j = 0; j < AM; ++j) {
        const ppox::u32x4 r = ppox::philox4x32_10(ppox::u32x4{(uint32_t)lane, (uint32_t)j, ENV_B_TAG, 0u}, k0, k1);
        brow[j] = (r.x & 1u) ? 1.0 : -1.0;
    }
    if (lane < DM) ss[lane] = 0.0;
    wave_sync();
    double fit = 0.0;
    for (int t = 0; t < T; ++t) {
        // layer 0: h1 = arctan(s @ W0)
        double acc = 0.0;
#pragma unroll
        for (int i = 0; i < DM; ++i)
            if (i < D) acc = acc + ss[i] * w0[i];
        const double h1 = lane < H1 ? atan(acc) : 0.0;
        wave_sync();
        hs[lane] = h1;
        wave_sync();
        // layer 1: h2 = arctan(h1 @ W1) — four interleaved fma chains (the 64-term dot is
        // otherwise one dependent add chain per step; numpy's BLAS dot reassociates too)
        double c0 = 0.0, c1 = 0.0, c2 = 0.0, c3 = 0.0;
#pragma unroll
        for (int k = 0; k < HMAX; k += 4) {
            if (k < H1) c0 = fma(hs[k], w1[k], c0);
            if (k + 1 < H1) c1 = fma(hs[k + 1], w1[k + 1], c1);
            if (k + 2 < H1) c2 = fma(hs[k + 2], w1[k + 2], c2);
            if (k + 3 < H1) c3 = fma(hs[k + 3], w1[k + 3], c3);
        }
        const double h2 = lane < H2 ? atan((c0 + c1) + (c2 + c3)) : 0.0;
        // head: a = tanh(h2 @ W2)
        double a2 = 0.0;
#pragma unroll
        for (int j = 0; j < AM; ++j) {
            if (j < A) {
                const double aj = tanh(wave_sum(h2 * w2[j]));
                if (lane == 0) as[j] = aj;
                a2 = a2 + aj * aj;
            }
        }
        wave_sync();
        // env: s' = 0.9 s + 0.1 B a + 0.02 xi_t ; r = s'[0] - 0.05 |a|^2
        if (lane < D) {
            double ba = 0.0;
#pragma unroll
            for (int j = 0; j < AM; ++j)
                if (j < A) ba = ba + brow[j] * as[j];
            const double s = ss[lane];
            ss[lane] = (0.9 * s + 0.1 * ba) + 0.02 * xi[(long long)t * D + lane];
        }
        wave_sync();
        fit = fit + (ss[0] - 0.05 * a2);
    }
    if (lane == 0) {
        fitness[p] = fit;
        if (bc) {
            bc[2 * p] = ss[0];
            bc[2 * p + 1] = D > 1 ? ss[1] : 0.0;
        }
    }
}

// pass 1: partial[c][j] = sum over members of chunk c (in order) of coef[p] * eps[p][j]
__global__ void __launch_bounds__(256) es_update_partial(const double* __restrict__ eps, const double* __restrict__ coef,
                                                         long long P, long long n, int chunk,
                                                         double* __restrict__ partial) {
    const long long j = (long long)blockIdx.x * 256 + threadIdx.x;
    const int c = blockIdx.y;
    if (j >= n) return;
    const long long p0 = (long long)c * chunk, p1 = p0 + chunk < P ? p0 + chunk : P;
    double s = 0.0;
    for (long long p = p0; p < p1; ++p) s = s + coef[p] * eps[p * n + j];
    partial[(long long)c * n + j] = s;
}

__global__ void __launch_bounds__(256) es_update_final(const double* __restrict__ partial, int nchunk, long long n,
                                                       double* __restrict__ out) {
    const long long j = (long long)blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    double s = 0.0;
    for (int c = 0; c < nchunk; ++c) s = s + partial[(long long)c * n + j];
    out[j] = s;
}

constexpr int UPD_CHUNK = 128;

}  // namespace

extern "C" int ppox_es_noise(int64_t P, int64_t n_params, int64_t member0, int64_t generation, uint64_t seed,
                             double* eps, void* stream) {
    PPOX_REQUIRE(eps && P > 0 && n_params > 0 && member0 >= 0, "ppox_es_noise: bad arguments");
    const long long total = P * ((n_params + 1) / 2);
    const unsigned blocks = (unsigned)std::min<long long>((total + 255) / 256, 16384);
    es_noise_kernel<<<blocks, 256, 0, ppox::as_stream(stream)>>>(P, n_params, member0, (uint32_t)generation,
                                                                 (uint32_t)seed, (uint32_t)(seed >> 32), eps);
    PPOX_LAUNCHED("ppox_es_noise");
}

extern "C" int ppox_es_env_noise(int32_t T, int32_t D, uint64_t env_seed, double* xi, void* stream) {
    PPOX_REQUIRE(xi && T > 0 && D > 0, "ppox_es_env_noise: bad arguments");
    es_env_noise_kernel<<<ppox::ceil_div((long long)T * D, 256), 256, 0, ppox::as_stream(stream)>>>(
        T, D, (uint32_t)env_seed, (uint32_t)(env_seed >> 32), xi);
    PPOX_LAUNCHED("ppox_es_env_noise");
}

extern "C" int ppox_es_evaluate(const double* w, const double* eps, double sigma, int64_t P, int32_t D, int32_t H1,
                                int32_t H2, int32_t A, int32_t T, uint64_t env_seed, const double* xi, double* fitness,
                                double* bc, void* stream) {
    PPOX_REQUIRE(w && xi && fitness && P > 0 && T > 0, "ppox_es_evaluate: bad arguments");
    PPOX_REQUIRE(D >= 1 && D <= 32 && H1 >= 1 && H1 <= HMAX && H2 >= 1 && H2 <= HMAX && A >= 1 && A <= 8,
                 "ppox_es_evaluate: sizes must satisfy D <= 32, hidden <= 64, A <= 8 (two hidden layers)");
    const unsigned blocks = ppox::ceil_div(P, 4);
    hipStream_t s = ppox::as_stream(stream);
    const uint32_t k0 = (uint32_t)env_seed, k1 = (uint32_t)(env_seed >> 32);
    if (D <= 8 && A <= 2)
        es_eval_kernel<8, 2><<<blocks, 256, 0, s>>>(w, eps, sigma, P, D, H1, H2, A, T, k0, k1, xi, fitness, bc);
    else
        es_eval_kernel<32, 8><<<blocks, 256, 0, s>>>(w, eps, sigma, P, D, H1, H2, A, T, k0, k1, xi, fitness, bc);
    PPOX_LAUNCHED("ppox_es_evaluate");
}

extern "C" int64_t ppox_es_update_workspace_bytes(int64_t P, int64_t n_params) {
    return ((P + UPD_CHUNK - 1) / UPD_CHUNK) * n_params * (int64_t)sizeof(double);
}

extern "C" int ppox_es_update(const double* eps, const double* coef, int64_t P, int64_t n_params, double* workspace,
                              int64_t workspace_bytes, double* out, void* stream) {
    PPOX_REQUIRE(eps && coef && workspace && out && P > 0 && n_params > 0, "ppox_es_update: bad arguments");
    PPOX_REQUIRE(workspace_bytes >= ppox_es_update_workspace_bytes(P, n_params), "ppox_es_update: workspace too small");
    const int nchunk = (int)((P + UPD_CHUNK - 1) / UPD_CHUNK);
    PPOX_REQUIRE(nchunk <= 65535, "ppox_es_update: population too large");
    hipStream_t s = ppox::as_stream(stream);
    es_update_partial<<<dim3(ppox::ceil_div(n_params, 256), nchunk), 256, 0, s>>>(eps, coef, P, n_params, UPD_CHUNK,
                                                                                    workspace);
    PPOX_LAUNCHED_NORET("ppox_es_update");
    es_update_final<<<ppox::ceil_div(n_params, 256), 256, 0, s>>>(workspace, nchunk, n_params, out);
    PPOX_LAUNCHED("ppox_es_update");
}
