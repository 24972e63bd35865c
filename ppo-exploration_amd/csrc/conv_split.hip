// K6, split-f16 form — the NatureCNN convolutions on the f16 matrix cores with fp32-class accuracy.
//
// Every f32 operand is scaled by a power of two and split into two f16 planes (conv_common.h, "split-f16"):
//   h = rn16(x s), l = rn16(x s - h)
// A product a*b is hA hB + (hA lB + lA hB), three v_mfma_f32_32x32x16_f16 with each product exact in f32.
// The hA hB terms accumulate in their own f32 accumulator and the small terms in a second one; the two are
// added once in the epilogue and unscaled by an exact power of two.  conv1's input is a uint8 frame (0..255),
// exact in ONE f16 plane, so the conv1 forward and weight gradient need only two products (x wh + x wl).
// Accuracy is therefore that of an f32 FMA chain up to summation order (tests: tests/test_kernels_gpu.py,
// split vs f32 MFMA vs fp64).  Same layers, layouts and fused epilogues as conv.hip.
#include <algorithm>

#include "conv_common.h"

namespace {

// ---------------------------------------------------------------------------
// conv1 forward, register-direct: each wave owns 32*MT output pixels x 32
// channels, no LDS.  K chunk c (32 values) = input channel c/2, kernel rows
// 4(c&1)..+3.  A lane of half h loads two 8-byte runs (kernel rows 4(c&1)+2h
// and +1); MFMA step s of the chunk takes the run of row 4(c&1)+2h+s, so the
// MFMA k index (s, h, e) is natural k = (c/2)*64 + (4(c&1) + 2h + s)*8 + e.
// The weights are packed in that order, plane by plane (pack_fwd1_split).
// ---------------------------------------------------------------------------

// Persistent: the whole split weight set (32 KB) is staged in LDS once per
// workgroup (B fragments then cost LDS, not TA, bandwidth), and each wave walks
// a contiguous range of row tiles.  The kernel is load-latency bound, so the
// input of the NEXT tile (all 8 chunks, 16*MT 8-byte loads per lane) is loaded while
// the current tile runs its 32*MT MFMAs.  Workgroups with adjacent row ranges
// share an XCD (xcd_remap): the overlapping input windows of one frame stack
// are read through one L2.
// PLANES: h1 is written as its two f16 planes (H1P: per pixel 32 hi then 32 lo f16, 128 B like f32),
// h1 * 2^E = hi + lo with E = *a.yexp (ppox_nature_pack_all: from the weight bound of conv1's
// output), the operand format of the split conv2 forward / weight gradient; its amax is recorded when
// a.amax_y is set (the bound of conv2's PX output)
// IDX (rows through the rollout index, round 3): each tile's idx values are loaded one tile ahead in
// inline asm (tile k + 1's during tile k's frame loads) and waited for by a counted vmcnt that leaves
// the 16 frame loads issued after them in flight; a plain load there made hipcc drain every load in
// flight (vmcnt(0)) at each tile to get the fresh idx value, then the frames' addresses.
__device__ inline uint32_t fwd1_idx_load(const long long* p) {
    uint32_t v;
    asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ uint32_t kFwd1Dummy[128];  // store target of the rows past the batch (never read)
constexpr int FWD1_FAST_EPI = 1;  // the H1P epilogue's whole-tile form (round 4); 0: the per-row form for every tile
// the H1P epilogue's stores non-temporal (streaming: h1 is read back from HBM by the conv2 forward
// and weight gradient, not from L2): 1-GPU line +1.0-1.2 % A/B (conv2 forward 281 -> 270 us at 16,384
// rows, the conv1 forward itself unchanged), profiles/r05y.  The direct kernels' stores made
// non-temporal the same way ran 4x slower (their counted vmcnt waits include the stores).
constexpr int FWD1_NT = 1;
__device__ inline void fwd1_store(uint32_t* p, uint32_t v) {
    if constexpr (FWD1_NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}
template <int MT, bool PLANES = false, bool IDX = false>
__global__ void __launch_bounds__(256, MT == 1 ? 3 : 2) fwd1_split_kernel(Args a, unsigned tiles_per_wave) {
    using L = G1;
    constexpr int NCH = L::K / 32, NQ = NCH * 2 * NPL;
    __shared__ u32x4 Wl[NQ * 64];
    {
        const u32x4* wq = reinterpret_cast<const u32x4*>(a.wp);
        for (int i = threadIdx.x; i < NQ * 64; i += 256) Wl[i] = wq[i];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned M = (unsigned)(a.batch * L::P);
    const unsigned ntile = (M + 32 * MT - 1) / (32 * MT);
    const unsigned wid = (unsigned)xcd_remap(blockIdx.x, gridDim.x) * 4 + wave;
    const unsigned t_begin = wid * tiles_per_wave;
    const unsigned t_end = min(ntile, t_begin + tiles_per_wave);
    if (t_begin >= t_end) return;  // wave-uniform; nothing below synchronises
    const uint8_t* x = reinterpret_cast<const uint8_t*>(a.x);
    const u32x4* Wlane = Wl + lane;

    // the whole K extent of a tile: per row slot i and chunk c, two 8-byte runs
    using Raw = uint32_t[MT][NCH][4];
    // IDX: this lane's rollout-row index of a tile's row slot i (clamped rows: the tile's first)
    auto idx_ptr = [&](unsigned tile, int i) {
        const unsigned m0 = tile * 32 * MT;
        unsigned m = m0 + i * 32 + (lane & 31);
        m = m < M ? m : m0;
        return a.idx + m / L::P;
    };
    uint32_t ixv[MT];  // IDX: the idx values of the tile about to be loaded
    if constexpr (IDX) {
#pragma unroll
        for (int i = 0; i < MT; ++i) ixv[i] = (uint32_t)*idx_ptr(t_begin, i);
    }
    const uint32_t T32 = (uint32_t)a.T, N32 = (uint32_t)a.Nenv;  // IDX: host-checked T * Nenv < 2^32
    auto load_tile = [&](unsigned tile, Raw& r) {
        const unsigned m0 = tile * 32 * MT;
        uint32_t ix[MT];
        if constexpr (IDX) {
            // this tile's idx values (loaded a tile ago; the 16 * MT frame loads of the tile after them
            // may stay in flight), then the next tile's, ahead of this tile's frame loads
#pragma unroll
            for (int i = 0; i < MT; ++i) ix[i] = ixv[i];
            if constexpr (MT == 1)
                asm volatile("s_waitcnt vmcnt(16)" : "+v"(ix[0]) :: "memory");
            else
                asm volatile("s_waitcnt vmcnt(32)" : "+v"(ix[0]), "+v"(ix[1]) :: "memory");
            const unsigned nt = tile + 1 < t_end ? tile + 1 : tile;
#pragma unroll
            for (int i = 0; i < MT; ++i) ixv[i] = fwd1_idx_load(idx_ptr(nt, i));
        }
#pragma unroll
        for (int i = 0; i < MT; ++i) {
            unsigned m = m0 + i * 32 + (lane & 31);
            m = m < M ? m : m0;  // clamped rows are computed but never stored
            const unsigned n = m / L::P, p = m - n * L::P, oy = p / L::OW, ox = p % L::OW;
            long long sb;
            if constexpr (IDX) {
                const uint32_t q = ix[i] / T32;
                sb = (long long)((ix[i] - q * T32) * N32 + q) * (long long)(L::CIN * L::IH * L::IW);
            } else {
                sb = u8_sample_base(a, n, (long long)L::CIN * L::IH * L::IW);
            }
            const uint8_t* b = x + sb + (oy * L::S + (lane >> 5) * 2) * L::IW + ox * L::S;
#pragma unroll
            for (int c = 0; c < NCH; ++c) {
                const uint8_t* q = b + (c >> 1) * (L::IH * L::IW) + (c & 1) * 4 * L::IW;
                const uint2 v0 = *reinterpret_cast<const uint2*>(q);
                const uint2 v1 = *reinterpret_cast<const uint2*>(q + L::IW);
                r[i][c][0] = v0.x;
                r[i][c][1] = v0.y;
                r[i][c][2] = v1.x;
                r[i][c][3] = v1.y;
            }
        }
    };
    const int co = lane & 31;
    const float bias = a.bias[co];
    const float uw = exp2i(-*a.wexp);  // the weights were packed times 2^E; frames are exact
    const float sy = PLANES ? exp2i(*a.yexp) : 1.f;  // H1P output scale
    float om = 0.f;                    // the largest value this lane stored (h1's amax)
    auto run_tile = [&](unsigned tile, const Raw& r) {
        f32x16 hi[MT], lo[MT];
#pragma unroll
        for (int i = 0; i < MT; ++i) hi[i] = lo[i] = zero16();
        // B fragments are read from LDS one (chunk, step) ahead of their MFMAs
        u32x4 rb[2][NPL];
#pragma unroll
        for (int p = 0; p < NPL; ++p) rb[0][p] = Wlane[p * 64];
#pragma unroll
        for (int c = 0; c < NCH; ++c)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int q = c * 2 + s, cur = q & 1;
                if (q + 1 < 2 * NCH) {
#pragma unroll
                    for (int p = 0; p < NPL; ++p) rb[cur ^ 1][p] = Wlane[((q + 1) * NPL + p) * 64];
                }
#pragma unroll
                for (int i = 0; i < MT; ++i) {
                    const u32x4 av = u8x8_to_f16(r[i][c][2 * s], r[i][c][2 * s + 1]);
                    hi[i] = mfma_f16(av, rb[cur][0], hi[i]);
                    lo[i] = mfma_f16(av, rb[cur][1], lo[i]);
                }
                // keep the scheduler from hoisting every chunk's LDS reads (192 VGPRs)
                __builtin_amdgcn_sched_barrier(0);
            }
        const unsigned m0 = tile * 32 * MT;
        // C/D map: col = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5).  The ReLU
        // bitmask word of tile row L (its 32 channels) is half (L >> 2) & 1 of the ballot of
        // element e = (L & 3) + 4 * (L >> 3): lane L < 32 collects it and stores it
        const int eL = (lane & 3) + 4 * ((lane >> 3) & 3), hL = (lane >> 2) & 1;
        if constexpr (PLANES && FWD1_FAST_EPI) {
            if (m0 + 32 * MT <= M) {  // uniform: a whole tile (every tile but a ragged last one)
                // rows e, e + 1 (consecutive) as one pair: the value math on packed f32x2, their two
                // splits in one split2h, one DPP swap of the hi and of the lo words for both rows, and
                // v_perm_b32 assembles the even lane's (hi co, hi co + 1) and the odd lane's (lo co - 1,
                // lo co) words; the stores are one base address plus immediate row offsets (no
                // per-row 64-bit address arithmetic, no clamp).  Bitwise the rounding of the form below.
                const bool odd = co & 1;
                const f32x2 uw2 = {uw, uw}, b2 = {bias, bias};
#pragma unroll
                for (int i = 0; i < MT; ++i) {
                    uint32_t word = 0;
                    uint16_t* yb = reinterpret_cast<uint16_t*>(a.y) +
                                   (long long)(m0 + i * 32 + 4 * (lane >> 5)) * (2 * L::COUT) +
                                   (odd ? L::COUT + co - 1 : co);
#pragma unroll
                    for (int e = 0; e < 16; e += 2) {
                        f32x2 v2 = ((f32x2){hi[i][e], hi[i][e + 1]} + (f32x2){lo[i][e], lo[i][e + 1]}) * uw2 + b2;
                        v2.x = fmaxf(v2.x, 0.f);
                        v2.y = fmaxf(v2.y, 0.f);
                        om = fmaxf(om, fmaxf(v2.x, v2.y));
                        uint32_t h, l;
                        split2h(v2, sy, h, l);
                        const uint32_t ph = (uint32_t)__builtin_amdgcn_mov_dpp((int)h, 0xB1, 0xF, 0xF, false);
                        const uint32_t pl = (uint32_t)__builtin_amdgcn_mov_dpp((int)l, 0xB1, 0xF, 0xF, false);
                        const uint32_t lo_w = odd ? pl : h, hi_w = odd ? l : ph;  // (low half, high half) sources
                        const int r0 = (e & 3) + 8 * (e >> 2);                    // row of e; e + 1 is the next
                        fwd1_store(reinterpret_cast<uint32_t*>(yb + r0 * (2 * L::COUT)),
                                   __builtin_amdgcn_perm(hi_w, lo_w, 0x05040100u));
                        fwd1_store(reinterpret_cast<uint32_t*>(yb + (r0 + 1) * (2 * L::COUT)),
                                   __builtin_amdgcn_perm(hi_w, lo_w, 0x07060302u));
                        if (a.bits_y) {  // uniform
                            const unsigned long long b0 = __ballot(v2.x > 0.f), b1 = __ballot(v2.y > 0.f);
                            word = eL == e ? (uint32_t)(hL ? b0 >> 32 : b0) : word;
                            word = eL == e + 1 ? (uint32_t)(hL ? b1 >> 32 : b1) : word;
                        }
                    }
                    const unsigned mw = m0 + i * 32 + lane;
                    if (a.bits_y)  // uniform
                        *(lane < 32 ? a.bits_y + mw : kFwd1Dummy + 64 + lane) = word;
                }
                return;
            }
        }
#pragma unroll
        for (int i = 0; i < MT; ++i) {
            uint32_t word = 0;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const unsigned m = m0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
                const float v = fmaxf((hi[i][e] + lo[i][e]) * uw + bias, 0.f);
                om = fmaxf(om, v);  // a row past the end recomputed row m0, which is stored
                if constexpr (PLANES) {
                    // channel pairs (co, co ^ 1) sit in lanes L, L ^ 1: one DPP swap, then the even
                    // lane stores the pair's hi halves and the odd lane their lo halves, 4 B each, so a
                    // row is two 64-B runs of 4-byte stores (as many store instructions as f32)
                    const float vs = v * sy;
                    const _Float16 hv = (_Float16)vs;
                    const _Float16 lv = (_Float16)(vs - (float)hv);  // exact in f32
                    const uint32_t w = (uint32_t)__builtin_bit_cast(uint16_t, hv) |
                                       ((uint32_t)__builtin_bit_cast(uint16_t, lv) << 16);
                    const uint32_t pw = (uint32_t)__builtin_amdgcn_mov_dpp((int)w, 0xB1, 0xF, 0xF, false);  // [1,0,3,2]
                    const bool odd = co & 1;
                    const uint32_t out = odd ? ((pw >> 16) | (w & 0xFFFF0000u)) : ((w & 0xFFFFu) | (pw << 16));
                    uint16_t* y16 = reinterpret_cast<uint16_t*>(a.y) + (long long)m * (2 * L::COUT) +
                                    (odd ? L::COUT + co - 1 : co);
                    // unconditional (rows past the end go to a dummy word): no branch, so hipcc's
                    // waits on the next tile's frame loads keep their counts
                    *reinterpret_cast<uint32_t*>(m < M ? y16 : reinterpret_cast<uint16_t*>(kFwd1Dummy + lane)) = out;
                } else {
                    *(m < M ? a.y + (long long)m * L::COUT + co : reinterpret_cast<float*>(kFwd1Dummy + lane)) = v;
                }
                if (a.bits_y) {  // uniform
                    const unsigned long long b = __ballot(v > 0.f);
                    word = eL == e ? (uint32_t)(hL ? b >> 32 : b) : word;
                }
            }
            const unsigned mw = m0 + i * 32 + lane;
            if (a.bits_y)  // uniform
                *(lane < 32 && mw < M ? a.bits_y + mw : kFwd1Dummy + 64 + lane) = word;
        }
    };
    // the next tile's loads unconditional (past the last tile: the last again, never run), so every
    // run_tile waits for its own loads only, with the next tile's in flight
    Raw r0, r1;
    load_tile(t_begin, r0);
#pragma unroll 1
    for (unsigned tile = t_begin; tile < t_end; tile += 2) {
        load_tile(tile + 1 < t_end ? tile + 1 : t_end - 1, r1);
        run_tile(tile, r0);
        if (tile + 1 >= t_end) break;
        load_tile(tile + 2 < t_end ? tile + 2 : t_end - 1, r0);
        run_tile(tile + 1, r1);
    }
    amax_record(a.amax_y, om);  // (H1P: the bound of conv2's PX output starts from it)
}

constexpr int SPLIT_FWD1_MT = 1;
// waves the persistent kernel spreads its tiles over: 256 CUs x resident waves per CU
// (VGPRs: 3 workgroups at MT = 1, 140 VGPRs; 2 at MT = 2; 32 KB of LDS each)
constexpr int SPLIT_RESIDENT_WAVES = SPLIT_FWD1_MT == 1 ? 3072 : 2048;
// below 8,192 rows: 2,048 waves (more tiles per wave over which its weight staging and pipeline fill
// are spread; per-rank shape 199.6 vs 201.3-201.7 ms, same box; the 16,384-row line unchanged)
inline long long fwd1_waves(long long batch, long long ntile) {
    return std::min<long long>(ntile, batch < 8192 ? std::min(2048, SPLIT_RESIDENT_WAVES) : SPLIT_RESIDENT_WAVES);
}

}  // namespace

// conv1 forward writing H1P (see fwd1_split_kernel<MT, true>): h1 as its two f16 planes at the
// exponent the weight packing derived (ppox_nature_pack_all with b1)
extern "C" int ppox_nature_conv1_fwd_planes(const void* x, int64_t batch, const int64_t* idx, int64_t T,
                                            int64_t N_env, int64_t x_sample_stride, const uint16_t* wq1,
                                            const float* bias, uint16_t* h1p, uint32_t* amax_y, uint32_t* relu_bits,
                                            void* stream) {
    if (batch == 0) return PPOX_OK;
    PPOX_REQUIRE(x && wq1 && bias && h1p && batch > 0, "ppox_nature_conv1_fwd_planes: bad arguments");
    PPOX_REQUIRE(ppox::aligned16(wq1), "ppox_nature_conv1_fwd_planes: packed weights must be 16-byte aligned");
    PPOX_REQUIRE(batch * G1::P < (1LL << 31), "ppox_nature_conv1_fwd_planes: batch too large for 32-bit rows");
    PPOX_REQUIRE(!(reinterpret_cast<uintptr_t>(x) & 3) && (idx || x_sample_stride % 4 == 0),
                 "ppox_nature_conv1_fwd_planes: u8 input must be 4-byte aligned");
    if (idx) PPOX_REQUIRE(T > 0 && N_env > 0 && T * N_env < (1LL << 31), "ppox_nature_conv1_fwd_planes: idx needs T and N_env (T * N_env < 2^31)");
    const long long pl = ppox_conv::planes(1);
    Args a{x, reinterpret_cast<const long long*>(idx), T, N_env, x_sample_stride, nullptr, bias, nullptr,
           reinterpret_cast<float*>(h1p), batch, nullptr, amax_y, pack_exp(wq1, pl)};
    a.wp = reinterpret_cast<const float*>(wq1);
    a.bits_y = relu_bits;
    a.yexp = h1p_exp(wq1, pl);
    constexpr int MT = SPLIT_FWD1_MT;
    const long long ntile = ppox::ceil_div(batch * G1::P, 32 * MT);
    const long long waves = fwd1_waves(batch, ntile);
    const unsigned per = ppox::ceil_div(ntile, waves);
    if (idx)
        fwd1_split_kernel<MT, true, true><<<ppox::ceil_div(ppox::ceil_div(ntile, per), 4), 256, 0,
                                            ppox::as_stream(stream)>>>(a, per);
    else
        fwd1_split_kernel<MT, true><<<ppox::ceil_div(ppox::ceil_div(ntile, per), 4), 256, 0, ppox::as_stream(stream)>>>(
            a, per);
    PPOX_LAUNCHED("ppox_nature_conv1_fwd_planes");
}

extern "C" int64_t ppox_nature_split_pack_elems(int32_t which) {
    const long long p = (which >= 1 && which <= 3) || which == 12 || which == 13 ? ppox_conv::planes(which) : -1;
    return p < 0 ? -1 : p + 2 * PACK_TAIL32;  // + the tail (amax partials, scale exponent)
}

extern "C" int ppox_nature_pack_split(const float* w1, const float* w2, const float* w3, uint16_t* q1, uint16_t* q2,
                                      uint16_t* q3, uint16_t* qd2, uint16_t* qd3, void* stream) {
    // any packed buffer may be null: that packing is skipped
    PPOX_REQUIRE((!q1 || w1) && (!q2 || w2) && (!q3 || w3) && (!qd2 || w2) && (!qd3 || w3),
                 "ppox_nature_pack_split: null weights");
    return ppox_conv::pack_split(w1, w2, w3, q1, q2, q3, qd2, qd3, ppox::as_stream(stream));
}

extern "C" int ppox_nature_conv_fwd_split(int32_t layer, const void* x, int64_t batch, const int64_t* idx, int64_t T,
                                          int64_t N_env, int64_t x_sample_stride, const uint16_t* wq,
                                          const float* bias, float* y, const uint32_t* amax_x, uint32_t* amax_y,
                                          uint32_t* relu_bits, const int* x_exp, int* y_exp_out, void* stream) {
    if (batch == 0) return PPOX_OK;  // empty shard / minibatch: no pointers to check
    PPOX_REQUIRE(layer >= 1 && layer <= 3, "ppox_nature_conv_fwd_split: layer must be 1, 2 or 3");
    PPOX_REQUIRE(x && wq && bias && y && batch >= 0, "ppox_nature_conv_fwd_split: bad arguments");
    PPOX_REQUIRE(ppox::aligned16(wq), "ppox_nature_conv_fwd_split: packed weights must be 16-byte aligned");
    if (layer != 1) {
        PPOX_REQUIRE(!idx, "ppox_nature_conv_fwd_split: idx is for layer 1 only");
        return ppox_conv::split_fwd23(layer, x, batch, wq, bias, y, amax_x, amax_y, relu_bits, x_exp, y_exp_out,
                                      ppox::as_stream(stream));
    }
    PPOX_REQUIRE(!amax_x, "ppox_nature_conv_fwd_split: layer 1 reads uint8 frames (no amax_x)");
    PPOX_REQUIRE(!x_exp && !y_exp_out, "ppox_nature_conv_fwd_split: layer 1's planes output is ppox_nature_conv1_fwd_planes");
    PPOX_REQUIRE(batch * G1::P < (1LL << 31), "ppox_nature_conv_fwd_split: batch too large for 32-bit rows");
    Args a{x, reinterpret_cast<const long long*>(idx), T, N_env, x_sample_stride, nullptr, bias, nullptr, y, batch,
           nullptr, amax_y, pack_exp(wq, ppox_conv::planes(1))};
    a.wp = reinterpret_cast<const float*>(wq);
    a.bits_y = relu_bits;
    hipStream_t s = ppox::as_stream(stream);
    PPOX_REQUIRE(!(reinterpret_cast<uintptr_t>(x) & 3) && (idx || x_sample_stride % 4 == 0),
                 "ppox_nature_conv_fwd_split: u8 input must be 4-byte aligned");
    if (idx) PPOX_REQUIRE(T > 0 && N_env > 0 && T * N_env < (1LL << 31), "ppox_nature_conv_fwd_split: idx needs T and N_env (T * N_env < 2^31)");
    constexpr int MT = SPLIT_FWD1_MT;
    const long long ntile = ppox::ceil_div(batch * G1::P, 32 * MT);
    const long long waves = fwd1_waves(batch, ntile);
    const unsigned per = ppox::ceil_div(ntile, waves);
    if (idx)
        fwd1_split_kernel<MT, false, true><<<ppox::ceil_div(ppox::ceil_div(ntile, per), 4), 256, 0, s>>>(a, per);
    else
        fwd1_split_kernel<MT><<<ppox::ceil_div(ppox::ceil_div(ntile, per), 4), 256, 0, s>>>(a, per);
    PPOX_LAUNCHED("ppox_nature_conv_fwd_split");
}
