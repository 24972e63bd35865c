// Direct split-f16 convolution forwards for conv2 and conv3 (round 4; .ipynb_checkpoints/
// models-checkpoint.py:55-57, Conv2d(32, 64, 4, stride 2) / Conv2d(64, 64, 3, stride 1), each + ReLU):
// the weights live in registers, the input images in LDS.
//
// Why: the im2col GEMM (sgemm_kernel<SgFwd2P> / <SgFwd<G3>>) stages every 128-row tile's A rows
// (im2col: each input pixel copied up to 4 / 9 times) and the whole packed weight matrix (131 / 147
// KB) through L2 -> LDS, 426 / 442 KB per tile; at the ~70 GB/s per CU that LDS-DMA path sustains,
// staging, not the MFMA, bounds it.  Here each CU
//   * holds the packed B (64 columns x K, hi / lo f16 planes) in VGPRs: wave w keeps the 32 columns of
//     column tile j = w & 1 — NCH chunks x 2 k-steps x 2 planes fragments (conv2: 64 = 256 VGPRs,
//     conv3: 72 = 288), loaded once per launch;
//   * streams whole input sample images (PX / H1P planes: conv3 81 pixels x 256 B, conv2 400 x 128 B)
//     into an LDS ring by LDS-DMA, each pixel read from HBM once;
//   * walks its contiguous range of samples in phases of 64 output rows (rows = (sample, oy, ox), the
//     im2col rows): wave w computes the 32-row block rg = w >> 1 of the phase for its column tile,
//     the A fragments read straight from the images (implicit im2col: a row's tap (ky, kx) is the
//     pixel (S oy + ky, S ox + kx) of its sample's image, 16 B per lane and plane).
// Same MFMA sequence as the GEMM (its chunk order — conv2's taps in input-parity classes — and per
// chunk k-steps 0, 1: hi += aH bH, lo += aH bL, lo += aL bH, mfma_split3), so the output is bitwise
// the sg2 kernel's (tests/test_dconv_gpu.py).
// LDS image layout (bank-conflict-free fragment reads): a 16-lane ds_read_b128 lane group reads 16
// rows whose index m (within the workgroup's range) is distinct mod 16, one 16-B piece each.  Every
// pixel gets a key from its coordinates such that a row's pixel at tap (ky, kx) has key
// (m + const(tap)) & 15 — conv3: key(n, y, x) = (n + 7 y + x) & 15 (m = 49 n + 7 oy + ox, 49 = 1 mod 16);
// conv2: key(n, y, x) = (n + 9 (y >> 1) + (x >> 1)) & 15 (m = 81 n + 9 oy + ox).  conv3 pixels are 256 B
// (all 64 banks): piece p is stored at p ^ key.  conv2 pixels are 128 B (half the banks): the pixel
// pair (x, x ^ 1) is swapped when key & 1 (the bank half), piece p stored at p ^ (key >> 1).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <utility>

#include "conv_common.h"

namespace {

// the direct kernels' activation / gradient outputs: plain stores (non-temporal ones ran the kernels 4x slower:
// their counted vmcnt waits include the stores, which then wait for HBM — DESIGN §4.1)
__device__ inline void out_store2(void* p, uint32_t x, uint32_t y) { *reinterpret_cast<uint2*>(p) = make_uint2(x, y); }

constexpr int DC_PD = 2;  // k-steps of A-fragment reads in flight ahead of the MFMAs

// conv3: h2 planes (81 pixels x 64 channels: per pixel hi[0:32] lo[0:32] hi[32:64] lo[32:64])
struct DcF3 {
    using L = G3;
    static constexpr int PIXB = 256, NPIX = 81, DMAS = 6, NSLOT = 7, NCH = 18;
    static constexpr int NA = 60;  // B fragments (of 72) kept in AGPRs
    // chunk c: tap c >> 1, channel group c & 1
    static constexpr int tap(int c) { return c >> 1; }
    static constexpr int bchunk(int c) { return c; }
    static constexpr int group(int c) { return c & 1; }
};
// conv2: H1P (400 pixels x 32 channels: per pixel hi[0:32] lo[0:32]); chunk c = one tap, walked in
// the sg2 kernel's input-parity classes (SgFwd::tap_of, SG_FWD2_PARITY)
struct DcF2 {
    using L = G2;
    static constexpr int PIXB = 128, NPIX = 400, DMAS = 13, NSLOT = 3, NCH = 16;
    static constexpr int NA = 64;  // B fragments (of 64) kept in AGPRs
    static constexpr int tap(int c) {
        const int cls = c >> 2, i = c & 3;
        return ((cls >> 1) + 2 * (i >> 1)) * 4 + (cls & 1) + 2 * (i & 1);
    }
    static constexpr int bchunk(int c) { return tap(c); }
    static constexpr int group(int) { return 0; }
};

template <class F>
struct DcGeo {
    static constexpr int IMG = F::NPIX * F::PIXB;              // bytes per sample image
    static constexpr int REAL_DMAS = (IMG + 1023) / 1024;      // 1-KB DMAs that cover it
    // a ring slot: the image's 1-KB DMAs (a wave's DMAs past the last re-copy it: the same bytes to the
    // same place)
    static constexpr int SLOT = REAL_DMAS * 1024;
    static constexpr int BIAS = F::NSLOT * SLOT;  // the output's 64 scaled biases
    static constexpr int LDS = BIAS + 64 * 4;
    static_assert(REAL_DMAS <= 4 * F::DMAS, "dconv: the image fits its DMAs");
    static_assert(LDS <= 160 * 1024, "dconv: LDS");
    static_assert(F::L::P % 16 == 1, "dconv: the row key is m mod 16");
};

// one buffer LDS-DMA of 16 B per lane: descriptor over [base, base + bytes) (uniform), lane offset, sample offset
// (a helper: the builtins written in a kernel template's body made hipcc drop the template's host stubs)
__device__ inline void dc_buffer_dma(const void* base, int bytes, uint8_t* dst, uint32_t voff, int soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(__builtin_amdgcn_make_buffer_rsrc((void*)base, 0, bytes, 0x00020000),
                                             (__attribute__((address_space(3))) void*)dst, 16, voff, soff, 0, 0);
}

template <class Fn, int... I>
__device__ inline void dc_unroll(Fn&& fn, std::integer_sequence<int, I...>) {
    (fn(std::integral_constant<int, I>{}), ...);
}

template <int OFF>
__device__ inline u32x4 dc_read(uint32_t addr) {
    u32x4 r;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
    return r;
}
template <int N>
__device__ inline void dc_lgkm(u32x4& a, u32x4& b) {
    asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N));
}
template <int N>
__device__ inline void dc_lgkm(u32x4& a, u32x4& b, u32x4& c) {
    asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(a), "+v"(b), "+v"(c) : "n"(N));
}
// wait until at most D k of this wave's vector-memory operations are outstanding (k uniform, < 4)
template <int D>
__device__ inline void dc_vm_wait(int k) {
    static_assert(3 * D < 64, "vmcnt is 6 bits");
    if (k <= 0)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (k == 1)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D) : "memory");
    else if (k == 2)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * D) : "memory");
    else
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * D) : "memory");
}

// MFMA as inline asm, so the operands' register files are explicit: the weights are srcA (AGPRs, "a": the
// fragments of chunks below F::NA, else VGPRs), the image fragment srcB and the accumulators VGPRs.  The
// output tile is then channels x pixels (lane (r, h): pixel r, channels (q & 3) + 8 (q >> 2) + 4 h), so a
// lane holds runs of 4 adjacent channels of one pixel: the PX epilogue stores 8-B plane runs with no
// cross-lane exchange.  Per output element the products and their k order are the GEMM's (a x^T w sum
// either way).  hipcc does not know these are MFMAs: VALU reads of an accumulator are padded by hand
// (dc_acc_fence), and an accumulator is never written by the VALU (the first k-step takes C = 0).
// PAD: the srcB fragment was just written by the VALU (a fragment split in registers): the 2 wait
// states a VALU write -> MFMA operand read needs go inside the string (hipcc pads nothing in asm)
template <bool BA, bool PAD = false>
__device__ inline void dc_mfma(f32x16& c, const u32x4& x, const u32x4& w) {
    if constexpr (BA && PAD)
        asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %2, %1, %0" : "+v"(c) : "v"(x), "a"(w));
    else if constexpr (BA)
        asm volatile("v_mfma_f32_32x32x16_f16 %0, %2, %1, %0" : "+v"(c) : "v"(x), "a"(w));
    else
        asm volatile("v_mfma_f32_32x32x16_f16 %0, %2, %1, %0" : "+v"(c) : "v"(x), "v"(w));
}
template <bool BA, bool PAD = false>
__device__ inline void dc_mfma0(f32x16& c, const u32x4& x, const u32x4& w) {  // c = w x
    if constexpr (BA && PAD)
        asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %2, %1, 0" : "=&v"(c) : "v"(x), "a"(w));
    else if constexpr (BA)
        asm volatile("v_mfma_f32_32x32x16_f16 %0, %2, %1, 0" : "=&v"(c) : "v"(x), "a"(w));
    else
        asm volatile("v_mfma_f32_32x32x16_f16 %0, %2, %1, 0" : "=&v"(c) : "v"(x), "v"(w));
}
// >= 18 wait states between a 16-pass MFMA writing an accumulator and a VALU reading it
__device__ inline void dc_acc_fence(f32x16& h, f32x16& l) {
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" : "+v"(h), "+v"(l));
}

// BITS: write the output's ReLU bitmask (a.bits_y).  Input planes (a.x, exponent *a.xexp), output
// planes (exponent from the bound, as the sg2 PX epilogue: *a.yexp_out by workgroup 0).
template <class F, bool BITS>
__global__ void __launch_bounds__(256, 1) dconv_fwd_kernel(Args a, const u32x4* __restrict__ wq) {
    using L = typename F::L;
    using Gm = DcGeo<F>;
    constexpr int NK = 2 * F::NCH;  // k-steps
    __shared__ __attribute__((aligned(16))) uint8_t lds[Gm::LDS];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int j = wave & 1, rg = wave >> 1;  // column tile, row block of a phase
    const int r = lane & 31, h = lane >> 5;
    const long long S0 = blockIdx.x * a.batch / gridDim.x, S1 = (blockIdx.x + 1) * a.batch / gridDim.x;
    const int NS = (int)(S1 - S0);
    if (NS <= 0) return;
    const int MR = NS * L::P;  // rows of the range
    const int F_ = (MR + 63) / 64;
    const uint8_t* xb = reinterpret_cast<const uint8_t*>(a.x) + S0 * Gm::IMG;
    const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)lds);

    // DMA d = wave + 4 i (i < DMAS) of a sample covers slot bytes [1024 d, 1024 d + 1024) (past the
    // image: the last DMA again, or its last pixel, into the slot's pad); lane -> LDS pixel u, piece
    // position pos; the source pixel / piece follow from the sample's key
    int dpk[F::DMAS];  // LDS pixel u (low 16 bits) | its key offset << 16
#pragma unroll
    for (int i = 0; i < F::DMAS; ++i) {
        int d = wave + 4 * i;
        d = d < Gm::REAL_DMAS ? d : Gm::REAL_DMAS - 1;
        const int b = d * 1024 + lane * 16;
        int u = b / F::PIXB;
        u = u < F::NPIX ? u : F::NPIX - 1;
        const int y = u / L::IW, x = u % L::IW;
        dpk[i] = u | ((L::S == 1 ? L::OW * y + x : 9 * (y >> 1) + (x >> 1)) << 16);
    }
    // DMA i of sample n (range-relative): a buffer LDS-DMA — the range's descriptor (uniform), the sample in
    // soffset, the lane's 32-bit offset in voffset (no 64-bit address arithmetic per DMA; round 4 used
    // global_load_lds)
    auto issue_one = [&](int n, int i) {
        int d = wave + 4 * i;
        d = d < Gm::REAL_DMAS ? d : Gm::REAL_DMAS - 1;
        const int key = (n + (dpk[i] >> 16)) & 15, u = dpk[i] & 0xFFFF;
        uint32_t off;
        if constexpr (F::PIXB == 256) {
            off = (uint32_t)(u * 256 + (((lane & 15) ^ key) << 4));
        } else {  // conv2: the pixel pair swapped by key & 1, the piece by key >> 1
            off = (uint32_t)((u ^ (key & 1)) * 128 + (((lane & 7) ^ (key >> 1)) << 4));
        }
        uint8_t* dst = lds + (n % F::NSLOT) * Gm::SLOT + d * 1024;
        dc_buffer_dma(xb, NS * Gm::IMG, dst, off, n * Gm::IMG);
    };
    auto issue_sample = [&](int n) {
#pragma unroll
        for (int i = 0; i < F::DMAS; ++i) issue_one(n, i);
    };
    // prologue: the first samples' DMAs, then the weights, the bias, the scales
    int issued = NS < F::NSLOT ? NS : F::NSLOT;
    for (int n = 0; n < issued; ++n) issue_sample(n);
    u32x4 bq[F::NCH][2][2];
#pragma unroll
    for (int c = 0; c < F::NCH; ++c)
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int p = 0; p < 2; ++p) bq[c][s][p] = wq[((((F::bchunk(c) * 2 + s) * 2 + j) * 2 + p) * 64) + lane];
    const int ex = *a.xexp, ew = *a.wexp;
    const uint32_t am = amax_read(a.amax_x), nm = amax_read(a.ynorm), bm = *a.ybias;
    const int ey = bound_exp(am, nm, bm);
    const float bnd = __uint_as_float(am) * __uint_as_float(nm) + __uint_as_float(bm);
    const float sy = __builtin_isfinite(bnd) ? exp2i(ey) : __builtin_nanf("");
    // the epilogue in the output's scaled domain: y = relu((x ua) (uw sy) + bias sy) is the sg2 form's
    // relu((x ua) uw + bias) sy exactly (powers of two), and its planes are y's split
    const float ua = exp2i(-ex), uws = exp2i(-ew) * sy;
    if (threadIdx.x < 64) reinterpret_cast<float*>(lds + Gm::BIAS)[threadIdx.x] = a.bias[threadIdx.x] * sy;
    if (blockIdx.x == 0 && threadIdx.x == 0) *a.yexp_out = ey;
    __builtin_amdgcn_s_waitcnt(0);  // everything above landed (hipcc's own bookkeeping sees it)
    __syncthreads();                // (the biases)
    asm volatile("s_nop 4" ::: "memory");  // (VALU-written B registers before the first MFMA reads them)

    // output planes: pixel row p of the range at byte 256 p; lane (r, h) of column tile j writes channels
    // 8 t + 4 h .. + 3 of it (t = q >> 2): high plane 8 B at 128 j + 16 t + 8 h, low plane 64 B further
    uint8_t* yb = reinterpret_cast<uint8_t*>(a.y) + 2 * px_index(S0 * L::P * 64);
    const uint32_t ylane = (uint32_t)(r * 256 + 128 * j + 8 * h);
    const uint32_t bias_lane = lds0 + Gm::BIAS + (uint32_t)((j * 32 + 4 * h) * 4);
    uint32_t* bits = BITS ? a.bits_y + S0 * L::P * 2 : nullptr;
    uint32_t om = 0u;  // the largest stored scaled value's bits (values >= 0)
    f32x16 H0, L0, H1, L1;

    // epilogue group t (accumulator elements 4 t .. 4 t + 3) of the 32-pixel block at range row pmb:
    // epi_val: the four scaled values (bs: their scaled biases, read from LDS a k-step before);
    // epi_store: their planes' two 8-B runs; epi_mask: the amax and the ReLU bits.  FULL: every row of the
    // block is in the range (else the lane's pixel pmb + r must be)
    auto epi_val = [&](auto T, const f32x16& PH, const f32x16& PL, const u32x4& bs, float (&y)[4]) {
        constexpr int t = decltype(T)::value;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            y[k] = fmaxf((PH[4 * t + k] + PL[4 * t + k]) * ua * uws + __uint_as_float(bs[k]), 0.f);
    };
    auto epi_store = [&](auto T, auto FULL, int pmb, const float (&y)[4]) {
        constexpr int t = decltype(T)::value;
        uint32_t hw[2], lw[2];
        split2h((f32x2){y[0], y[1]}, 1.f, hw[0], lw[0]);
        split2h((f32x2){y[2], y[3]}, 1.f, hw[1], lw[1]);
        uint8_t* dst = yb + ((uint32_t)pmb * 256u + ylane + 16 * t);
        if (decltype(FULL)::value || pmb + r < MR) {
            out_store2(dst, hw[0], hw[1]);
            out_store2(dst + 64, lw[0], lw[1]);
        }
    };
    auto epi_mask = [&](auto T, const float (&y)[4], int& bw) {
        constexpr int t = decltype(T)::value;
        const uint32_t u0 = __float_as_uint(y[0]), u1 = __float_as_uint(y[1]), u2 = __float_as_uint(y[2]),
                       u3 = __float_as_uint(y[3]);
        om = max(om, max(max(u0, u1), max(u2, u3)) & 0x7FFFFFFFu);
        if constexpr (BITS) {
#pragma unroll
            for (int k = 0; k < 4; ++k) bw |= y[k] > 0.f ? (1 << (8 * t + k)) : 0;
        }
    };
    // the bitmask word of the lane's pixel: its half (channels 4 h + 8 t + k) joined with lane r ^ 32's
    auto epi_bits = [&](auto FULL, int pmb, int bw) {
        if constexpr (BITS) {
            const uint32_t w = (uint32_t)(bw << (4 * h)) | (uint32_t)(__shfl_xor(bw, 32) << (4 * (1 - h)));
            if (lane < 32 && (decltype(FULL)::value || pmb + r < MR)) bits[(pmb + r) * 2 + j] = w;
        }
    };
    // refill DMAs of a phase: up to RMAX samples, DMA x = t * DMAS + i at k-step 16 + x (NK - 16) / (RMAX DMAS),
    // after the epilogue's stores (k-steps 0-16), so the next wait's younger operations are the DMAs
    constexpr int RMAX = 2, NDMA = RMAX * F::DMAS;
    static_assert(NK > 17, "dconv: the epilogue's k-steps");

    // phase f: accumulate its rows into (H, Lo); the previous phase's (PH, PL) epilogue (when prev) rides
    // along the k walk.  Samples this phase reads: [nlo, nhi]; their DMAs waited for (the later samples'
    // may stay in flight: samples are issued in order, and any store issued after them only makes the
    // count more conservative), then one barrier: every wave's DMAs landed, every wave done with phase
    // f - 1's fragment reads
    auto phase = [&](int f, f32x16& H, f32x16& Lo, const f32x16& PH, const f32x16& PL, auto PREV) {
        const int m0 = 64 * f;
        const int nlo = m0 / L::P, nhi = min((m0 + 63) / L::P, NS - 1);
        dc_vm_wait<F::DMAS>(issued - 1 - nhi);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        // refill: samples up to nlo + NSLOT - 1 (the slots of samples < nlo are free), issued inside the
        // k walk
        const int rA = issued, nref = min(nlo + F::NSLOT, NS) - issued;
        issued += nref;
        // this lane's A row: m = m0 + 32 rg + r (past the range: its last row, never stored)
        int m = m0 + 32 * rg + r;
        m = m < MR ? m : MR - 1;
        const int n = m / L::P, p = m - n * L::P, oy = p / L::OW, ox = p - oy * L::OW;
        const uint32_t base = lds0 + (n % F::NSLOT) * Gm::SLOT + (L::S * oy * L::IW + L::S * ox) * F::PIXB;
        const int key0 = m & 15;  // the row's key (P = 1 mod 16)
        // k-step i = 2 c + s: its plane-pl fragment address (the tap's pixel offset: the immediate)
        auto addr = [&](int i, int pl) {
            const int c = i >> 1, s = i & 1, tap = F::tap(c), ky = tap / L::KW, kx = tap % L::KW;
            const uint32_t P16 = (uint32_t)((F::group(c) << 3) | (pl << 2) | (s << 1)) << 4;
            if constexpr (F::PIXB == 256) {
                const uint32_t kt = (uint32_t)(((key0 + L::OW * ky + kx) & 15) ^ h) << 4;
                return base + (P16 ^ kt);
            } else {
                // pixel x = 2 ox + kx (low bit kx & 1) flipped by key & 1: +-128 B
                const int key = (key0 + 9 * (ky >> 1) + (kx >> 1)) & 15;
                const uint32_t kt = (uint32_t)((key >> 1) ^ h) << 4;
                const uint32_t bt = base + (uint32_t)((key & 1) * ((kx & 1) ? -128 : 128));
                return bt + (P16 ^ kt);
            }
        };
        constexpr int PD = DC_PD, NB = PD + 1;  // k-steps of fragment reads in flight, buffers
        u32x4 fa[NB][2];
        auto rd = [&](auto I) {
            constexpr int i = decltype(I)::value;
            constexpr int tap = F::tap(i >> 1), off = ((tap / L::KW) * L::IW + tap % L::KW) * F::PIXB;
            fa[i % NB][0] = dc_read<off>(addr(i, 0));
            fa[i % NB][1] = dc_read<off>(addr(i, 1));
        };
        auto rd1 = [&](auto I, auto PL) {  // one plane of k-step i's fragment
            constexpr int i = decltype(I)::value, pl = decltype(PL)::value;
            constexpr int tap = F::tap(i >> 1), off = ((tap / L::KW) * L::IW + tap % L::KW) * F::PIXB;
            fa[i % NB][pl] = dc_read<off>(addr(i, pl));
        };
        dc_unroll([&](auto I) { rd(I); }, std::make_integer_sequence<int, PD>{});
        dc_lgkm<2 * (PD - 1)>(fa[0][0], fa[0][1]);
        const int pmb = m0 - 64 + 32 * rg;
        int bw = 0;
        u32x4 bs = {0u, 0u, 0u, 0u};  // the epilogue group's scaled biases
        float y[4];
        // k-step i: its three MFMAs with the other work in their gaps (one wave per SIMD issues in order:
        // an MFMA occupies the matrix pipe 32 cycles, of which its issue takes 8).  The previous phase's
        // epilogue: group t's biases read at k-step 2 t (before the fragment reads, so the step's counted
        // wait covers them), its values, stores and mask bits in the three gaps of k-step 2 t + 1, the
        // bitmask word at k-step 8; the refill DMAs from k-step 16; then the wait for k-step i + 1's
        // fragments (the later k-steps' may stay in flight)
        dc_unroll(
            [&](auto I) {
                constexpr int i = decltype(I)::value;
                // mfma_split3: hi += aH bH, lo += aH bL, lo += aL bH (weight fragment (c, s, p) in AGPRs below NA)
                constexpr int fb = (i >> 1) * 4 + (i & 1) * 2;
                constexpr bool A0 = fb < F::NA, A1 = fb + 1 < F::NA;
                const u32x4& b0 = bq[i >> 1][i & 1][0];
                const u32x4& b1 = bq[i >> 1][i & 1][1];
                constexpr bool P = decltype(PREV)::value;
                constexpr bool EPI_BIAS = P && i < 8 && (i & 1) == 0, EPI = P && i < 8 && (i & 1) == 1;
                using T = std::integral_constant<int, i / 2>;
                if constexpr (i == 0)
                    dc_mfma0<A0>(H, fa[0][0], b0);
                else
                    dc_mfma<A0>(H, fa[i % NB][0], b0);
                if constexpr (EPI_BIAS) bs = dc_read<0>(bias_lane + 32 * (i / 2));
                if constexpr (P && i == 8) epi_bits(std::true_type{}, pmb, bw);
                if constexpr (i + PD < NK) rd1(std::integral_constant<int, i + PD>{}, std::integral_constant<int, 0>{});
                if constexpr (EPI) epi_val(T{}, PH, PL, bs, y);
                if constexpr (i == 0)
                    dc_mfma0<A1>(Lo, fa[0][0], b1);
                else
                    dc_mfma<A1>(Lo, fa[i % NB][0], b1);
                if constexpr (i + PD < NK) rd1(std::integral_constant<int, i + PD>{}, std::integral_constant<int, 1>{});
                if constexpr (EPI) epi_store(T{}, std::true_type{}, pmb, y);
                dc_mfma<A0>(Lo, fa[i % NB][1], b0);
                if constexpr (EPI) epi_mask(T{}, y, bw);
                // the refill DMAs whose k-step this is
                dc_unroll(
                    [&](auto X) {
                        constexpr int x = decltype(X)::value, t = x / F::DMAS;
                        if constexpr (16 + x * (NK - 16) / NDMA == i) {
                            if (t < nref) issue_one(rA + t, x % F::DMAS);
                        }
                    },
                    std::make_integer_sequence<int, NDMA>{});
                constexpr int later = (i + PD < NK ? i + PD : NK - 1) - (i + 1);  // k-steps read after i + 1
                if constexpr (i + 1 < NK) {
                    if constexpr (EPI_BIAS)
                        dc_lgkm<2 * later>(fa[(i + 1) % NB][0], fa[(i + 1) % NB][1], bs);
                    else
                        dc_lgkm<2 * later>(fa[(i + 1) % NB][0], fa[(i + 1) % NB][1]);
                }
            },
            std::make_integer_sequence<int, NK>{});
        // (a refill of more than RMAX samples: never after phase 0, whose samples the prologue issued)
        for (int t = RMAX; t < nref; ++t) issue_sample(rA + t);
        dc_acc_fence(H, Lo);
    };
    // the last phase's epilogue (its block may run past the range)
    auto final_epi = [&](const f32x16& PH, const f32x16& PL) {
        const int pmb = 64 * (F_ - 1) + 32 * rg;
        int bw = 0;
        dc_unroll(
            [&](auto T) {
                constexpr int t = decltype(T)::value;
                const u32x4 bs = *reinterpret_cast<const u32x4*>(lds + Gm::BIAS + (j * 32 + 4 * h + 8 * t) * 4);
                float y[4];
                epi_val(T, PH, PL, bs, y);
                epi_store(T, std::false_type{}, pmb, y);
                epi_mask(T, y, bw);
            },
            std::make_integer_sequence<int, 4>{});
        epi_bits(std::false_type{}, pmb, bw);
    };

    // phases alternate between the accumulator sets (H0, L0) and (H1, L1); the previous set's epilogue
    // runs inside the next phase
    phase(0, H0, L0, H1, L1, std::false_type{});
    int f = 1;
#pragma unroll 1
    for (; f + 1 < F_; f += 2) {
        phase(f, H1, L1, H0, L0, std::true_type{});
        phase(f + 1, H0, L0, H1, L1, std::true_type{});
    }
    if (f < F_) phase(f, H1, L1, H0, L0, std::true_type{});
    if ((F_ - 1) & 1)
        final_epi(H1, L1);
    else
        final_epi(H0, L0);
    amax_record(a.amax_y, __uint_as_float(om) * exp2i(-ey));  // (unscaled: exact)
}

// ---------------------------------------------------------------------------------------------
// The fc dgrad in the same form (round 4): g3 = (h3 > 0) * (df W), df (rows x 512) as PX planes
// (ppox_px_split), W the fc weight's dgrad packing (64-column blocks, split_frag_index), g3 written as
// PX planes (NHWC features), .ipynb_checkpoints/models-checkpoint.py:58-59 backward.  Workgroup
// (column group cg, row group rr): its 4 waves hold the weights of column tiles 4 cg .. 4 cg + 3 (32
// features each, 64 fragments = 256 AGPRs), and walk the rows [r0, r1) in phases of 32; each phase's df
// rows (2 KB each) are DMA'd into a 2-slot LDS ring (16-B pieces XOR-keyed by row & 15: conflict-free
// b128 reads) and read by all four waves.  Same per-element MFMA sequence as the sg2 fc dgrad
// (Px<SgRows<512, 3136, FC_DGRAD, .., true>, true, true>), so g3, its amax and exponent are bitwise its.
constexpr int FCD_N = 3136, FCD_TILES = FCD_N / 32, FCD_ROWB = 2048, FCD_PH = 32;
constexpr int FCD_SLOT = FCD_PH * FCD_ROWB, FCD_LDS = 2 * FCD_SLOT;
static_assert(FCD_LDS <= 160 * 1024, "fcd: LDS");

__global__ void __launch_bounds__(256, 1) fcd_kernel(Args a, const u32x4* __restrict__ wq, int nrg) {
    constexpr int NK = 32, KC = 16;  // k-steps, 32-k chunks
    __shared__ __attribute__((aligned(16))) uint8_t lds[FCD_LDS];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int cg = blockIdx.x / nrg, rr = blockIdx.x % nrg;
    const int T = cg * 4 + wave;                 // this wave's column tile
    const bool live = T < FCD_TILES;             // (the last group's waves 2, 3: DMAs and barriers only)
    const int Tc = live ? T : FCD_TILES - 1;
    const long long r0 = rr * a.batch / nrg, r1 = (rr + 1) * a.batch / nrg;
    const int MR = (int)(r1 - r0);
    if (MR <= 0) return;
    const int F_ = (MR + FCD_PH - 1) / FCD_PH;
    const uint8_t* xb = reinterpret_cast<const uint8_t*>(a.x) + r0 * FCD_ROWB;
    const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)lds);

    // phase f's rows into slot f & 1: wave w DMAs rows 8 w .. 8 w + 7 (two 1-KB DMAs each; LDS piece q of
    // row rho holds global piece q ^ (rho & 15)); rows past the range re-read the last row (never stored)
    auto issue_phase = [&](int f) {
        uint8_t* dst = lds + (f & 1) * FCD_SLOT;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int rho = wave * 8 + (i >> 1), d = i & 1;
            int row = f * FCD_PH + rho;
            row = row < MR ? row : MR - 1;
            const uint32_t q = (uint32_t)(d * 64 + lane);
            const uint32_t off = (uint32_t)row * FCD_ROWB + ((q ^ (uint32_t)(rho & 15)) << 4);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(xb + off),
                                             (__attribute__((address_space(3))) void*)(dst + rho * FCD_ROWB + d * 1024),
                                             16, 0, 0);
        }
    };
    issue_phase(0);
    // the weights of tile Tc: 64-column block Tc / 2, column tile Tc & 1 of it, all 16 chunks
    u32x4 bq[KC][2][2];
#pragma unroll
    for (int c = 0; c < KC; ++c)
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int p = 0; p < 2; ++p)
                bq[c][s][p] = wq[(long long)((Tc >> 1) * KC + c) * (2 * 2 * NPL * 64) + (((s * 2 + (Tc & 1)) * 2 + p) * 64) + lane];
    const int ex = *a.xexp, ew = *a.wexp;
    const uint32_t am = amax_read(a.amax_x), nm = amax_read(a.ynorm), bm = *a.ybias;
    const int ey = bound_exp(am, nm, bm);
    const float bnd = __uint_as_float(am) * __uint_as_float(nm) + __uint_as_float(bm);
    const float sy = __builtin_isfinite(bnd) ? exp2i(ey) : __builtin_nanf("");
    const float ua = exp2i(-ex), uws = exp2i(-ew) * sy;  // (the sg2 value (acc ua) uw, times sy: exact)
    if (blockIdx.x == 0 && threadIdx.x == 0) *a.yexp_out = ey;
    __builtin_amdgcn_s_waitcnt(0);
    asm volatile("s_nop 4" ::: "memory");

    uint16_t* y16 = reinterpret_cast<uint16_t*>(a.y);
    uint32_t om = 0u;
    f32x16 H0, L0, H1, L1;
    // epilogue group t of the 32-row block at range row pmb: lane (r, h) = row r0 + pmb + r, features
    // 32 Tc + 8 t + 4 h .. + 3 (mask bits of word mw)
    auto epi = [&](auto Tt, const f32x16& PH, const f32x16& PL, int pmb, uint32_t mw, auto FULL) {
        constexpr int t = decltype(Tt)::value;
        if (!live) return;  // (uniform: a tile past the last computed nothing)
        float y[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            y[k] = (mw >> (8 * t + 4 * h + k)) & 1u ? (PH[4 * t + k] + PL[4 * t + k]) * ua * uws : 0.f;
        uint32_t hw[2], lw[2];
        split2h((f32x2){y[0], y[1]}, 1.f, hw[0], lw[0]);
        split2h((f32x2){y[2], y[3]}, 1.f, hw[1], lw[1]);
        const long long m = r0 + pmb + r;
        uint16_t* dst = y16 + 2 * (m * FCD_N + Tc * 32) + 8 * t + 4 * h;
        if (decltype(FULL)::value || pmb + r < MR) {
            out_store2(dst, hw[0], hw[1]);
            out_store2(dst + 32, lw[0], lw[1]);
        }
        om = max(om, max(max(__float_as_uint(y[0]) & 0x7FFFFFFFu, __float_as_uint(y[1]) & 0x7FFFFFFFu),
                         max(__float_as_uint(y[2]) & 0x7FFFFFFFu, __float_as_uint(y[3]) & 0x7FFFFFFFu)));
    };
    auto mask_word = [&](int pmb) {
        long long m = r0 + pmb + r;
        m = m < r1 ? m : r1 - 1;
        return a.bits_mask[m * FCD_TILES + Tc];
    };

    auto phase = [&](int f, f32x16& H, f32x16& Lo, const f32x16& PH, const f32x16& PL, auto PREV) {
        // this phase's rows (DMA'd during the previous phase) landed for every wave; every wave done with
        // the slot the next phase refills
        asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        constexpr bool P = decltype(PREV)::value;
        const int pmb = FCD_PH * (f - 1);
        const uint32_t mw = P ? mask_word(pmb) : 0u;
        const uint32_t base = lds0 + (f & 1) * FCD_SLOT + r * FCD_ROWB;
        const uint32_t kx = (uint32_t)((r & 15) ^ h) << 4;
        auto addr = [&](int i, int pl) {  // k-step i = 2 c + s: piece 8 c + 4 pl + 2 s + h of row r
            const int c = i >> 1, s = i & 1;
            const uint32_t P16 = (uint32_t)(((c & 1) << 3) | (pl << 2) | (s << 1)) << 4;
            return base + (P16 ^ kx);
        };
        constexpr int PD = 2, NB = 3;
        u32x4 fa[NB][2];
        auto rd1 = [&](auto I, auto PLc) {
            constexpr int i = decltype(I)::value, pl = decltype(PLc)::value;
            fa[i % NB][pl] = dc_read<((i >> 1) >> 1) * 256>(addr(i, pl));
        };
        rd1(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
        rd1(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{});
        rd1(std::integral_constant<int, 1>{}, std::integral_constant<int, 0>{});
        rd1(std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{});
        dc_lgkm<2>(fa[0][0], fa[0][1]);
        dc_unroll(
            [&](auto I) {
                constexpr int i = decltype(I)::value;
                const u32x4& b0 = bq[i >> 1][i & 1][0];
                const u32x4& b1 = bq[i >> 1][i & 1][1];
                if (live) {
                    if constexpr (i == 0)
                        dc_mfma0<true>(H, fa[0][0], b0);
                    else
                        dc_mfma<true>(H, fa[i % NB][0], b0);
                }
                if constexpr (i + PD < NK) rd1(std::integral_constant<int, i + PD>{}, std::integral_constant<int, 0>{});
                if (live) {
                    if constexpr (i == 0)
                        dc_mfma0<true>(Lo, fa[0][0], b1);
                    else
                        dc_mfma<true>(Lo, fa[i % NB][0], b1);
                }
                if constexpr (i + PD < NK) rd1(std::integral_constant<int, i + PD>{}, std::integral_constant<int, 1>{});
                if constexpr (P && (i & 1) && i < 8) epi(std::integral_constant<int, i / 2>{}, PH, PL, pmb, mw, std::true_type{});
                if (live) dc_mfma<true>(Lo, fa[i % NB][1], b0);
                // the next phase's rows: 16 DMAs over k-steps 16 .. 31
                if constexpr (i == 16) {
                    if (f + 1 < F_) issue_phase(f + 1);
                }
                constexpr int later = (i + PD < NK ? i + PD : NK - 1) - (i + 1);
                if constexpr (i + 1 < NK) dc_lgkm<2 * later>(fa[(i + 1) % NB][0], fa[(i + 1) % NB][1]);
            },
            std::make_integer_sequence<int, NK>{});
        dc_acc_fence(H, Lo);
    };
    auto final_epi = [&](const f32x16& PH, const f32x16& PL) {
        const int pmb = FCD_PH * (F_ - 1);
        const uint32_t mw = mask_word(pmb);
        dc_unroll([&](auto Tt) { epi(Tt, PH, PL, pmb, mw, std::false_type{}); }, std::make_integer_sequence<int, 4>{});
    };
    phase(0, H0, L0, H1, L1, std::false_type{});
    int f = 1;
#pragma unroll 1
    for (; f + 1 < F_; f += 2) {
        phase(f, H1, L1, H0, L0, std::true_type{});
        phase(f + 1, H0, L0, H1, L1, std::true_type{});
    }
    if (f < F_) phase(f, H1, L1, H0, L0, std::true_type{});
    if ((F_ - 1) & 1)
        final_epi(H1, L1);
    else
        final_epi(H0, L0);
    amax_record(a.amax_y, __uint_as_float(om) * exp2i(-ey));
}

// ---------------------------------------------------------------------------------------------
// The conv2 dgrad in the direct form (round 5): g1 = (h1 > 0) * conv2^T(g2), .ipynb_checkpoints/
// models-checkpoint.py:55 backward (reached through ppo.py:241).  Conv2d(32, 64, 4, stride 2): an input
// pixel (iy, ix) of parity class (py, px) = (iy & 1, ix & 1) takes exactly the taps (py + 2 dy, px + 2 dx),
// dy, dx in {0, 1}, from the output pixels (a - dy, b - dx), a = iy >> 1, b = ix >> 1 — so a class is an
// implicit GEMM over its 10 x 10 input pixels with K = 4 taps x 64 channels of g2 (taps off the 9 x 9
// image read zeros), N = the 32 input channels: no col2im, every output written once.
//   * wave c (one per SIMD) owns class c = 2 py + px: its 4 taps' weights (the qd2 packing, k-step s =
//     4 t + (co >> 4), t = 2 dy + dx) live in 128 AGPRs as MFMA srcA, so the tile is channels x pixels;
//   * whole g2 sample images (PX planes, 81 pixels x 256 B) and conv1's ReLU bitmask of the sample
//     (400 words) stream into an LDS ring by LDS-DMA, each byte read from HBM once;
//   * a workgroup walks its contiguous range of samples in phases of 64 class rows (row m = 100 n + 10 a
//     + b of sample n of the range); the four waves walk the same rows of their four classes, so a phase
//     reads at most two samples.  An image pixel's 16-B pieces are stored at p ^ key, key = (4 n + 10 y
//     + x) & 15 (100 = 4 mod 16): a row's pixel at tap t then has key (m - 10 dy - dx) & 15, so a lane
//     group of ds_read_b128 (16 rows distinct mod 16) hits 16 distinct bank quads; a tap off the image reads
//     a zero pixel at the same piece positions.
// Every k-step is three v_mfma_f32_32x32x16_f16 (Wh gh, Wh gl, Wl gh), fp32-class as every split kernel;
// its k order (the four taps summed in the accumulators) is not the col2im form's, so the result is held
// to the fp64 bounds, not bitwise (tests/test_ddgrad2_gpu.py).
constexpr int DD2_PIXB = 256, DD2_NPIX = 81, DD2_IMG = DD2_NPIX * DD2_PIXB;  // g2 planes of one sample
constexpr int DD2_MASKB = 400 * 4;                                            // conv1's bitmask of one sample
constexpr int DD2_IMG_DMAS = (DD2_IMG + 1023) / 1024;                         // 21
constexpr int DD2_MASK0 = DD2_IMG_DMAS * 1024;                                // mask offset in a slot
constexpr int DD2_REAL_DMAS = DD2_IMG_DMAS + (DD2_MASKB + 1023) / 1024;      // 23
constexpr int DD2_SLOT = DD2_REAL_DMAS * 1024, DD2_DMAS = (DD2_REAL_DMAS + 3) / 4;  // per wave: 6
constexpr int DD2_NSLOT = 4, DD2_ZERO = DD2_NSLOT * DD2_SLOT, DD2_LDS = DD2_ZERO + 256;
constexpr int DD2_ROWS = 100;  // class rows per sample
static_assert(DD2_LDS <= 160 * 1024, "ddgrad2: LDS");

// A phase is 64 class rows per wave (two 32-row tiles A, B: 6 MFMAs per k-step), so its barrier, DMA wait
// and row setup are spread over 96 MFMAs; the next phase's per-lane row setup (tap addresses, output
// offsets) is computed in the MFMA gaps of the current one, the previous phase's epilogue rides in its k
// walk.  One accumulator per tile takes all three products of a k-step (Wh gh + Wh gl + Wl gh): each
// MFMA rounds once per 16 MACs, so the sum is still fp32-class (3 roundings per 16 MACs against an f32
// FMA chain's 16) — held to the fp64 bounds by tests/test_ddgrad2_gpu.py — and the registers of a
// second (lo) set pay for the two tiles.
__global__ void __launch_bounds__(256, 1) ddgrad2_kernel(Args a, const u32x4* __restrict__ wq) {
    constexpr int NK = 16;  // k-steps: 4 taps x 4 channel quarters
    constexpr int PR = 64;  // class rows per phase (two tiles)
    __shared__ __attribute__((aligned(16))) uint8_t lds[DD2_LDS];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int py = wave >> 1, px = wave & 1;  // this wave's class
    const int r = lane & 31, h = lane >> 5;
    const long long S0 = blockIdx.x * a.batch / gridDim.x, S1 = (blockIdx.x + 1) * a.batch / gridDim.x;
    const int NS = (int)(S1 - S0);
    if (NS <= 0) return;
    const int MR = NS * DD2_ROWS;
    const int F_ = (MR + PR - 1) / PR;
    const uint8_t* gb = reinterpret_cast<const uint8_t*>(a.x) + S0 * DD2_IMG;
    const uint8_t* mb = reinterpret_cast<const uint8_t*>(a.bits_mask) + S0 * DD2_MASKB;
    const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)lds);

    // DMA d = wave + 4 i of a sample fills slot bytes [1024 d, 1024 d + 1024): d < 21 image pixels (lane ->
    // LDS pixel u, piece position lane & 15 holding the global piece (lane & 15) ^ key), d = 21, 22 the
    // bitmask words (past their end: the last piece again, into the slot's pad), d > 22 DMA 22 again.
    // Per DMA slot i: the lane's byte offset within the sample's image (without the key) or bitmask, and
    // the pixel's key offset (10 y + x) & 15
    uint32_t doff[DD2_DMAS], dkey[DD2_DMAS];
#pragma unroll
    for (int i = 0; i < DD2_DMAS; ++i) {
        int d = wave + 4 * i;
        d = d < DD2_REAL_DMAS ? d : DD2_REAL_DMAS - 1;
        int u = (d * 1024 + lane * 16) / DD2_PIXB;
        u = u < DD2_NPIX ? u : DD2_NPIX - 1;
        int mo = (d - DD2_IMG_DMAS) * 1024 + lane * 16;
        mo = mo < DD2_MASKB ? mo : DD2_MASKB - 16;
        doff[i] = d < DD2_IMG_DMAS ? (uint32_t)(u * DD2_PIXB) : (uint32_t)mo;
        dkey[i] = (uint32_t)((10 * (u / 9) + u % 9) & 15);
    }
    // buffer descriptors (wave-uniform: built from kernel arguments and blockIdx only) of the range's g2
    // planes and bitmask words (the LDS-DMA sources: sample n at soffset n * bytes, the lane's piece in the
    // 32-bit voffset) and of its g1 rows (the epilogue's stores: a dead row's offset is past the end, so the
    // hardware drops its store — no branch)
    const auto g_rs = __builtin_amdgcn_make_buffer_rsrc((void*)gb, 0, NS * DD2_IMG, 0x00020000);
    const auto m_rs = __builtin_amdgcn_make_buffer_rsrc((void*)mb, 0, NS * DD2_MASKB, 0x00020000);
    auto issue_one = [&](int n, auto I) {
        constexpr int i = decltype(I)::value;
        int d = wave + 4 * i;  // (uniform)
        d = d < DD2_REAL_DMAS ? d : DD2_REAL_DMAS - 1;
        auto* dst = (__attribute__((address_space(3))) void*)(lds + (n % DD2_NSLOT) * DD2_SLOT + d * 1024);
        const uint32_t key = (uint32_t)(4 * n + dkey[i]) & 15u;
        const uint32_t vimg = doff[i] + ((((uint32_t)lane & 15u) ^ key) << 4);
        if (4 * i + 3 < DD2_IMG_DMAS || d < DD2_IMG_DMAS)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(g_rs, dst, 16, vimg, n * DD2_IMG, 0, 0);
        else
            __builtin_amdgcn_raw_ptr_buffer_load_lds(m_rs, dst, 16, doff[i], n * DD2_MASKB, 0, 0);
    };
    auto issue_sample = [&](int n) {
        dc_unroll([&](auto I) { issue_one(n, I); }, std::make_integer_sequence<int, DD2_DMAS>{});
    };
    int issued = NS < DD2_NSLOT ? NS : DD2_NSLOT;
    for (int n = 0; n < issued; ++n) issue_sample(n);
    // the class's weights: k-step s = 4 t + q (tap t = 2 dy + dx -> kernel tap (py + 2 dy, px + 2 dx),
    // channels 16 q .. 16 q + 15), planes p — fragment ((tap * 4 + q) * 2 + p) of the qd2 packing
    u32x4 bq[NK][2];
#pragma unroll
    for (int s = 0; s < NK; ++s) {
        const int t = s >> 2, tap = (py + 2 * (t >> 1)) * 4 + px + 2 * (t & 1);
#pragma unroll
        for (int p = 0; p < 2; ++p) bq[s][p] = wq[((tap * 4 + (s & 3)) * 2 + p) * 64 + lane];
    }
    // the accumulators' unscale, one exponent at a time (powers of two: exact): their sum leaves exp2i's range when
    // g2 is tiny (its exponent clamped at 126 — a minibatch whose loss gradient all but vanished: a 2,046-row rank
    // pass of the C4 run wrote Inf into g1 through the combined 2^-(126 + 14))
    const float us = exp2i(-*a.xexp), usw = exp2i(-*a.wexp);
    if (threadIdx.x < 16) reinterpret_cast<u32x4*>(lds + DD2_ZERO)[threadIdx.x] = u32x4{0u, 0u, 0u, 0u};

    // a tile's lane row: (n, a, b) of class row m, advanced by PR rows per phase without divisions
    struct Pos {
        int m, n, ra, rb;
    };
    auto pos_of = [&](int m) {
        Pos P;
        P.m = m;
        P.n = m / DD2_ROWS;
        const int rem = m - P.n * DD2_ROWS;
        P.ra = rem / 10;
        P.rb = rem - 10 * P.ra;
        return P;
    };
    auto advance = [&](Pos& P) {  // + 64 rows = + 6 a-rows and 4 b-columns
        P.m += PR;
        P.rb += PR % 10;
        const bool cb = P.rb >= 10;
        P.rb -= cb ? 10 : 0;
        P.ra += PR / 10 + (cb ? 1 : 0);
        const bool ca = P.ra >= 10;
        P.ra -= ca ? 10 : 0;
        P.n += ca ? 1 : 0;
    };
    // a tile's per-lane setup: the read pixel of each tap (its base | (key ^ h) << 4; off the image: the
    // zero pixel), the output pixel's byte offset in g1 (past the end for a dead row), its mask word's address
    struct Rows {
        uint32_t tb[4];
        int o;  // the output pixel's byte offset in the range's g1
        uint32_t ma;
    };
    auto rows = [&](const Pos& P) {
        Rows R;
        const bool live = P.m < MR;
        const int n = live ? P.n : NS - 1, ra = live ? P.ra : 9, rb = live ? P.rb : 9;
        const uint32_t sbase = lds0 + (uint32_t)((n % DD2_NSLOT) * DD2_SLOT);
        const uint32_t pix = sbase + (uint32_t)((9 * ra + rb) * DD2_PIXB);
        const int mkey = 4 * n + 10 * ra + rb;
        const bool oky[2] = {ra != 9, ra != 0}, okx[2] = {rb != 9, rb != 0};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int dy = t >> 1, dx = t & 1;
            const uint32_t key = ((uint32_t)(mkey - 10 * dy - dx) & 15u) ^ (uint32_t)h;
            const uint32_t at = pix - (uint32_t)((9 * dy + dx) * DD2_PIXB);
            R.tb[t] = ((oky[dy] && okx[dx]) ? at : lds0 + DD2_ZERO) | (key << 4);
        }
        const int q = (2 * ra + py) * 20 + 2 * rb + px;
        R.o = live ? (n * 400 + q) * 128 : 0x7FFFFF00;  // byte offset in the range's g1 (dead: past the end)
        R.ma = sbase + DD2_MASK0 + (uint32_t)(q * 4);
        return R;
    };
    Pos QA = pos_of(r), QB = pos_of(32 + r);
    Rows RA = rows(QA), RB = rows(QB);  // phase 0's
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    asm volatile("s_nop 4" ::: "memory");  // (VALU-written B registers before the first MFMA reads them)

    const auto o_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(a.y + S0 * (400 * 32)), 0, NS * (400 * 32 * 4), 0x00020000);
    float om = 0.f;
    f32x16 A0, B0, A1, B1;
    int poA = 0x7FFFFF00, poB = 0x7FFFFF00;  // the previous phase's output byte offsets and mask words (>> 4 h)
    uint32_t pmA = 0u, pmB = 0u;

    // epilogue group t of a tile: channels 8 t + 4 h + k of the lane's pixel, times conv1's ReLU bit
    auto epi = [&](auto T, const f32x16& C, int o, uint32_t mw) {
        constexpr int t = decltype(T)::value;
        const f32x2 v01 = ((f32x2){C[4 * t], C[4 * t + 1]} * (f32x2){us, us}) * (f32x2){usw, usw};
        const f32x2 v23 = ((f32x2){C[4 * t + 2], C[4 * t + 3]} * (f32x2){us, us}) * (f32x2){usw, usw};
        const float vv[4] = {v01.x, v01.y, v23.x, v23.y};
        float v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // bit -> all-ones or zero (one v_bfe_i32), ANDed with the value's bits
            uint32_t mk;
            asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(mk) : "v"(mw), "n"(8 * t + k));
            v[k] = __uint_as_float(__float_as_uint(vv[k]) & mk);
        }
        __builtin_amdgcn_raw_buffer_store_b128(
            u32x4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])}, o_rs,
            (uint32_t)o + (uint32_t)(32 * t + 16 * h), 0, 0);
        om = fmaxf(om, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
    };
    // refill DMAs (at most one sample per phase: 64 rows < 100) over k-steps 9 .. 14
    constexpr int RMAX = 1, NDMA = RMAX * DD2_DMAS;

    auto phase = [&](int f, f32x16& CA, f32x16& CB, const f32x16& PA, const f32x16& PB, auto PREV) {
        const int m0 = PR * f;
        const int nlo = m0 / DD2_ROWS, nhi = min((m0 + PR - 1) / DD2_ROWS, NS - 1);
        dc_vm_wait<DD2_DMAS>(issued - 1 - nhi);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        const int rA = issued, nref = min(nlo + DD2_NSLOT, NS) - issued;
        issued += nref;
        // this phase's mask words (for the next phase's epilogue), then k-steps 0 and 1's fragments
        uint32_t mwA, mwB;
        asm volatile("ds_read_b32 %0, %1" : "=v"(mwA) : "v"(RA.ma));
        asm volatile("ds_read_b32 %0, %1" : "=v"(mwB) : "v"(RB.ma));
        // k-step i, plane pl, tile: piece 8 (q >> 1) + 4 pl + 2 (q & 1) + h of the tap's pixel
        auto addr = [&](const Rows& R, int i, int pl) {
            const int q = i & 3;
            return R.tb[i >> 2] ^ ((uint32_t)(8 * (q >> 1) + 4 * pl + 2 * (q & 1)) << 4);
        };
        constexpr int PD = 2, NB = PD + 1;
        u32x4 fa[NB][2][2];  // [k-step buffer][tile][plane]
        auto rd = [&](auto I, auto TL, auto PLc) {
            constexpr int i = decltype(I)::value, tl = decltype(TL)::value, pl = decltype(PLc)::value;
            fa[i % NB][tl][pl] = dc_read<0>(addr(tl ? RB : RA, i, pl));
        };
        using Z = std::integral_constant<int, 0>;
        using O = std::integral_constant<int, 1>;
        dc_unroll([&](auto I) { rd(I, Z{}, Z{}); rd(I, Z{}, O{}); rd(I, O{}, Z{}); rd(I, O{}, O{}); },
                  std::make_integer_sequence<int, PD>{});
        asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(fa[0][0][0]), "+v"(fa[0][0][1]), "+v"(fa[0][1][0]),
                     "+v"(fa[0][1][1]), "+v"(mwA), "+v"(mwB));
        mwA >>= 4 * h;
        mwB >>= 4 * h;
        Rows NA, NBr;  // the next phase's row setup, computed in this phase's gaps
        dc_unroll(
            [&](auto I) {
                constexpr int i = decltype(I)::value;
                constexpr bool P = decltype(PREV)::value;
                const u32x4& b0 = bq[i][0];
                const u32x4& b1 = bq[i][1];
                const u32x4(&x)[2][2] = fa[i % NB];
                if constexpr (i == 0) {
                    dc_mfma0<true>(CA, x[0][0], b0);
                    dc_mfma0<true>(CB, x[1][0], b0);
                } else {
                    dc_mfma<true>(CA, x[0][0], b0);
                    dc_mfma<true>(CB, x[1][0], b0);
                }
                if constexpr (i + PD < NK) rd(std::integral_constant<int, i + PD>{}, Z{}, Z{});
                if constexpr (i + PD < NK) rd(std::integral_constant<int, i + PD>{}, Z{}, O{});
                dc_mfma<true>(CA, x[0][0], b1);
                dc_mfma<true>(CB, x[1][0], b1);
                if constexpr (i + PD < NK) rd(std::integral_constant<int, i + PD>{}, O{}, Z{});
                if constexpr (i + PD < NK) rd(std::integral_constant<int, i + PD>{}, O{}, O{});
                // the previous phase's epilogue, one group per k-step: tile A's at k-steps 0 .. 3, tile B's at
                // 4 .. 7 — early, so its stores complete before the next phase's vmcnt wait, which (gfx9: one
                // counter for loads and stores) covers every store issued before this phase's refill DMAs
                if constexpr (P && i < 8) {
                    if constexpr (i < 4)
                        epi(std::integral_constant<int, i>{}, PA, poA, pmA);
                    else
                        epi(std::integral_constant<int, i - 4>{}, PB, poB, pmB);
                }
                dc_mfma<true>(CA, x[0][1], b0);
                dc_mfma<true>(CB, x[1][1], b0);
                if constexpr (i == 8) {
                    advance(QA);
                    advance(QB);
                }
                if constexpr (i == 9) NA = rows(QA);
                if constexpr (i == 11) NBr = rows(QB);
                dc_unroll(
                    [&](auto X) {
                        constexpr int x_ = decltype(X)::value, t = x_ / DD2_DMAS;
                        if constexpr (9 + x_ == i) {
                            if (t < nref) issue_one(rA + t, std::integral_constant<int, x_ % DD2_DMAS>{});
                        }
                    },
                    std::make_integer_sequence<int, NDMA>{});
                constexpr int later = (i + PD < NK ? i + PD : NK - 1) - (i + 1);
                if constexpr (i + 1 < NK) {
                    constexpr int j = (i + 1) % NB;
                    asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(fa[j][0][0]), "+v"(fa[j][0][1]), "+v"(fa[j][1][0]),
                                 "+v"(fa[j][1][1]) : "n"(4 * later));
                }
            },
            std::make_integer_sequence<int, NK>{});
        for (int t = RMAX; t < nref; ++t) issue_sample(rA + t);
        poA = RA.o;
        poB = RB.o;
        pmA = mwA;
        pmB = mwB;
        RA = NA;
        RB = NBr;
        dc_acc_fence(CA, CB);
    };
    auto final_epi = [&](const f32x16& PA, const f32x16& PB) {
        dc_unroll([&](auto T) { epi(T, PA, poA, pmA); }, std::make_integer_sequence<int, 4>{});
        dc_unroll([&](auto T) { epi(T, PB, poB, pmB); }, std::make_integer_sequence<int, 4>{});
    };
    phase(0, A0, B0, A1, B1, std::false_type{});
    int f = 1;
#pragma unroll 1
    for (; f + 1 < F_; f += 2) {
        phase(f, A1, B1, A0, B0, std::true_type{});
        phase(f + 1, A0, B0, A1, B1, std::true_type{});
    }
    if (f < F_) phase(f, A1, B1, A0, B0, std::true_type{});
    if ((F_ - 1) & 1)
        final_epi(A1, B1);
    else
        final_epi(A0, B0);
    amax_record(a.amax_y, om);
}

// ---------------------------------------------------------------------------
// The fc forward on PX h3 in wide tiles (round 5): f = relu(h3 W^T + b), .ipynb_checkpoints/
// models-checkpoint.py:58-59 (Linear(3136, 512) + ReLU).  The sg2 GEMM's 128 x 64 tiles stage 2.4 MB
// of A and B through L2 -> LDS per tile (9.6 MB per CU at 16,384 rows), which bounds it at the ~70 GB/s
// per CU that path sustains; a 256 x 128 tile stages 4.8 MB for the same MFMA work per CU (one tile per CU
// at 16,384 rows: 64 row tiles x 4 column groups).  8 waves (two per SIMD): wave w owns rows 64 (w >> 1)
// .. + 63 and columns 64 (w & 1) .. + 63 of the tile — 2 x 2 tiles of 32 x 32 with the sg2 form's hi / lo
// accumulator pair (one accumulator for all three products measured 2.5x the f32 GEMM's error at K = 3136),
// 8 fragment reads and 12 MFMAs per k-step.  Per 32-k chunk
// the 256 A rows (PX: 32 hi + 32 lo f16, 128 B, pieces XOR-swizzled by (row >> 1) & 7 as the sg2 kernel)
// and the two 64-column packed B blocks (16 KB) are LDS-DMA'd into a 3-slot ring, each wave its own 32
// rows and two B pieces.  The four column groups of a row tile run on one XCD (xcd_remap): A is read
// from HBM about once, B about once per XCD.  fp32-class; the k order is the sg2 form's but not its 64-column
// tiles' instruction interleave, so it is held to the fp64 bound (tests/test_fcw_gpu.py).
constexpr int FCW_ROWS = 256, FCW_KC = 3136 / 32, FCW_ROWB = 3136 * 4;  // rows per tile, chunks, PX row bytes
constexpr int FCW_BQ = 2 * 2 * 2 * 64;                                  // u32x4 per 64-column B block chunk
constexpr int FCW_AB = FCW_ROWS * 128, FCW_SLOT = FCW_AB + 2 * FCW_BQ * 16, FCW_NSLOT = 3;
constexpr int FCW_LDS = FCW_NSLOT * FCW_SLOT;  // 147,456 B
constexpr int FCW_SK = 8;                       // K-splits of the small-batch form
static_assert(FCW_LDS <= 160 * 1024, "fcw: LDS");

template <int N>
__device__ inline void fcw_lgkm(u32x4 (&x)[8], u32x4 (&y)[8]) {
    asm volatile("s_waitcnt lgkmcnt(%16)"
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),
                   "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7])
                 : "n"(N));
}
template <int N>
__device__ inline void sg_vm_wait_n() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// SK > 1 (small batches, round 5): split over K — workgroup (row tile, split ks, column group) walks chunks
// [98 ks / SK, 98 (ks + 1) / SK) and stores its unscaled partial product to slab a.y[ks][row][512]
// (no bias, no ReLU: fc_fwd_sk_reduce_actor adds the SK partials in order); a row tile's SK x 4 workgroups
// run on one XCD
template <int SK>
__global__ void __launch_bounds__(512, 1) fcw_kernel(Args a, const u32x4* __restrict__ wq) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[FCW_LDS];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long long L = xcd_remap(blockIdx.x, gridDim.x);
    const int cg = (int)(L & 3), ks = (int)((L >> 2) % SK);
    const long long m0 = ((L >> 2) / SK) * FCW_ROWS, M = a.batch;
    const int c0 = ks * FCW_KC / SK, nck = (ks + 1) * FCW_KC / SK - c0;  // this workgroup's chunks
    const int rg = wave >> 1, ch = wave & 1;
    const int r = lane & 31, h = lane >> 5;
    const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)lds);

    // DMA sources: A instruction j of this wave: row 32 w + 8 j + (lane >> 3) (past the batch: the last row,
    // never stored), LDS piece lane & 7 <- global piece (lane & 7) ^ ((row >> 1) & 7); B pieces 2 w, 2 w + 1
    // of the chunk's 16 (block 2 cg + (piece >> 3), 1-KB piece piece & 7 of its 8 KB)
    const uint8_t* asrc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int row = 32 * wave + 8 * j + (lane >> 3);
        long long m = m0 + row;
        m = m < M ? m : M - 1;
        asrc[j] = reinterpret_cast<const uint8_t*>(a.x) + m * FCW_ROWB + ((((lane & 7) ^ ((row >> 1) & 7))) << 4);
    }
    const u32x4* bsrc[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int q = 2 * wave + i;
        bsrc[i] = wq + (long long)(2 * cg + (q >> 3)) * FCW_KC * FCW_BQ + (q & 7) * 64 + lane;
    }
    auto issue = [&](int c, auto S) {
        constexpr int slot = decltype(S)::value;
        c = c0 + (c < nck ? c : nck - 1);  // past the end: the last chunk again, never read
        uint8_t* base = lds + slot * FCW_SLOT;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(asrc[j] + c * 128),
                                             (__attribute__((address_space(3))) void*)(base + (wave * 32 + 8 * j) * 128),
                                             16, 0, 0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(bsrc[i] + c * FCW_BQ),
                                             (__attribute__((address_space(3))) void*)(base + FCW_AB + (2 * wave + i) * 1024),
                                             16, 0, 0);
    };
    const int ex = *a.xexp, ew = *a.wexp;
    const float us = exp2i(-ex) * exp2i(-ew);

    f32x16 acc[2][2], acl[2][2];  // hi products / the two cross products (the sg2 form's pair)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[i][t] = acl[i][t] = zero16();
    const uint32_t sw = (uint32_t)((r >> 1) & 7);
    const uint32_t a_lane = lds0 + (uint32_t)((64 * rg + r) * 128), b_lane = lds0 + FCW_AB + ch * (FCW_BQ * 16) + lane * 16;
    // chunk in slot S: both k-steps' 16 fragment reads up front, k-step 0's MFMAs once its 8 landed
    auto compute = [&](auto S) {
        constexpr int slot = decltype(S)::value;
        u32x4 f[2][8];  // [k-step][A (row tile i, plane p) 0..3 | B (column tile t, plane p) 4..7]
#pragma unroll
        for (int s = 0; s < 2; ++s) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int p = 0; p < 2; ++p)
                    f[s][2 * i + p] = dc_read<0>(a_lane + slot * FCW_SLOT + i * 32 * 128 +
                                                 ((((uint32_t)(4 * p + 2 * s + h)) ^ sw) << 4));
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int p = 0; p < 2; ++p)
                    f[s][4 + 2 * t + p] = dc_read<0>(b_lane + slot * FCW_SLOT + (((s * 2 + t) * 2 + p) * 64) * 16);
        }
        auto mm = [&](const u32x4 (&g)[8]) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int t = 0; t < 2; ++t) acc[i][t] = mfma_f16(g[2 * i], g[4 + 2 * t], acc[i][t]);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int t = 0; t < 2; ++t) acl[i][t] = mfma_f16(g[2 * i], g[4 + 2 * t + 1], acl[i][t]);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int t = 0; t < 2; ++t) acl[i][t] = mfma_f16(g[2 * i + 1], g[4 + 2 * t], acl[i][t]);
        };
        fcw_lgkm<8>(f[0], f[1]);
        mm(f[0]);
        fcw_lgkm<0>(f[0], f[1]);
        mm(f[1]);
    };
    auto step = [&](int c, auto S, auto S2) {
        sg_vm_wait_n<6>();  // this wave's DMAs of chunk c landed (chunk c + 1's may be in flight)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        issue(c + 2, S2);
        compute(S);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    issue(0, I0{});
    issue(1, I1{});
#pragma unroll 1
    for (int c = 0; c < nck; c += 3) {
        step(c, I0{}, I2{});
        if (c + 1 < nck) step(c + 1, I1{}, I0{});
        if (c + 2 < nck) step(c + 2, I2{}, I1{});
    }
    sg_vm_wait_n<0>();  // the clamped tail DMAs, before the LDS is released
    if constexpr (SK > 1) {  // the partial product (its split's slab)
        float* slab = a.y + (long long)ks * M * 512;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int n = 128 * cg + 64 * ch + 32 * t + r;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const long long m = m0 + 64 * rg + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h;
                    if (m < M) slab[m * 512 + n] = (acc[i][t][q] + acl[i][t][q]) * us;
                }
        }
        return;
    }
    float om = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int n = 128 * cg + 64 * ch + 32 * t + r;
        const float b = a.bias[n];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const long long m = m0 + 64 * rg + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h;
                const float v = fmaxf((acc[i][t][q] + acl[i][t][q]) * us + b, 0.f);
                if (m < M) {
                    a.y[m * 512 + n] = v;
                    om = fmaxf(om, v);
                }
            }
    }
    amax_record(a.amax_y, om);
}

// ---------------------------------------------------------------------------
// The heads' backward to the fc output in one launch (round 5): for the critic's hidden layer e = relu(f Wh^T
// + bh) (models-checkpoint.py:80-84 extra_layer) and the actor head (Linear(512, A)),
//   de = (e > 0) * dv wc                                   (the critic head's grad through its ReLU)
//   df = (f > 0) * (dout Wa + de Wh)                       (into the fc layer, times the fc ReLU)
// — what head_dgrad_outer_kernel + the sg2 hidden-layer dgrad computed in two launches with de staged through
// HBM.  de Wh = dv * ((e > 0) * wc) Wh: the GEMM's A operand is wc's two f16 planes (split once per workgroup
// at wc's own exponent) masked by e > 0, so no amax of de is needed before the GEMM and dv scales the product in
// the epilogue.  The fcd_kernel pattern: workgroup (column group cg, row group) holds the 4 column tiles 4 cg
// .. 4 cg + 3 of Wh's dgrad packing in AGPRs (64 fragments each) and walks its rows in phases of 32: the
// phase's A rows are built in LDS by all 256 threads from e (coalesced float4 reads: thread t always handles
// columns 4 (t & 127) .. + 3, whose wc planes it keeps in 4 registers), column group 0 also storing de; then
// the 32 k-steps of 3 MFMAs; then the epilogue (dout Wa from LDS, the fc mask, df and its amax).  fp32-class
// (held to the fp64 bound: tests/test_hbw_gpu.py); de bitwise head_dgrad_outer_kernel's.
constexpr int HBW_PH = 32, HBW_ROWB = 2048, HBW_SLOT = HBW_PH * HBW_ROWB;  // A rows: 512 j x 2 planes x f16
constexpr int HBW_WA = 2 * HBW_SLOT, HBW_LDS = HBW_WA + 8 * 512 * 4;      // + Wa (<= 8 actions) f32

struct HbwArgs {
    const float *dout, *wa, *dv, *wc, *e, *f;
    float *df, *de;
    uint32_t *amax_de, *amax_df;
    const int* wexp;  // Wh's dgrad packing exponent
    long long rows;
    int nrg;  // row groups
};

template <int NO>
__global__ void __launch_bounds__(256, 1) hbw_kernel(HbwArgs a, const u32x4* __restrict__ wq) {
    constexpr int NK = 32, KC = 16;
    __shared__ __attribute__((aligned(16))) uint8_t lds[HBW_LDS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;
    const long long L = xcd_remap(blockIdx.x, gridDim.x);
    const int cg = (int)(L & 3), rr = (int)(L >> 2);
    const int T = cg * 4 + wave;  // this wave's column tile (32 of the 512 inputs)
    const long long r0 = rr * a.rows / a.nrg, r1 = (rr + 1) * a.rows / a.nrg;
    const int MR = (int)(r1 - r0);
    if (MR <= 0) return;
    const int F_ = (MR + HBW_PH - 1) / HBW_PH;
    const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)lds);

    // wc's split at its own exponent (every workgroup derives the same): thread t keeps columns 4 (t & 127) ..
    // (wc sits in the flat parameter buffer at an offset that depends on the action count: four dword loads,
    // no 16-B alignment asked of it)
    const int c4 = tid & 127;
    const float4 w4 = make_float4(a.wc[4 * c4], a.wc[4 * c4 + 1], a.wc[4 * c4 + 2], a.wc[4 * c4 + 3]);
    uint32_t wmax = max(max(__float_as_uint(fabsf(w4.x)), __float_as_uint(fabsf(w4.y))),
                        max(__float_as_uint(fabsf(w4.z)), __float_as_uint(fabsf(w4.w))));
    wmax = wave_max_u32(wmax);
    uint32_t* red = reinterpret_cast<uint32_t*>(lds + HBW_WA);
    if (lane == 0) red[wave] = wmax;
    // Wa to LDS after the reduction (it shares the space): [o][512]
    __syncthreads();
    const uint32_t wm = max(max(red[0], red[1]), max(red[2], red[3]));
    __syncthreads();
    for (int i = tid; i < NO * 128; i += 256)
        reinterpret_cast<float4*>(lds + HBW_WA)[i] = reinterpret_cast<const float4*>(a.wa)[i];
    const int ec = split_scale_exp(wm);
    uint32_t wh[2], wl[2];
    split2h((f32x2){w4.x, w4.y}, exp2i(ec), wh[0], wl[0]);
    split2h((f32x2){w4.z, w4.w}, exp2i(ec), wh[1], wl[1]);
    // the weights of tile T: 64-column block T >> 1, tile T & 1, all 16 chunks (the fcd_kernel load)
    u32x4 bq[KC][2][2];
#pragma unroll
    for (int c = 0; c < KC; ++c)
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int p = 0; p < 2; ++p)
                bq[c][s][p] = wq[(long long)((T >> 1) * KC + c) * (2 * 2 * NPL * 64) + (((s * 2 + (T & 1)) * 2 + p) * 64) + lane];
    const float us = exp2i(-ec) * exp2i(-*a.wexp);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();  // (Wa in LDS)
    asm volatile("s_nop 4" ::: "memory");

    float om_df = 0.f, om_de = 0.f;
    // build phase f's A rows into slot f & 1: float4 k of thread t is row 2 k + (t >> 7) of the phase, columns
    // 4 c4 .. 4 c4 + 3 — the planes' 8-B half (c4 & 1) of piece ((j >> 5) & 1) 8 + p 4 + ((j >> 3) & 3) of the row's
    // 256-B unit j >> 6, the piece stored at position piece ^ (row & 15) (fcd_kernel's layout)
    const int j0 = 4 * c4;
    const uint32_t unit = (uint32_t)(j0 >> 6) * 256, pc = (uint32_t)(((j0 >> 5) & 1) * 8 + ((j0 >> 3) & 3)),
                   half = (uint32_t)((j0 >> 2) & 1) * 8;
    auto build = [&](int f) {
        uint8_t* slot = lds + (f & 1) * HBW_SLOT;
        // the phase's 16 rows of e and dv loaded together (one memory round trip; in groups of 4 the build
        // took four per phase, most of the kernel's time at 16,384 rows)
        float4 evs[16];
        float ss[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            long long m = r0 + (long long)f * HBW_PH + 2 * k + (tid >> 7);
            m = m < r1 ? m : r1 - 1;
            evs[k] = reinterpret_cast<const float4*>(a.e)[m * 128 + c4];
            ss[k] = a.dv[m];
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int row = 2 * k + (tid >> 7);
            long long m = r0 + (long long)f * HBW_PH + row;
            const bool live = m < r1;
            m = live ? m : r1 - 1;
            const float4 ev = evs[k];
            const float s = ss[k];
            const uint32_t m0 = (ev.x > 0.f ? 0xFFFFu : 0u) | (ev.y > 0.f ? 0xFFFF0000u : 0u);
            const uint32_t m1 = (ev.z > 0.f ? 0xFFFFu : 0u) | (ev.w > 0.f ? 0xFFFF0000u : 0u);
            const uint32_t key = (uint32_t)(row & 15);
            uint8_t* rb = slot + row * HBW_ROWB + unit + half;
            *reinterpret_cast<uint2*>(rb + ((pc ^ key) << 4)) = make_uint2(wh[0] & m0, wh[1] & m1);
            *reinterpret_cast<uint2*>(rb + (((pc + 4) ^ key) << 4)) = make_uint2(wl[0] & m0, wl[1] & m1);
            if (cg == 0 && live) {  // de, as head_dgrad_outer_kernel: (e > 0) ? dv * wc : 0
                float4 o;
                o.x = ev.x > 0.f ? s * w4.x : 0.f;
                o.y = ev.y > 0.f ? s * w4.y : 0.f;
                o.z = ev.z > 0.f ? s * w4.z : 0.f;
                o.w = ev.w > 0.f ? s * w4.w : 0.f;
                reinterpret_cast<float4*>(a.de)[m * 128 + c4] = o;
                om_de = fmaxf(om_de, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
            }
        }
    };
    f32x16 H, Lo;
    const uint32_t kx = (uint32_t)((r & 15) ^ h) << 4;
    for (int f = 0; f < F_; ++f) {
        build(f);
        __syncthreads();  // the phase's A rows written; (two slots: every wave is past phase f - 2's reads)
        const uint32_t base = lds0 + (f & 1) * HBW_SLOT + r * HBW_ROWB;
        auto addr = [&](int i, int pl) {  // k-step i = 2 c + s: piece 8 (c & 1) + 4 pl + 2 s + h of row r
            const int c = i >> 1, s = i & 1;
            const uint32_t P16 = (uint32_t)(((c & 1) << 3) | (pl << 2) | (s << 1)) << 4;
            return base + (P16 ^ kx);
        };
        constexpr int PD = 2, NB = 3;
        u32x4 fa[NB][2];
        auto rd1 = [&](auto I, auto PLc) {
            constexpr int i = decltype(I)::value, pl = decltype(PLc)::value;
            fa[i % NB][pl] = dc_read<((i >> 1) >> 1) * 256>(addr(i, pl));
        };
        using Z = std::integral_constant<int, 0>;
        using O = std::integral_constant<int, 1>;
        // the epilogue's operands, loaded before the k walk: lane (r, h) = row r of the phase
        long long m = r0 + (long long)f * HBW_PH + r;
        const bool live = m < r1;
        m = live ? m : r1 - 1;
        float go[NO];
#pragma unroll
        for (int o = 0; o < NO; ++o) go[o] = a.dout[m * NO + o];
        const float sv = a.dv[m];
        float4 fv[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) fv[t] = reinterpret_cast<const float4*>(a.f)[m * 128 + ((32 * T + 8 * t + 4 * h) >> 2)];
        rd1(Z{}, Z{});
        rd1(Z{}, O{});
        rd1(O{}, Z{});
        rd1(O{}, O{});
        dc_lgkm<2>(fa[0][0], fa[0][1]);
        dc_unroll(
            [&](auto I) {
                constexpr int i = decltype(I)::value;
                const u32x4& b0 = bq[i >> 1][i & 1][0];
                const u32x4& b1 = bq[i >> 1][i & 1][1];
                if constexpr (i == 0)
                    dc_mfma0<true>(H, fa[0][0], b0);
                else
                    dc_mfma<true>(H, fa[i % NB][0], b0);
                if constexpr (i + PD < NK) rd1(std::integral_constant<int, i + PD>{}, Z{});
                if constexpr (i == 0)
                    dc_mfma0<true>(Lo, fa[0][0], b1);
                else
                    dc_mfma<true>(Lo, fa[i % NB][0], b1);
                if constexpr (i + PD < NK) rd1(std::integral_constant<int, i + PD>{}, O{});
                dc_mfma<true>(Lo, fa[i % NB][1], b0);
                constexpr int later = (i + PD < NK ? i + PD : NK - 1) - (i + 1);
                if constexpr (i + 1 < NK) dc_lgkm<2 * later>(fa[(i + 1) % NB][0], fa[(i + 1) % NB][1]);
            },
            std::make_integer_sequence<int, NK>{});
        dc_acc_fence(H, Lo);
        // epilogue: inputs 32 T + 8 t + 4 h + k of the lane's row
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int i0 = 32 * T + 8 * t + 4 * h;
            float4 d = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int o = 0; o < NO; ++o) {  // dout Wa, in head_dgrad_outer_kernel's order
                const float4 wv = *reinterpret_cast<const float4*>(lds + HBW_WA + (o * 512 + i0) * 4);
                d.x = fmaf(go[o], wv.x, d.x);
                d.y = fmaf(go[o], wv.y, d.y);
                d.z = fmaf(go[o], wv.z, d.z);
                d.w = fmaf(go[o], wv.w, d.w);
            }
            float4 y;
            y.x = fv[t].x > 0.f ? d.x + ((H[4 * t] + Lo[4 * t]) * us) * sv : 0.f;
            y.y = fv[t].y > 0.f ? d.y + ((H[4 * t + 1] + Lo[4 * t + 1]) * us) * sv : 0.f;
            y.z = fv[t].z > 0.f ? d.z + ((H[4 * t + 2] + Lo[4 * t + 2]) * us) * sv : 0.f;
            y.w = fv[t].w > 0.f ? d.w + ((H[4 * t + 3] + Lo[4 * t + 3]) * us) * sv : 0.f;
            if (live) {
                reinterpret_cast<float4*>(a.df)[m * 128 + (i0 >> 2)] = y;
                om_df = fmaxf(om_df, fmaxf(fmaxf(fabsf(y.x), fabsf(y.y)), fmaxf(fabsf(y.z), fabsf(y.w))));
            }
        }
    }
    amax_record(a.amax_df, om_df);
    if (cg == 0) amax_record(a.amax_de, om_de);
}

// ---------------------------------------------------------------------------
// The conv3 dgrad in the direct form (round 5): g2 = (h2 > 0) * conv3^T(g3), PX g3 in, PX g2 out,
// .ipynb_checkpoints/models-checkpoint.py:57 backward (reached through ppo.py:241).  An h2 pixel
// (iy, ix) takes tap (ky, kx) from the g3 pixel (iy - ky, ix - kx) when that lies on the 7 x 7 image — an
// implicit GEMM with rows = the 81 h2 pixels of each sample, K = 9 taps x 64 channels of g3, N = the 64
// input channels: every output written once, no col2im.  As dconv_fwd_kernel<DcF3>:
//   * wave w holds the 72 weight fragments of column tile j = w & 1 (the qd3 packing, 240 AGPRs + 48
//     VGPRs) and computes row block w >> 1 of each 64-row phase;
//   * whole g3 sample images (PX planes, 49 pixels x 256 B) and conv2's ReLU bitmask of the sample (81 x 2
//     words) stream into an LDS ring by LDS-DMA (buffer loads: the image's tail past pixel 48 reads zeros);
//   * the image's 16-B pieces are stored at p ^ key, key = (n + 9 y + x) & 15 (81 = 1 mod 16), so a row
//     m = 81 n + 9 iy + ix reads tap (ky, kx) at key (m - 9 ky - kx) & 15: the 16 rows of a lane group
//     hit 16 distinct bank quads; a tap off the image reads a zero pixel at the same piece positions.
// The taps off the image cost MFMAs (729 tap-rows per sample for 441 real, 1.65x) — the price of K = 576
// in registers and one pass over each g3 image; the im2col sgemm (SgDgradPM) walks only the real taps but
// stages 442 KB per 128-row tile through LDS.  fp32-class; its k order is not the sgemm's, so it is held
// to the fp64 bounds (tests/test_ddgrad3_gpu.py).
typedef unsigned int w3u2 __attribute__((ext_vector_type(2)));
constexpr int DD3_IMG = 49 * 256, DD3_IMG_DMAS = (DD3_IMG + 1023) / 1024;  // 13
constexpr int DD3_MASKB = 81 * 8, DD3_MASK0 = DD3_IMG_DMAS * 1024;
constexpr int DD3_REAL_DMAS = DD3_IMG_DMAS + 1, DD3_SLOT = DD3_REAL_DMAS * 1024, DD3_DMAS = 4;
constexpr int DD3_NSLOT = 6, DD3_ZERO = DD3_NSLOT * DD3_SLOT, DD3_LDS = DD3_ZERO + 256;
static_assert(DD3_LDS <= 160 * 1024 && DD3_REAL_DMAS <= 4 * DD3_DMAS, "ddgrad3: LDS / DMAs");

__global__ void __launch_bounds__(256, 1) ddgrad3_kernel(Args a, const u32x4* __restrict__ wq) {
    constexpr int NK = 36, NA = 60;  // k-steps (9 taps x 4 channel quarters); weight fragments in AGPRs
    constexpr int P2 = 81;           // output rows per sample
    __shared__ __attribute__((aligned(16))) uint8_t lds[DD3_LDS];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int j = wave & 1, rg = wave >> 1;
    const int r = lane & 31, h = lane >> 5;
    const long long S0 = blockIdx.x * a.batch / gridDim.x, S1 = (blockIdx.x + 1) * a.batch / gridDim.x;
    const int NS = (int)(S1 - S0);
    if (NS <= 0) return;
    const int MR = NS * P2, F_ = (MR + 63) / 64;
    const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)lds);

    // DMA d = wave + 4 i: d < 13 image bytes [1024 d, + 1024) (lane -> LDS pixel u, piece position lane & 15
    // holding global piece (lane & 15) ^ key; pixels past 48: zeros), d = 13 the bitmask words (past them:
    // the next sample's, into the slot's pad), d > 13 the 14th again
    uint32_t doff[DD3_DMAS], dkey[DD3_DMAS];
#pragma unroll
    for (int i = 0; i < DD3_DMAS; ++i) {
        int d = wave + 4 * i;
        d = d < DD3_REAL_DMAS ? d : DD3_REAL_DMAS - 1;
        const int u = (d * 1024 + lane * 16) / 256;
        const int mo = lane * 16 < DD3_MASKB ? lane * 16 : DD3_MASKB - 8;
        doff[i] = d < DD3_IMG_DMAS ? (u < 49 ? (uint32_t)(u * 256) : 0x80000000u) : (uint32_t)mo;
        dkey[i] = (uint32_t)((9 * (u / 7) + u % 7) & 15);
    }
    const uint8_t* gb = reinterpret_cast<const uint8_t*>(a.x) + S0 * DD3_IMG;
    const uint8_t* mb = reinterpret_cast<const uint8_t*>(a.bits_mask) + S0 * DD3_MASKB;
    const auto g_rs = __builtin_amdgcn_make_buffer_rsrc((void*)gb, 0, NS * DD3_IMG, 0x00020000);
    const auto m_rs = __builtin_amdgcn_make_buffer_rsrc((void*)mb, 0, NS * DD3_MASKB, 0x00020000);
    auto issue_one = [&](int n, auto I) {
        constexpr int i = decltype(I)::value;
        int d = wave + 4 * i;
        d = d < DD3_REAL_DMAS ? d : DD3_REAL_DMAS - 1;
        auto* dst = (__attribute__((address_space(3))) void*)(lds + (n % DD3_NSLOT) * DD3_SLOT + d * 1024);
        const uint32_t key = (uint32_t)(n + dkey[i]) & 15u;
        if (d < DD3_IMG_DMAS)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(g_rs, dst, 16, doff[i] + ((((uint32_t)lane & 15u) ^ key) << 4),
                                                     n * DD3_IMG, 0, 0);
        else
            __builtin_amdgcn_raw_ptr_buffer_load_lds(m_rs, dst, 16, doff[i], n * DD3_MASKB, 0, 0);
    };
    auto issue_sample = [&](int n) {
        dc_unroll([&](auto I) { issue_one(n, I); }, std::make_integer_sequence<int, DD3_DMAS>{});
    };
    int issued = NS < DD3_NSLOT ? NS : DD3_NSLOT;
    for (int n = 0; n < issued; ++n) issue_sample(n);
    // the weights of column tile j: k-step i = 2 c + s (chunk c: tap c >> 1, channel half c & 1), planes p
    u32x4 bq[NK / 2][2][2];
#pragma unroll
    for (int c = 0; c < NK / 2; ++c)
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int p = 0; p < 2; ++p) bq[c][s][p] = wq[((((c * 2 + s) * 2 + j) * 2 + p) * 64) + lane];
    const int ex = *a.xexp, ew = *a.wexp;
    const uint32_t am = amax_read(a.amax_x), nm = amax_read(a.ynorm), bm = *a.ybias;
    const int ey = bound_exp(am, nm, bm);
    const float bnd = __uint_as_float(am) * __uint_as_float(nm) + __uint_as_float(bm);
    const float sy = __builtin_isfinite(bnd) ? exp2i(ey) : __builtin_nanf("");
    const float us = exp2i(-ex) * (exp2i(-ew) * sy);  // accumulators -> the output's scaled domain (exact)
    if (blockIdx.x == 0 && threadIdx.x == 0) *a.yexp_out = ey;
    if (threadIdx.x < 16) reinterpret_cast<u32x4*>(lds + DD3_ZERO)[threadIdx.x] = u32x4{0u, 0u, 0u, 0u};

    // a lane's row: (n, iy, ix) of range row m, advanced by 64 rows per phase without divisions
    struct Pos {
        int m, n, iy, ix;
    };
    Pos Q;
    {
        Q.m = 32 * rg + r;
        Q.n = Q.m / P2;
        const int rem = Q.m - Q.n * P2;
        Q.iy = rem / 9;
        Q.ix = rem - 9 * Q.iy;
    }
    auto advance = [&](Pos& P) {  // + 64 rows = + 7 image rows and 1 column
        P.m += 64;
        P.ix += 1;
        const bool cx = P.ix >= 9;
        P.ix -= cx ? 9 : 0;
        P.iy += 7 + (cx ? 1 : 0);
        const bool cy = P.iy >= 9;
        P.iy -= cy ? 9 : 0;
        P.n += cy ? 1 : 0;
    };
    // per-lane setup of a phase: each tap's read pixel base | (key ^ h) << 4 (off the image: the zero pixel),
    // the output pixel's byte offset in the range's g2 planes, its bitmask word's LDS address
    struct Rows {
        uint32_t tb[9];
        uint32_t ma;
    };
    auto rows = [&](const Pos& P) {
        Rows R;
        const bool live = P.m < MR;
        const int n = live ? P.n : NS - 1, iy = live ? P.iy : 8, ix = live ? P.ix : 8;
        const uint32_t sbase = lds0 + (uint32_t)((n % DD3_NSLOT) * DD3_SLOT);
        const int mkey = n + 9 * iy + ix;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int ky = t / 3, kx = t % 3, y = iy - ky, x = ix - kx;
            const bool ok = y >= 0 && y <= 6 && x >= 0 && x <= 6;
            const uint32_t key = ((uint32_t)(mkey - 9 * ky - kx) & 15u) ^ (uint32_t)h;
            R.tb[t] = (ok ? sbase + (uint32_t)((7 * y + x) * 256) : lds0 + DD3_ZERO) | (key << 4);
        }
        R.ma = sbase + DD3_MASK0 + (uint32_t)((9 * iy + ix) * 8 + 4 * j);
        return R;
    };
    Rows RW = rows(Q);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    asm volatile("s_nop 4" ::: "memory");  // (VALU-written B registers before the first MFMA reads them)

    const auto o_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(reinterpret_cast<uint8_t*>(a.y) + S0 * (P2 * 256)), 0,
                                                        NS * (P2 * 256), 0x00020000);
    const uint32_t ylane = (uint32_t)(128 * j + 8 * h);
    uint32_t om = 0u;
    f32x16 H0, L0, H1, L1;
    int po = 0x7FFFFF00;  // the previous phase's output byte offset (dead rows: past the end) and mask word
    uint32_t pmw = 0u;
    // epilogue group t of the previous phase: channels 32 j + 8 t + 4 h + k of the lane's pixel, times conv2's
    // ReLU bit; the planes' two 8-B runs (a dead row's offset is past the end: the store is dropped)
    auto epi = [&](auto T, const f32x16& PH, const f32x16& PL) {
        constexpr int t = decltype(T)::value;
        float y[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint32_t mk;
            asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(mk) : "v"(pmw), "n"(8 * t + k));
            y[k] = __uint_as_float(__float_as_uint((PH[4 * t + k] + PL[4 * t + k]) * us) & mk);
        }
        uint32_t hw[2], lw[2];
        split2h((f32x2){y[0], y[1]}, 1.f, hw[0], lw[0]);
        split2h((f32x2){y[2], y[3]}, 1.f, hw[1], lw[1]);
        const uint32_t o = (uint32_t)po + ylane + 16 * t;
        __builtin_amdgcn_raw_buffer_store_b64((w3u2){hw[0], hw[1]}, o_rs, o, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b64((w3u2){lw[0], lw[1]}, o_rs, o + 64, 0, 0);
        om = max(om, max(max(__float_as_uint(y[0]) & 0x7FFFFFFFu, __float_as_uint(y[1]) & 0x7FFFFFFFu),
                         max(__float_as_uint(y[2]) & 0x7FFFFFFFu, __float_as_uint(y[3]) & 0x7FFFFFFFu)));
    };
    constexpr int NDMA = DD3_DMAS;  // refill: at most one sample per phase (64 rows < 81), from k-step 16

    auto phase = [&](int f, f32x16& H, f32x16& Lo, const f32x16& PH, const f32x16& PL, auto PREV) {
        const int m0 = 64 * f;
        const int nlo = m0 / P2, nhi = min((m0 + 63) / P2, NS - 1);
        dc_vm_wait<DD3_DMAS>(issued - 1 - nhi);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        const int rA = issued, nref = min(nlo + DD3_NSLOT, NS) - issued;
        issued += nref;
        const int live = Q.m < MR;
        const int orow = live ? Q.m * 256 : 0x7FFFFF00;
        uint32_t mw;
        asm volatile("ds_read_b32 %0, %1" : "=v"(mw) : "v"(RW.ma));
        // k-step i = 2 c + s, plane pl: piece 8 (c & 1) + 4 pl + 2 s + h of tap c >> 1's pixel
        auto addr = [&](int i, int pl) {
            const int c = i >> 1, s = i & 1;
            return RW.tb[c >> 1] ^ ((uint32_t)(8 * (c & 1) + 4 * pl + 2 * s) << 4);
        };
        constexpr int PD = DC_PD, NB = PD + 1;
        u32x4 fa[NB][2];
        auto rd1 = [&](auto I, auto PLc) {
            constexpr int i = decltype(I)::value, pl = decltype(PLc)::value;
            fa[i % NB][pl] = dc_read<0>(addr(i, pl));
        };
        using Z = std::integral_constant<int, 0>;
        using O = std::integral_constant<int, 1>;
        dc_unroll([&](auto I) { rd1(I, Z{}); rd1(I, O{}); }, std::make_integer_sequence<int, PD>{});
        asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(fa[0][0]), "+v"(fa[0][1]), "+v"(mw) : "n"(2 * (PD - 1)));
        Pos QN = Q;
        Rows RN;  // the next phase's setup, in this phase's gaps
        dc_unroll(
            [&](auto I) {
                constexpr int i = decltype(I)::value;
                constexpr int fb = (i >> 1) * 4 + (i & 1) * 2;
                constexpr bool A0 = fb < NA, A1 = fb + 1 < NA;
                const u32x4& b0 = bq[i >> 1][i & 1][0];
                const u32x4& b1 = bq[i >> 1][i & 1][1];
                constexpr bool P = decltype(PREV)::value;
                if constexpr (i == 0)
                    dc_mfma0<A0>(H, fa[0][0], b0);
                else
                    dc_mfma<A0>(H, fa[i % NB][0], b0);
                if constexpr (i + PD < NK) rd1(std::integral_constant<int, i + PD>{}, Z{});
                if constexpr (i == 0)
                    dc_mfma0<A1>(Lo, fa[0][0], b1);
                else
                    dc_mfma<A1>(Lo, fa[i % NB][0], b1);
                if constexpr (i + PD < NK) rd1(std::integral_constant<int, i + PD>{}, O{});
                // the previous phase's epilogue at k-steps 1, 3, 5, 7 — early, so its stores complete before
                // the next phase's vmcnt wait (gfx9: one counter for loads and stores)
                if constexpr (P && (i & 1) && i < 8) epi(std::integral_constant<int, i / 2>{}, PH, PL);
                dc_mfma<A0>(Lo, fa[i % NB][1], b0);
                if constexpr (i == 10) {
                    advance(QN);
                }
                if constexpr (i == 12) RN = rows(QN);
                dc_unroll(
                    [&](auto X) {
                        constexpr int x = decltype(X)::value;
                        if constexpr (16 + x * 4 == i) {
                            if (nref > 0) issue_one(rA, std::integral_constant<int, x>{});
                        }
                    },
                    std::make_integer_sequence<int, NDMA>{});
                constexpr int later = (i + PD < NK ? i + PD : NK - 1) - (i + 1);
                if constexpr (i + 1 < NK) dc_lgkm<2 * later>(fa[(i + 1) % NB][0], fa[(i + 1) % NB][1]);
            },
            std::make_integer_sequence<int, NK>{});
        for (int t = 1; t < nref; ++t) issue_sample(rA + t);  // (only phase 0 could: the prologue issued those)
        po = orow;
        pmw = mw >> (4 * h);
        Q = QN;
        RW = RN;
        dc_acc_fence(H, Lo);
    };
    auto final_epi = [&](const f32x16& PH, const f32x16& PL) {
        dc_unroll([&](auto T) { epi(T, PH, PL); }, std::make_integer_sequence<int, 4>{});
    };
    phase(0, H0, L0, H1, L1, std::false_type{});
    int f = 1;
#pragma unroll 1
    for (; f + 1 < F_; f += 2) {
        phase(f, H1, L1, H0, L0, std::true_type{});
        phase(f + 1, H0, L0, H1, L1, std::true_type{});
    }
    if (f < F_) phase(f, H1, L1, H0, L0, std::true_type{});
    if ((F_ - 1) & 1)
        final_epi(H1, L1);
    else
        final_epi(H0, L0);
    amax_record(a.amax_y, __uint_as_float(om) * exp2i(-ey));
}

// ---------------------------------------------------------------------------
// conv3 weight gradient, direct (round 5; models-checkpoint.py:57 Conv2d(64, 64, 3) trained by ppo.py:241):
//   dW3[co][ci][ky][kx] = sum over samples n and output pixels p = (oy, ox) of h2[n][oy + ky][ox + kx][ci] g3[n][p][co]
//   db3[co]             = sum g3[n][p][co]
// The im2col form (wgrad_split_kernel) stages nine copies of every h2 pixel through L2 and leaves ~400
// partial slabs at 16,384 rows.  Here one 256-thread workgroup per CU walks its own range of samples: per
// sample the PX h2 image (81 pixels x 256 B) and the PX g3 image (49 x 256 B) stream into an LDS ring by
// LDS-DMA, laid out as (channel half, plane) sub-images of 64-B rows, so the transposing LDS read
// (ds_read_b64_tr_b16; lane (h, g16, qq, pp) supplies row 8 h + 4 r + qq of a k-step, 8 B at column
// 32 g16 + 8 pp, as wgrad2_planes_kernel) builds the MFMA fragments straight from the images: A = h2 rows
// (M = the 32 input channels of a half, K = 16 output pixels read at the tap's offset), B = g3 rows (N = 32
// output channels).  A sample's 49 pixels are 4 k-steps of 16 (g3 rows 49..63 are zero: DMA'd from past the
// buffer's end, which the hardware returns as zeros).
//   * wave w: h2 channel half ca = w & 1; taps 0..3 (w < 2) or 5..8 for both output-channel halves, and the
//     centre tap 4 for output half w >> 1 — 9 tiles of 32 x 32, 27 MFMAs per k-step on every SIMD;
//   * the h2 sub-images have a row pitch of 11 slots: the 4 rows a lane quad reads for 4 consecutive output
//     pixels p sit at slot 11 (oy + ky) + ox + kx = p + const (mod 4) (7 = 11 = -1 mod 4), 4 distinct bank
//     quarters for every tap — conflict-free; g3 rows are consecutive pixels;
//   * a k-step's fragment reads (8 of g3, 4 per tap of h2) are issued one unit ahead of their MFMAs; the
//     three products of a split pair (Hh Gh, Hh Gl, Hl Gh) go into one accumulator per tile (as ddgrad2:
//     fp32-class, held to the fp64 bound by tests/test_dwgrad3_gpu.py);
//   * the bias: wave w sums the g3 fragment (output half w >> 1, plane w & 1) with v_dot2_f32_f16 x ones.
// Per-workgroup partial slabs, summed in a fixed order by wgrad_reduce (deterministic).
constexpr int W3_HP = 11;                                       // h2 sub-image row pitch (slots)
constexpr int W3_HSUB = 9 * W3_HP * 64;                         // 6,336 B: one h2 (channel half, plane) sub-image
constexpr int W3_GSUB = 64 * 64;                                // 4,096 B: one g3 sub-image (rows 49..63 zero)
constexpr int W3_H0 = 4 * W3_GSUB;                              // the h2 sub-images follow the g3 ones
constexpr int W3_REAL_DMAS = 16 + (4 * W3_HSUB + 1023) / 1024;  // 41 1-KB DMAs per sample
constexpr int W3_SLOT = W3_REAL_DMAS * 1024, W3_DMAS = (W3_REAL_DMAS + 3) / 4;  // per wave: 11
constexpr int W3_NSLOT = 3, W3_LDS = W3_NSLOT * W3_SLOT;        // 125,952 B
constexpr int W3_HIMG = 81 * 256, W3_GIMG = 49 * 256;           // PX bytes per sample
constexpr int W3_SLAB = 576 * 64;                               // floats of a partial slab
static_assert(W3_LDS <= 160 * 1024, "dwgrad3: LDS");

struct W3PArgs {
    const uint8_t* h2;  // PX h2 [batch][81][256 B]
    const uint8_t* g3;  // PX g3 [batch][49][256 B]
    const int* h_exp;   // h2 * 2^h_exp = hi + lo
    const int* g_exp;
    float* slab;   // [gridDim.x][576][64] (k = tap * 64 + ci)
    float* bslab;  // [gridDim.x][64]
    long long batch;
};

template <int OFF>
__device__ inline w3u2 w3_tr(uint32_t addr) {  // (asm: hipcc would wait for the ring's DMAs before a plain read)
    w3u2 r;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
    return r;
}
__device__ inline u32x4 w3_cat(w3u2 x0, w3u2 x1) { return u32x4{x0.x, x0.y, x1.x, x1.y}; }
template <int N>
__device__ inline void w3_lgkm(w3u2 (&x)[8]) {
    asm volatile("s_waitcnt lgkmcnt(%8)"
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7])
                 : "n"(N));
}
template <int N>
__device__ inline void w3_lgkm(w3u2 (&x)[8], w3u2 (&y)[8]) {
    asm volatile("s_waitcnt lgkmcnt(%16)"
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),
                   "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7])
                 : "n"(N));
}
// the slot offset of tap t in an h2 sub-image
template <int T>
constexpr int w3_toff() { return (W3_HP * (T / 3) + T % 3) * 64; }

__global__ void __launch_bounds__(256, 1) dwgrad3_kernel(W3PArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[W3_LDS];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ca = wave & 1, hb = wave >> 1;
    const long long S0 = blockIdx.x * a.batch / gridDim.x, S1 = (blockIdx.x + 1) * a.batch / gridDim.x;
    const int NS = (int)(S1 - S0);  // >= 1 (grid <= batch)
    const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)lds);

    // DMA d = wave + 4 i (past the 41st: the 41st again) fills slot bytes [1024 d, 1024 d + 1024).  d < 16: g3
    // sub-image d >> 2 = 2 b + P, rows 16 (d & 3) + (lane >> 2), piece lane & 3 (rows >= 49: past the end, zeros);
    // else h2: byte e = 1024 (d - 16) + 16 lane of the h2 sub-images, sub-image e / W3_HSUB = 2 ca + P, slot
    // (e % W3_HSUB) >> 6 = 11 iy + ix (ix >= 9 and the tail past the 4th sub-image: zeros)
    uint32_t doff[W3_DMAS];
#pragma unroll
    for (int i = 0; i < W3_DMAS; ++i) {
        int d = wave + 4 * i;
        d = d < W3_REAL_DMAS ? d : W3_REAL_DMAS - 1;
        if (d < 16) {
            const int row = 16 * (d & 3) + (lane >> 2);
            doff[i] = row < 49 ? (uint32_t)(row * 256 + (d >> 2) * 64 + (lane & 3) * 16) : 0x80000000u;
        } else {
            const int e = 1024 * (d - 16) + 16 * lane, sh = e / W3_HSUB, sl = (e % W3_HSUB) >> 6;
            const int iy = sl / W3_HP, ix = sl % W3_HP;
            doff[i] = (sh < 4 && ix < 9) ? (uint32_t)((9 * iy + ix) * 256 + sh * 64 + ((e >> 4) & 3) * 16)
                                         : 0x80000000u;
        }
    }
    const auto h_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(a.h2 + S0 * W3_HIMG), 0, NS * W3_HIMG, 0x00020000);
    const auto g_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(a.g3 + S0 * W3_GIMG), 0, NS * W3_GIMG, 0x00020000);
    auto issue_sample = [&](int n) {
        const int slot = n % W3_NSLOT;
        dc_unroll(
            [&](auto I) {
                constexpr int i = decltype(I)::value;
                int d = wave + 4 * i;
                d = d < W3_REAL_DMAS ? d : W3_REAL_DMAS - 1;
                auto* dst = (__attribute__((address_space(3))) void*)(lds + slot * W3_SLOT + d * 1024);
                if (d < 16)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(g_rs, dst, 16, doff[i], n * W3_GIMG, 0, 0);
                else
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(h_rs, dst, 16, doff[i], n * W3_HIMG, 0, 0);
            },
            std::make_integer_sequence<int, W3_DMAS>{});
    };
    const int ahead = NS < W3_NSLOT - 1 ? NS : W3_NSLOT - 1;
    for (int n = 0; n < ahead; ++n) issue_sample(n);

    // per-lane fragment row addresses (slot 0): k-step ks, row quad r -> output pixel p (rows past 48: pixel 48,
    // whose g3 partner rows are zero)
    const int h = lane >> 5, g16 = (lane >> 4) & 1, qq = (lane >> 2) & 3, pp = lane & 3;
    const uint32_t lcol = (uint32_t)(g16 * 32 + pp * 8);
    uint32_t abase[4][2];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            int p = 16 * ks + 8 * h + 4 * r + qq;
            p = p < 49 ? p : 48;
            abase[ks][r] = lds0 + W3_H0 + (uint32_t)(ca * 2 * W3_HSUB + (W3_HP * (p / 7) + p % 7) * 64) + lcol;
        }
    const uint32_t bbase = lds0 + (uint32_t)((8 * h + qq) * 64) + lcol;

    f32x16 acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t] = zero16();
    float bsum = 0.f;
    const f16x2 ones = {(_Float16)1.0f, (_Float16)1.0f};

    // one sample: 16 units (k-step ks, tap slot j: j < 3 one tap x both output halves, j = 3 the tap-half's
    // last tap x both halves + the centre tap x half hb); unit u + 1's reads are issued before unit u's MFMAs.
    // One code path for every wave (a branch on the tap half made hipcc shuttle the 144 accumulators between
    // AGPRs and VGPRs around it): the tap half is a uniform per-slot address delta, the centre tap's output
    // half a select of the g3 fragment
    int tdel[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) tdel[j] = hb ? (W3_HP * ((5 + j) / 3) + (5 + j) % 3 - (W3_HP * (j / 3) + j % 3)) * 64 : 0;
    auto sample = [&](uint32_t so) {
        uint32_t ab[4][2], bb = bbase + so;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
#pragma unroll
            for (int r = 0; r < 2; ++r) ab[ks][r] = abase[ks][r] + so;
        asm volatile("" : "+v"(bb), "+v"(ab[0][0]), "+v"(ab[0][1]), "+v"(ab[1][0]), "+v"(ab[1][1]), "+v"(ab[2][0]),
                     "+v"(ab[2][1]), "+v"(ab[3][0]), "+v"(ab[3][1]));
        w3u2 ra[2][8];  // [unit parity][(tap slot, plane, r)]
        w3u2 rb[2][8];  // [k-step parity][(half, plane, r)]
        auto reads = [&](auto U) {
            constexpr int u = decltype(U)::value, ks = u >> 2, j = u & 3;
            if constexpr (j == 0) {
                dc_unroll(
                    [&](auto X) {
                        constexpr int x = decltype(X)::value, b = x >> 2, P = (x >> 1) & 1, r = x & 1;
                        rb[ks & 1][x] = w3_tr<(2 * b + P) * W3_GSUB + ks * 1024 + r * 256>(bb);
                    },
                    std::make_integer_sequence<int, 8>{});
            }
            constexpr int nt = j == 3 ? 2 : 1;
            uint32_t at[2] = {ab[ks][0] + (uint32_t)tdel[j], ab[ks][1] + (uint32_t)tdel[j]};
            dc_unroll(
                [&](auto X) {
                    constexpr int x = decltype(X)::value, s = x >> 2, P = (x >> 1) & 1, r = x & 1;
                    if constexpr (s == 0)
                        ra[u & 1][x] = w3_tr<P * W3_HSUB + w3_toff<j>()>(at[r]);
                    else
                        ra[u & 1][x] = w3_tr<P * W3_HSUB + w3_toff<4>()>(ab[ks][r]);
                },
                std::make_integer_sequence<int, 4 * nt>{});
        };
        reads(std::integral_constant<int, 0>{});
        dc_unroll(
            [&](auto U) {
                constexpr int u = decltype(U)::value, ks = u >> 2, j = u & 3;
                if constexpr (u + 1 < 16) {
                    reads(std::integral_constant<int, u + 1>{});
                    // the reads issued after unit u's: unit u + 1's
                    constexpr int later = ((u + 1) & 3) == 0 ? 8 + 4 : (((u + 1) & 3) == 3 ? 8 : 4);
                    if constexpr (j == 0)
                        w3_lgkm<later>(ra[u & 1], rb[ks & 1]);
                    else
                        w3_lgkm<later>(ra[u & 1]);
                } else {
                    w3_lgkm<0>(ra[u & 1]);
                }
                u32x4 A[2][2], B[2][2];
#pragma unroll
                for (int b = 0; b < 2; ++b)
#pragma unroll
                    for (int P = 0; P < 2; ++P) B[b][P] = w3_cat(rb[ks & 1][b * 4 + P * 2], rb[ks & 1][b * 4 + P * 2 + 1]);
#pragma unroll
                for (int s = 0; s < 2; ++s)
#pragma unroll
                    for (int P = 0; P < 2; ++P) A[s][P] = w3_cat(ra[u & 1][s * 4 + P * 2], ra[u & 1][s * 4 + P * 2 + 1]);
                if constexpr (j == 0) {  // the bias: fragment (hb, ca) of this k-step
                    const u32x4 bh = hb ? B[1][0] : B[0][0], bl = hb ? B[1][1] : B[0][1];
                    const u32x4 bv = ca ? bl : bh;
                    // (the element copied out first: hipcc's bit_cast of an ext-vector element lvalue read
                    // element 0 for every e)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const uint32_t w = bv[e];
                        bsum = __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, w), ones, bsum, false);
                    }
                }
                constexpr int PA[3] = {0, 0, 1}, PB[3] = {0, 1, 0};
                u32x4 B4[2];
                if constexpr (j == 3) {
                    B4[0] = hb ? B[1][0] : B[0][0];
                    B4[1] = hb ? B[1][1] : B[0][1];
                }
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    acc[2 * j] = mfma_f16(A[0][PA[k]], B[0][PB[k]], acc[2 * j]);
                    acc[2 * j + 1] = mfma_f16(A[0][PA[k]], B[1][PB[k]], acc[2 * j + 1]);
                    if constexpr (j == 3) acc[8] = mfma_f16(A[1][PA[k]], B4[PB[k]], acc[8]);
                }
            },
            std::make_integer_sequence<int, 16>{});
    };

#pragma unroll 1
    for (int n = 0; n < NS; ++n) {
        dc_vm_wait<W3_DMAS>(n + 1 < NS ? 1 : 0);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (n + W3_NSLOT - 1 < NS) issue_sample(n + W3_NSLOT - 1);  // into sample n - 1's slot (all waves past it)
        sample((uint32_t)((n % W3_NSLOT) * W3_SLOT));
    }

    // one exponent at a time (their sum can leave exp2i's range: a tiny g3's exponent is clamped at 126)
    const float uo = exp2i(-*a.h_exp), uog = exp2i(-*a.g_exp);
    float* slab = a.slab + (long long)blockIdx.x * W3_SLAB;
    auto store_tile = [&](const f32x16& C, int tap, int b) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int k = tap * 64 + 32 * ca + (r & 3) + 8 * (r >> 2) + 4 * h;
            slab[k * 64 + 32 * b + (lane & 31)] = (C[r] * uo) * uog;
        }
    };
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        store_tile(acc[2 * j], hb ? 5 + j : j, 0);
        store_tile(acc[2 * j + 1], hb ? 5 + j : j, 1);
    }
    store_tile(acc[8], 4, hb);
    // bias: lane (c, h) of wave 2 b + P holds plane P's partial of channel 32 b + c over rows of half h
    __syncthreads();  // (every wave's last fragment reads are done)
    float* red = reinterpret_cast<float*>(lds);
    red[wave * 64 + lane] = bsum;
    __syncthreads();
    if (threadIdx.x < 64) {
        const int b = threadIdx.x >> 5, c = threadIdx.x & 31;
        const float th = red[(2 * b) * 64 + c] + red[(2 * b) * 64 + c + 32];
        const float tl = red[(2 * b + 1) * 64 + c] + red[(2 * b + 1) * 64 + c + 32];
        a.bslab[(long long)blockIdx.x * 64 + threadIdx.x] = (th + tl) * exp2i(-*a.g_exp);
    }
}

int dconv_cus() {
    static int cus[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    if (cus[dev] == 0 && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus[dev] = 0;
    return cus[dev];
}

bool env_on(const char* name, long long batch, bool dflt, long long dflt_min = 1) {
    const char* e = ppox::ab_env(name);
    if (!(e ? e[0] != '0' : dflt)) return false;
    char mn[64];
    snprintf(mn, sizeof mn, "%s_MIN", name);
    const char* m = ppox::ab_env(mn);
    return batch >= (m ? std::atoll(m) : dflt_min);
}

template <class F>
int launch_dconv(const Args& a, const uint16_t* wq, hipStream_t s, const char* name) {
    const int cus = dconv_cus();
    PPOX_REQUIRE(cus > 0, "%s: no device", name);
    PPOX_REQUIRE(a.xexp && a.yexp_out && a.amax_x && a.ybias && a.ynorm, "%s: the direct form needs PX operands",
                 name);
    const long long grid = std::min<long long>(a.batch, cus);
    const u32x4* w = reinterpret_cast<const u32x4*>(wq);
    if (a.bits_y)
        dconv_fwd_kernel<F, true><<<(unsigned)grid, 256, 0, s>>>(a, w);
    else
        dconv_fwd_kernel<F, false><<<(unsigned)grid, 256, 0, s>>>(a, w);
    PPOX_LAUNCHED(name);
}

}  // namespace

#ifndef DFCD_DEFAULT
#define DFCD_DEFAULT true  // the direct fc dgrad unless PPOX_DFCD says otherwise
#endif
#ifndef DDGRAD3_DEFAULT
#define DDGRAD3_DEFAULT true  // the direct conv3 dgrad (PX g3 -> PX g2) unless PPOX_DDGRAD3 says otherwise
#endif
#ifndef FCW_DEFAULT
#define FCW_DEFAULT true
#endif
#ifndef FCW_MIN
#define FCW_MIN 8192
#endif
#ifndef FCW_SK_MIN
#define FCW_SK_MIN 1024
#endif
#ifndef DDGRAD3_MIN
#define DDGRAD3_MIN 4096
#endif
#ifndef DWGRAD3_DEFAULT
#define DWGRAD3_DEFAULT true  // the direct conv3 weight gradient unless PPOX_DWGRAD3 says otherwise
#endif
#ifndef DCONV_DEFAULT
#define DCONV_DEFAULT true  // the direct forms unless PPOX_DCONV2 / PPOX_DCONV3 say otherwise
#endif

namespace ppox_conv {
// PPOX_DCONV3=0 / PPOX_DCONV2=0: the im2col sg2 GEMM instead; PPOX_DCONV3_MIN / PPOX_DCONV2_MIN: the
// smallest batch the direct form runs at (default 1).  Read at every launch: the tests switch forms
// within one process.
bool dconv_enabled(int layer, long long batch) {
    return env_on(layer == 2 ? "PPOX_DCONV2" : "PPOX_DCONV3", batch, DCONV_DEFAULT);
}

// conv3 forward, h2 planes in / h3 planes out; conv2 forward, H1P in / h2 planes out (x_exp: the H1P
// exponent) — one workgroup per CU, each a contiguous range of samples
int dconv_fwd(int layer, const void* x, int64_t batch, const uint16_t* wq, const float* bias, float* y,
              const uint32_t* amax_x, uint32_t* amax_y, uint32_t* relu_bits, const int* x_exp, int* y_exp_out,
              hipStream_t s) {
    Args a{x, nullptr, 0, 0, 0, nullptr, bias, nullptr, y, batch, amax_x, amax_y, pack_exp(wq, planes(layer))};
    a.bits_y = relu_bits;
    a.xexp = x_exp;
    a.yexp_out = y_exp_out;
    a.ynorm = pack_norm(wq, planes(layer));
    a.ybias = pack_bmax(wq, planes(layer));
    if (layer == 2) return launch_dconv<DcF2>(a, wq, s, "ppox_nature_conv2_fwd_planes");
    return launch_dconv<DcF3>(a, wq, s, "ppox_nature_conv_fwd_split");
}

// the conv2 dgrad on PX g2 (one workgroup per CU, each a contiguous range of samples)
int ddgrad2(const void* g2p, int64_t batch, const uint16_t* wqd2, float* g1, const uint32_t* relu_bits,
            uint32_t* amax_g1, const int* g_exp, const int* wexp, hipStream_t s) {
    const int cus = dconv_cus();
    PPOX_REQUIRE(cus > 0, "ppox_nature_conv_dgrad_split: no device");
    PPOX_REQUIRE(ppox::aligned16(g2p) && ppox::aligned16(g1) && ppox::aligned16(relu_bits) && g_exp && wexp,
                 "ppox_nature_conv_dgrad_split: the direct conv2 dgrad needs 16B-aligned g2 planes, g1, bitmask");
    Args a{g2p, nullptr, 0, 0, 0, nullptr, nullptr, nullptr, g1, batch, nullptr, amax_g1, wexp};
    a.bits_mask = relu_bits;
    a.xexp = g_exp;
    const long long grid = std::min<long long>(batch, cus);
    ddgrad2_kernel<<<(unsigned)grid, 256, 0, s>>>(a, reinterpret_cast<const u32x4*>(wqd2));
    PPOX_LAUNCHED("ppox_nature_conv_dgrad_split");
}

// the fc forward on PX h3 in 256 x 128 tiles (PPOX_FCW=0: the sg2 GEMM; _MIN: the smallest batch, default
// 8192: one tile per CU needs 16,384 rows, and below ~8,192 the split-K form fills the chip)
bool fcw_enabled(long long batch) { return env_on("PPOX_FCW", batch, FCW_DEFAULT, FCW_MIN); }
int fcw(const void* h3p, int64_t batch, const uint16_t* q_fwd, const float* bias, float* f, uint32_t* amax_f,
        const int* h3_exp, const int* wexp, hipStream_t s) {
    PPOX_REQUIRE(ppox::aligned16(h3p) && ppox::aligned16(q_fwd) && bias && f && h3_exp && wexp,
                 "ppox_nature_fc_fwd: the wide form needs PX h3 (16B-aligned)");
    Args a{h3p, nullptr, 0, 0, 0, nullptr, bias, nullptr, f, batch, nullptr, amax_f, wexp};
    a.xexp = h3_exp;
    const long long grid = ppox::ceil_div((long long)batch, (long long)FCW_ROWS) * 4;
    fcw_kernel<1><<<(unsigned)grid, 512, 0, s>>>(a, reinterpret_cast<const u32x4*>(q_fwd));
    PPOX_LAUNCHED("ppox_nature_fc_fwd");
}
// split over K (8 ways) into slab [8][batch][512] (the caller's fc_fwd_sk_reduce adds them): batches from
// PPOX_FCW_SK_MIN (1024) below the full-tile form's
bool fcw_sk_enabled(long long batch) {
    return env_on("PPOX_FCW", batch, FCW_DEFAULT, FCW_SK_MIN) && !fcw_enabled(batch);
}
int fcw_sk(const void* h3p, int64_t batch, const uint16_t* q_fwd, float* slab, const int* h3_exp, const int* wexp,
           hipStream_t s) {
    PPOX_REQUIRE(ppox::aligned16(h3p) && ppox::aligned16(q_fwd) && slab && h3_exp && wexp,
                 "ppox_nature_fc_fwd_splitk: the wide form needs PX h3 (16B-aligned)");
    Args a{h3p, nullptr, 0, 0, 0, nullptr, nullptr, nullptr, slab, batch, nullptr, nullptr, wexp};
    a.xexp = h3_exp;
    const long long grid = ppox::ceil_div((long long)batch, (long long)FCW_ROWS) * 4 * FCW_SK;
    fcw_kernel<FCW_SK><<<(unsigned)grid, 512, 0, s>>>(a, reinterpret_cast<const u32x4*>(q_fwd));
    PPOX_LAUNCHED("ppox_nature_fc_fwd_splitk");
}

// the heads' backward to the fc output in one launch (hbw_kernel): de and df (f32, masked), their amax
int head_backward(const float* dout, const float* wa, const float* dv, const float* wc, const float* e, const float* f,
                  const uint16_t* qhd, const int* wexp, int64_t rows, int n_out, float* df, float* de,
                  uint32_t* amax_de, uint32_t* amax_df, hipStream_t s) {
    if (rows == 0) return PPOX_OK;
    const int cus = dconv_cus();
    PPOX_REQUIRE(cus > 0, "ppox_head_backward: no device");
    PPOX_REQUIRE(n_out >= 1 && n_out <= 8, "ppox_head_backward: n_out must be 1..8");
    PPOX_REQUIRE(ppox::aligned16(wa) && ppox::aligned16(e) && ppox::aligned16(f) && ppox::aligned16(df) &&
                     ppox::aligned16(de) && ppox::aligned16(qhd),
                 "ppox_head_backward: 16B alignment (w_actor, e, f, df, de, q)");
    PPOX_REQUIRE(wc && dv && dout, "ppox_head_backward: null w_critic / dv / dout");
    const int nrg = (int)std::max<long long>(1, std::min<long long>(cus / 4, ppox::ceil_div((long long)rows, 32LL)));
    HbwArgs a{dout, wa, dv, wc, e, f, df, de, amax_de, amax_df, wexp, rows, nrg};
    const u32x4* w = reinterpret_cast<const u32x4*>(qhd);
    const unsigned grid = (unsigned)(4 * nrg);
    switch (n_out) {
#define PPOX_HBW(N) \
    case N: hbw_kernel<N><<<grid, 256, 0, s>>>(a, w); break;
        PPOX_HBW(1) PPOX_HBW(2) PPOX_HBW(3) PPOX_HBW(4) PPOX_HBW(5) PPOX_HBW(6) PPOX_HBW(7) PPOX_HBW(8)
#undef PPOX_HBW
    }
    PPOX_LAUNCHED("ppox_head_backward");
}

// the conv3 dgrad's direct form on PX g3 -> PX g2 (PPOX_DDGRAD3=0: the im2col sgemm; _MIN: the smallest
// batch); `a` carries the PX g2 arguments the sgemm form takes (x, xexp, wexp, amax_x, ynorm, ybias, y,
// yexp_out, amax_y, bits_mask)
// (from 4,096 rows: at the 8-GPU per-rank minibatch of 2,048 it measured 205.6 vs 199.9 ms per iteration
// against the sgemm, the persistent direct kernels of both streams taking whole CUs in turn)
bool ddgrad3_enabled(long long batch) { return env_on("PPOX_DDGRAD3", batch, DDGRAD3_DEFAULT, DDGRAD3_MIN); }
int ddgrad3(const void* g3p, int64_t batch, const uint16_t* wqd3, void* g2p, const uint32_t* amax_g3,
            uint32_t* amax_g2, const uint32_t* relu_bits, const int* g_exp, const int* wexp, const uint32_t* ynorm,
            const uint32_t* ybias, int* y_exp_out, hipStream_t s) {
    const int cus = dconv_cus();
    PPOX_REQUIRE(cus > 0, "ppox_nature_conv_dgrad_split: no device");
    PPOX_REQUIRE(ppox::aligned16(g3p) && ppox::aligned16(g2p) && relu_bits && g_exp && wexp && y_exp_out && amax_g3 &&
                     ynorm && ybias,
                 "ppox_nature_conv_dgrad_split: the direct conv3 dgrad needs PX g3 / g2 and the bound's operands");
    PPOX_REQUIRE(ppox::ceil_div((long long)batch, (long long)cus) * 81 * 256 < (1LL << 31),
                 "ppox_nature_conv_dgrad_split: batch too large for the direct conv3 dgrad");
    Args a{g3p, nullptr, 0, 0, 0, nullptr, nullptr, nullptr, reinterpret_cast<float*>(g2p), batch, amax_g3, amax_g2,
           wexp};
    a.bits_mask = relu_bits;
    a.xexp = g_exp;
    a.yexp_out = y_exp_out;
    a.ynorm = ynorm;
    a.ybias = ybias;
    const long long grid = std::min<long long>(batch, cus);
    ddgrad3_kernel<<<(unsigned)grid, 256, 0, s>>>(a, reinterpret_cast<const u32x4*>(wqd3));
    PPOX_LAUNCHED("ppox_nature_conv_dgrad_split");
}

// the conv3 weight gradient's direct form (PPOX_DWGRAD3=0: the im2col split form; _MIN: the smallest batch)
bool dwgrad3_enabled(long long batch) { return env_on("PPOX_DWGRAD3", batch, DWGRAD3_DEFAULT); }
long long dwgrad3_grid(long long batch) { return std::min<long long>(batch, dconv_cus()); }
int dwgrad3(const void* h2p, const void* g3p, int64_t batch, const int* h_exp, const int* g_exp, float* slab,
            float* bslab, hipStream_t s) {
    const long long grid = dwgrad3_grid(batch);
    PPOX_REQUIRE(grid > 0, "ppox_nature_conv_wgrad_split: no device");
    PPOX_REQUIRE(ppox::aligned16(h2p) && ppox::aligned16(g3p) && h_exp && g_exp,
                 "ppox_nature_conv_wgrad_split: the direct conv3 weight gradient needs 16B-aligned PX h2 / g3");
    PPOX_REQUIRE(ppox::ceil_div((long long)batch, grid) * W3_HIMG < (1LL << 31),
                 "ppox_nature_conv_wgrad_split: batch too large for the direct conv3 weight gradient");
    W3PArgs a{reinterpret_cast<const uint8_t*>(h2p), reinterpret_cast<const uint8_t*>(g3p), h_exp, g_exp, slab, bslab,
              batch};
    dwgrad3_kernel<<<(unsigned)grid, 256, 0, s>>>(a);
    PPOX_LAUNCHED("ppox_nature_conv_wgrad_split");
}

// the fc dgrad's direct form (PPOX_DFCD=1; _MIN: the smallest batch): df planes in, g3 planes out, h3's bitmask
bool dfcd_enabled(long long batch) { return env_on("PPOX_DFCD", batch, DFCD_DEFAULT); }
int dfcd(const void* dfp, int64_t batch, const uint16_t* wq, float* g3, const uint32_t* amax_df, uint32_t* amax_g3,
         const uint32_t* relu_bits, int* g3_exp_out, const int* df_exp, const int* wexp, const uint32_t* ynorm,
         const uint32_t* ybias, hipStream_t s) {
    const int cus = dconv_cus();
    PPOX_REQUIRE(cus > 0, "ppox_nature_fc_dgrad: no device");
    Args a{dfp, nullptr, 0, 0, 0, nullptr, nullptr, nullptr, g3, batch, amax_df, amax_g3, wexp};
    a.bits_mask = relu_bits;
    a.xexp = df_exp;
    a.yexp_out = g3_exp_out;
    a.ynorm = ynorm;
    a.ybias = ybias;
    constexpr int ngroups = (FCD_TILES + 3) / 4;
    const int nrg = (int)std::max<long long>(1, std::min<long long>(cus / ngroups, batch));
    fcd_kernel<<<(unsigned)(ngroups * nrg), 256, 0, s>>>(a, reinterpret_cast<const u32x4*>(wq), nrg);
    PPOX_LAUNCHED("ppox_nature_fc_dgrad");
}
}  // namespace ppox_conv
