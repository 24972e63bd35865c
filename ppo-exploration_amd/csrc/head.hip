// NatureCNN head backward helpers (the elementwise parts of the explicit training
// backward of CnnActorCritic, models.py; .ipynb_checkpoints/models-checkpoint.py:60-87):
//   ppox_relu_backward_:    g = act > 0 ? g : 0 (in place) — nn.ReLU backward
//   ppox_outer_relu_backward: d[b][j] = dv[b] * w[j] * (act[b][j] > 0) — the grad of
//       a ReLU layer feeding a Linear(H, 1) critic (extra_layer -> critic_ext)
// One pass each, float4 lanes (HBM-bound: 12 B / element).
#include "common.h"

namespace {

__global__ void __launch_bounds__(256) relu_bwd_kernel(float* __restrict__ g, const float* __restrict__ act,
                                                       long long n4) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
        float4 v = reinterpret_cast<float4*>(g)[i];
        const float4 a = reinterpret_cast<const float4*>(act)[i];
        v.x = a.x > 0.f ? v.x : 0.f;
        v.y = a.y > 0.f ? v.y : 0.f;
        v.z = a.z > 0.f ? v.z : 0.f;
        v.w = a.w > 0.f ? v.w : 0.f;
        reinterpret_cast<float4*>(g)[i] = v;
    }
}

__global__ void __launch_bounds__(256) outer_relu_kernel(const float* __restrict__ dv, const float* __restrict__ w,
                                                         const float* __restrict__ act, long long rows, int h4,
                                                         float* __restrict__ d) {
    const long long n4 = rows * h4;
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
    }
}

unsigned grid_for(long long n4) {
    const long long g = (n4 + 255) / 256;
    return (unsigned)(g < 4096 ? (g > 0 ? g : 1) : 4096);
}

}  // namespace

extern "C" int ppox_relu_backward_(float* grad, const float* act, int64_t n, void* stream) {
    PPOX_REQUIRE(grad && act && n >= 0 && n % 4 == 0, "ppox_relu_backward_: bad arguments (n % 4 == 0)");
    PPOX_REQUIRE(ppox::aligned16(grad) && ppox::aligned16(act), "ppox_relu_backward_: 16B alignment");
    if (n == 0) return PPOX_OK;
    relu_bwd_kernel<<<grid_for(n / 4), 256, 0, ppox::as_stream(stream)>>>(grad, act, n / 4);
    PPOX_LAUNCHED("ppox_relu_backward_");
}

extern "C" int ppox_outer_relu_backward(const float* dv, const float* w, const float* act, int64_t rows, int64_t h,
                                        float* out, void* stream) {
    PPOX_REQUIRE(dv && w && act && out && rows >= 0 && h > 0 && h % 4 == 0, "ppox_outer_relu_backward: bad arguments");
    PPOX_REQUIRE(ppox::aligned16(act) && ppox::aligned16(out),
                 "ppox_outer_relu_backward: 16B alignment");
    if (rows == 0) return PPOX_OK;
    outer_relu_kernel<<<grid_for(rows * h / 4), 256, 0, ppox::as_stream(stream)>>>(dv, w, act, rows, (int)(h / 4), out);
    PPOX_LAUNCHED("ppox_outer_relu_backward");
}
