// Cost of a fork point on the producing stream (dev probe): N x (kernel; event record) vs N x kernel vs N x
// hipExtLaunchKernelGGL(kernel, stop event), with the event's flags varied; another stream waits on every event
// (the backward's fork pattern).  Prints us per iteration.  Build: hipcc --offload-arch=gfx950 -O2 -o
// /tmp/event_probe tools/event_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>

__global__ void busy(float* p, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    float v = p[i];
#pragma unroll 1
    for (int k = 0; k < n; ++k) v = v * 1.0000001f + 1e-7f;
    p[i] = v;
}

__global__ void side_kernel(float* p) { p[threadIdx.x] += 1.f; }

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                 \
            return 1;                                                      \
        }                                                                  \
    } while (0)

int main() {
    const int N = 400, WORK = 2000, G = 1024;
    float *p, *q;
    CK(hipMalloc(&p, G * 256 * sizeof(float)));
    CK(hipMalloc(&q, 256 * sizeof(float)));
    hipStream_t s, side;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithPriority(&side, hipStreamNonBlocking, -1));
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    const unsigned flag_sets[3] = {hipEventDisableTiming, hipEventDisableTiming | 0x20000000u, 0u};
    const char* flag_names[3] = {"disable_timing", "disable_timing|no_system_fence", "default(timing)"};
    for (int mode = 0; mode < 3; ++mode)
        for (int fs = 0; fs < 3; ++fs) {
            if (mode == 0 && fs > 0) continue;
            hipEvent_t ev;
            CK(hipEventCreateWithFlags(&ev, flag_sets[fs]));
            for (int rep = 0; rep < 2; ++rep) {  // rep 0 warms up
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(t0, s));
                for (int i = 0; i < N; ++i) {
                    if (mode == 2) {
                        hipExtLaunchKernelGGL(busy, dim3(G), dim3(256), 0, s, nullptr, ev, 0, p, WORK);
                    } else {
                        busy<<<G, 256, 0, s>>>(p, WORK);
                        if (mode == 1) CK(hipEventRecord(ev, s));
                    }
                    if (mode != 0) {
                        CK(hipStreamWaitEvent(side, ev, 0));
                        side_kernel<<<1, 256, 0, side>>>(q);
                    }
                }
                CK(hipEventRecord(t1, s));
                CK(hipDeviceSynchronize());
                float ms = 0.f;
                CK(hipEventElapsedTime(&ms, t0, t1));
                if (rep == 1)
                    printf("%-22s %-32s %8.2f us per iteration\n",
                           mode == 0 ? "kernels only" : mode == 1 ? "kernel + record" : "ext launch stop event",
                           mode == 0 ? "-" : flag_names[fs], 1000.f * ms / N);
            }
            CK(hipEventDestroy(ev));
        }
    return 0;
}
