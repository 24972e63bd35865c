// Grid barrier vs kernel boundary (dev probe): the cost of one cooperative_groups grid.sync() inside a
// cooperative launch against one more dependent launch of a trivial kernel on the same stream.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/coop_probe tools/coop_probe.hip ; run: /tmp/coop_probe
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>

#include <cstdio>

namespace cg = cooperative_groups;

__global__ void tiny(float* x) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    x[i] = x[i] * 0.5f + 1.0f;
}

__global__ void synced(float* x, int rounds) {
    cg::grid_group g = cg::this_grid();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    for (int r = 0; r < rounds; ++r) {
        x[i] = x[i] * 0.5f + 1.0f;
        g.sync();
    }
}

#define CK(e)                                                                \
    do {                                                                     \
        hipError_t s_ = (e);                                                 \
        if (s_ != hipSuccess) {                                              \
            std::printf("%s failed: %s\n", #e, hipGetErrorString(s_));       \
            return 1;                                                        \
        }                                                                    \
    } while (0)

int main() {
    int dev = 0, cus = 0, coop = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    CK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev));
    std::printf("CUs %d cooperative %d\n", cus, coop);
    float* x = nullptr;
    CK(hipMalloc(&x, sizeof(float) * 4096 * 1024));
    CK(hipMemset(x, 0, sizeof(float) * 4096 * 1024));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int blocks : {256, 512, 1024}) {
        int per_cu = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(synced), 256, 0));
        if (per_cu * cus < blocks) {
            std::printf("blocks %d: not co-resident (%d per CU)\n", blocks, per_cu);
            continue;
        }
        const int R = 2000;
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipEventRecord(a, s));
            for (int r = 0; r < R; ++r) tiny<<<blocks, 256, 0, s>>>(x);
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float ms_l = 0.f;
            CK(hipEventElapsedTime(&ms_l, a, b));
            int rounds = R;
            void* args[] = {&x, &rounds};
            CK(hipEventRecord(a, s));
            CK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(synced), dim3(blocks), dim3(256), args, 0, s));
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float ms_s = 0.f;
            CK(hipEventElapsedTime(&ms_s, a, b));
            std::printf("blocks %4d: dependent launch %.2f us each, grid.sync %.2f us each\n", blocks,
                        ms_l * 1e3f / R, ms_s * 1e3f / R);
        }
    }
    CK(hipFree(x));
    return 0;
}
