// Cross-stream freshness of a small value written by one kernel and read by kernels of another stream (dev
// probe, round 6: the per-pass exponent / amax table the backward's side stream reads).  Per iteration:
//   side: R0 reads the word (every XCD's workgroups: the line may then sit in their caches)
//   side -> main event; main: W writes the word = iteration (one lane, one workgroup)
//   main -> side event; side: R reads the word in 2,048 workgroups and counts the ones that see another value
// for readers by scalar load, vector load, agent-scope (sc1) load and atomic add of 0; the writer by a plain or an
// agent-scope store; event flags default / no system fence; the side stream high or default priority; a "busy"
// variant keeps a long kernel running on a third stream meanwhile.  Prints the stale-read counts.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/probes/stale_probe.bin tools/probes/stale_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                 \
            return 1;                                                      \
        }                                                                  \
    } while (0)

template <int MODE>
__global__ void __launch_bounds__(64) reader(unsigned* buf, int z, unsigned want, unsigned* err, unsigned* sink) {
    unsigned v;
    if constexpr (MODE == 0) {
        v = buf[0];  // uniform: a scalar load
    } else if constexpr (MODE == 1) {
        v = buf[z * threadIdx.x];  // a vector load (z = 0 at run time)
    } else if constexpr (MODE == 2) {
        v = __hip_atomic_load(buf + z * threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        v = atomicAdd(buf + z * threadIdx.x, (unsigned)z);  // (a literal 0 becomes an sc1 load)
    }
    if (threadIdx.x == 0) {
        if (want != 0xffffffffu && v != want) {
            atomicAdd(err, 1u);
            atomicMax(err + 1, want - v);
        }
        if (v == 0xdeadbeefu) sink[blockIdx.x] = v;
    }
}

template <int MODE>
__global__ void writer(unsigned* buf, unsigned v) {
    if (threadIdx.x == 0) {
        if constexpr (MODE == 0)
            buf[0] = v;
        else
            __hip_atomic_store(buf, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void busy(float* p, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    float v = p[i];
#pragma unroll 1
    for (int k = 0; k < n; ++k) v = v * 1.0000001f + 1e-7f;
    p[i] = v;
}

typedef void (*ReaderFn)(unsigned*, int, unsigned, unsigned*, unsigned*);

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 3000;
    const int G = 2048;
    unsigned *buf, *err, *sink;
    float* bp;
    CK(hipMalloc(&buf, 4096));
    CK(hipMalloc(&err, 64));
    CK(hipMalloc(&sink, G * 4));
    CK(hipMalloc(&bp, 256 * 64 * 4));
    CK(hipMemset(bp, 0, 256 * 64 * 4));
    hipStream_t third;
    CK(hipStreamCreateWithFlags(&third, hipStreamNonBlocking));
    const ReaderFn readers[4] = {reader<0>, reader<1>, reader<2>, reader<3>};
    const char* rnames[4] = {"scalar", "vector", "sc1", "atomic"};
    const unsigned eflags[2] = {0u, 0x20000000u};
    const char* enames[2] = {"fence", "nofence"};
    unsigned it = 1;
    for (int prio = -1; prio <= 0; ++prio)
        for (int bz = 0; bz < 2; ++bz)
            for (int ef = 0; ef < 2; ++ef)
                for (int wm = 0; wm < 2; ++wm)
                    for (int rm = 0; rm < 4; ++rm) {
                        hipStream_t side;
                        CK(hipStreamCreateWithPriority(&side, hipStreamNonBlocking, prio));
                        hipEvent_t e1, e2;
                        CK(hipEventCreateWithFlags(&e1, eflags[ef]));
                        CK(hipEventCreateWithFlags(&e2, eflags[ef]));
                        CK(hipMemset(err, 0, 64));
                        CK(hipDeviceSynchronize());
                        for (int i = 0; i < N; ++i, ++it) {
                            if (bz && i % 50 == 0) busy<<<256, 64, 0, third>>>(bp, 20000);
                            readers[rm]<<<G, 64, 0, side>>>(buf, 0, 0xffffffffu, err, sink);
                            CK(hipEventRecord(e1, side));
                            CK(hipStreamWaitEvent(0, e1, 0));
                            if (wm == 0)
                                writer<0><<<1, 64, 0, 0>>>(buf, it);
                            else
                                writer<1><<<1, 64, 0, 0>>>(buf, it);
                            CK(hipEventRecord(e2, 0));
                            CK(hipStreamWaitEvent(side, e2, 0));
                            readers[rm]<<<G, 64, 0, side>>>(buf, 0, it, err, sink);
                        }
                        CK(hipDeviceSynchronize());
                        unsigned h[2];
                        CK(hipMemcpy(h, err, 8, hipMemcpyDeviceToHost));
                        printf("side prio %2d  busy %d  event %-7s  writer %-5s  reader %-6s  stale %6u of %d x %d  max lag %u\n",
                               prio, bz, enames[ef], wm ? "sc1" : "plain", rnames[rm], h[0], N, G, h[1]);
                        fflush(stdout);
                        CK(hipEventDestroy(e1));
                        CK(hipEventDestroy(e2));
                        CK(hipStreamDestroy(side));
                    }
    return 0;
}
