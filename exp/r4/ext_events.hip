// Cost of timing one kernel of a launch chain (experiment, not product):
// hipEventRecord before and after it versus hipExtLaunchKernel's start/stop
// events, on a chain of three ~15-us kernels like a small network's round.
// hipcc -O3 --offload-arch=gfx950 -o exp/r4/ext_events exp/r4/ext_events.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

__global__ void work(float *p, int n, int iters) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float v = p[i];
    for (int k = 0; k < iters; ++k) v = v * 1.000001f + 0.5f;
    p[i] = v;
}

int main() {
    const int n = 1 << 20, iters = 200, reps = 200;
    float *p;
    CK(hipMalloc(&p, n * sizeof(float)));
    CK(hipMemset(p, 0, n * sizeof(float)));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b, t0, t1;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventCreateWithFlags(&t0, hipEventDisableSystemFence));
    CK(hipEventCreateWithFlags(&t1, hipEventDisableSystemFence));
    const dim3 g(n / 256), bl(256);
    for (int mode = 0; mode < 3; ++mode) {
        for (int warm = 0; warm < 2; ++warm) {
            CK(hipEventRecord(a, s));
            float kern = 0;
            for (int r = 0; r < reps; ++r) {
                hipLaunchKernelGGL(work, g, bl, 0, s, p, n, iters);
                if (mode == 1) CK(hipEventRecord(t0, s));
                if (mode == 2) hipExtLaunchKernelGGL(work, g, bl, 0, s, t0, t1, 0, p, n, iters);
                else hipLaunchKernelGGL(work, g, bl, 0, s, p, n, iters);
                if (mode == 1) CK(hipEventRecord(t1, s));
                hipLaunchKernelGGL(work, g, bl, 0, s, p, n, iters);
                if (mode && r == reps - 1) {
                    CK(hipEventSynchronize(t1));
                    CK(hipEventElapsedTime(&kern, t0, t1));
                }
            }
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            if (warm)
                printf("{\"mode\": \"%s\", \"us_per_chain\": %.2f, \"timed_kernel_us\": %.2f}\n",
                       mode == 0 ? "untimed" : (mode == 1 ? "event_records" : "ext_launch_events"), 1e3 * ms / reps,
                       1e3 * kern);
        }
    }
    return 0;
}
