// Calibration microbenchmark (experiment, not product): what one random
// class-row gather of the round kernel costs in HBM traffic and time on
// MI355X, measured against known byte counts.
//   small : records of 8 planes x 8 B per 4 nodes (R_pad = 16, config 5
//           layout); one lane per node gathers planes 0-2 (24 B) of a random node
//   wide  : records of 8 planes x W=4 words (R_pad = 256, config 4 layout);
//           4 lanes per node gather planes 0-2 (96 B) of a random node
//   wide1 : as wide but only plane 0 (32 B of the row)
//   stream: coalesced 16-B/lane copy of the same state (known bytes)
// Every lane also streams its own 8 B of output, so a kernel moves
// n_lanes * 8 B of coalesced writes besides the gathers.
// hipcc -O3 --offload-arch=gfx950 -o exp/gather_calib exp/gather_calib.hip
// ./exp/gather_calib <small|wide|wide1|stream> [nodes]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef unsigned long long u64;
#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__);    \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

__global__ void make_targets(uint32_t *tg, uint32_t n, uint32_t salt) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) tg[i] = (uint32_t)(((u64)hash32((uint32_t)i * 2654435761u + salt) * n) >> 32);
}

__global__ void fill(u64 *p, u64 words) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (u64)gridDim.x * blockDim.x)
        p[i] = i * 0x9E3779B97F4A7C15ull;
}

__global__ __launch_bounds__(256) void gather_small(const u64 *__restrict__ S, const uint32_t *__restrict__ tg,
                                                    u64 *__restrict__ out, uint32_t n) {
    const u64 x = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= n) return;
    const uint32_t s = tg[x];
    const u64 b = (u64)(s >> 2) * 8;
    const uint32_t sh = (s & 3u) << 4;
    const u64 v = (S[b] >> sh) ^ (S[b + 1] >> sh) ^ (S[b + 2] >> sh);
    out[x] = v & 0xFFFF;
}

template <int NP>
__global__ __launch_bounds__(256) void gather_wide(const u64 *__restrict__ S, const uint32_t *__restrict__ tg,
                                                   u64 *__restrict__ out, uint32_t n) {
    const u64 seg = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (seg >= (u64)n * 4) return;
    const uint32_t x = (uint32_t)(seg >> 2), j = (uint32_t)(seg & 3);
    const uint32_t s = tg[x];
    const u64 b = (u64)s * 32 + j;
    u64 v = 0;
#pragma unroll
    for (int p = 0; p < NP; ++p) v ^= S[b + 4 * p];
    out[seg] = v;
}

__global__ __launch_bounds__(256) void stream_copy(const uint4 *__restrict__ S, uint4 *__restrict__ T, u64 n16) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (u64)gridDim.x * blockDim.x)
        T[i] = S[i];
}

int main(int argc, char **argv) {
    const char *mode = argc > 1 ? argv[1] : "small";
    const bool small = !strcmp(mode, "small");
    const uint32_t n = argc > 2 ? (uint32_t)atoll(argv[2]) : (small ? 100000000u : (1u << 24));
    const u64 words = small ? (u64)(n + 3) / 4 * 8 : (u64)n * 32;
    u64 *S, *T, *out;
    uint32_t *tg;
    CK(hipMalloc(&S, words * 8));
    CK(hipMalloc(&tg, (u64)n * 4));
    const u64 outw = small ? n : (u64)n * 4;
    CK(hipMalloc(&out, outw * 8));
    CK(hipMalloc(&T, !strcmp(mode, "stream") ? words * 8 : 8));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, S, words);
    hipLaunchKernelGGL(make_targets, dim3((n + 255) / 256), dim3(256), 0, 0, tg, n, 12345u);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 5;
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, 0));
        if (small) {
            hipLaunchKernelGGL(gather_small, dim3((n + 255) / 256), dim3(256), 0, 0, S, tg, out, n);
        } else if (!strcmp(mode, "wide")) {
            hipLaunchKernelGGL(gather_wide<3>, dim3((uint32_t)(((u64)n * 4 + 255) / 256)), dim3(256), 0, 0, S, tg,
                               out, n);
        } else if (!strcmp(mode, "wide1")) {
            hipLaunchKernelGGL(gather_wide<1>, dim3((uint32_t)(((u64)n * 4 + 255) / 256)), dim3(256), 0, 0, S, tg,
                               out, n);
        } else {
            hipLaunchKernelGGL(stream_copy, dim3(8192), dim3(256), 0, 0, (const uint4 *)S, (uint4 *)T, words / 2);
        }
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    double useful;  // bytes the kernel needs: gathered row bytes + target reads + output writes
    if (small) useful = (double)n * (24 + 4 + 8);
    else if (!strcmp(mode, "wide")) useful = (double)n * (96 + 4 * 4 + 32);
    else if (!strcmp(mode, "wide1")) useful = (double)n * (32 + 4 * 4 + 32);
    else useful = (double)words * 16;
    printf("{\"mode\": \"%s\", \"nodes\": %u, \"best_ms\": %.4f, \"gathers_per_ns\": %.3f, "
           "\"useful_GBps\": %.1f}\n",
           mode, n, best, !strcmp(mode, "stream") ? 0.0 : n / (best * 1e6), useful / (best * 1e-3) / 1e9);
    return 0;
}
