// Microbenchmark (experiment, not product): streaming and gather patterns of
// the 8-plane state on MI355X.  hipcc -O3 --offload-arch=gfx950 -o exp/layout_bench exp/layout_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
typedef unsigned long long u64;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// A: [x][p][W], lane (x,j): loads p*W+j  (current product layout, W=4)
__global__ __launch_bounds__(256) void strm_A(const u64* __restrict__ S, u64* __restrict__ T, uint32_t n, uint32_t W) {
    u64 seg = (u64)blockIdx.x * 256 + threadIdx.x;
    if (seg >= (u64)n * W) return;
    u64 x = seg / W, j = seg % W;
    u64 b = x * 8 * W + j;
    u64 v[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) v[p] = S[b + p * W];
    u64 acc = 0;
#pragma unroll
    for (int p = 0; p < 8; ++p) { acc ^= v[p]; }
#pragma unroll
    for (int p = 0; p < 8; ++p) T[b + p * W] = v[p] ^ (acc & 1);
}
// B: group-plane-major: [grp of 64 lanes][p][64] -> each plane instruction = 512 B contiguous
__global__ __launch_bounds__(256) void strm_B(const u64* __restrict__ S, u64* __restrict__ T, uint32_t n, uint32_t W) {
    u64 seg = (u64)blockIdx.x * 256 + threadIdx.x;
    if (seg >= (u64)n * W) return;
    u64 g = seg >> 6, l = seg & 63;
    u64 b = g * 8 * 64 + l;
    u64 v[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) v[p] = S[b + p * 64];
    u64 acc = 0;
#pragma unroll
    for (int p = 0; p < 8; ++p) { acc ^= v[p]; }
#pragma unroll
    for (int p = 0; p < 8; ++p) T[b + p * 64] = v[p] ^ (acc & 1);
}
// C: plain dwordx4 copy (ceiling)
__global__ __launch_bounds__(256) void strm_C(const uint4* __restrict__ S, uint4* __restrict__ T, u64 n16) {
    u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    for (; i < n16; i += (u64)gridDim.x * 256) T[i] = S[i];
}
// D: [x][p][W] but each lane loads its 8 planes as 4 x dwordx4 from a [x][W][p] layout
__global__ __launch_bounds__(256) void strm_D(const u64* __restrict__ S, u64* __restrict__ T, uint32_t n, uint32_t W) {
    u64 seg = (u64)blockIdx.x * 256 + threadIdx.x;
    if (seg >= (u64)n * W) return;
    const uint4* s4 = (const uint4*)(S + seg * 8);
    uint4* t4 = (uint4*)(T + seg * 8);
    uint4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = s4[q];
    uint32_t acc = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) acc ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
#pragma unroll
    for (int q = 0; q < 4; ++q) { v[q].x ^= acc & 1; t4[q] = v[q]; }
}
// Gathers: per lane (x,j), 2 random nodes; layout A (96 B contiguous per node when W=4)
__global__ __launch_bounds__(256) void gath_A(const u64* __restrict__ S, u64* __restrict__ T, const uint32_t* __restrict__ tg, uint32_t n, uint32_t W) {
    u64 seg = (u64)blockIdx.x * 256 + threadIdx.x;
    if (seg >= (u64)n * W) return;
    u64 x = seg / W, j = seg % W;
    u64 acc = 0;
    uint32_t s = tg[x];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        u64 b = (u64)s * 8 * W + j;
        acc ^= S[b] ^ S[b + W] ^ S[b + 2 * W];
        s = (s * 2654435761u + 12345u) % n;
    }
    T[seg] = acc;
}
// Gathers in layout B: node s's planes p at grp(s)*512 + p*64 + (s%16)*4 + j
__global__ __launch_bounds__(256) void gath_B(const u64* __restrict__ S, u64* __restrict__ T, const uint32_t* __restrict__ tg, uint32_t n, uint32_t W) {
    u64 seg = (u64)blockIdx.x * 256 + threadIdx.x;
    if (seg >= (u64)n * W) return;
    u64 x = seg / W, j = seg % W;
    u64 acc = 0;
    uint32_t s = tg[x];
    const uint32_t npg = 64 / W;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        u64 b = (u64)(s / npg) * 512 + (s % npg) * W + j;
        acc ^= S[b] ^ S[b + 64] ^ S[b + 128];
        s = (s * 2654435761u + 12345u) % n;
    }
    T[seg] = acc;
}

int main() {
    const uint32_t n = 1u << 24, W = 4;
    const u64 words = (u64)n * W * 8;
    u64 *S, *T; uint32_t* tg;
    CK(hipMalloc(&S, words * 8)); CK(hipMalloc(&T, words * 8)); CK(hipMalloc(&tg, n * 4));
    CK(hipMemset(S, 1, words * 8)); CK(hipMemset(T, 0, words * 8));
    std::vector<uint32_t> h(n); for (uint32_t i = 0; i < n; ++i) h[i] = (uint32_t)(((u64)i * 2654435761ull + 7) % n);
    CK(hipMemcpy(tg, h.data(), n * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const u64 lanes = (u64)n * W; const uint32_t grid = (uint32_t)((lanes + 255) / 256);
    auto time = [&](const char* name, double bytes, auto launch) {
        for (int w = 0; w < 2; ++w) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int it = 0; it < 10; ++it) launch();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 10;
        printf("%-28s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6);
    };
    double sb = 2.0 * words * 8;
    time("stream A [x][p][W]", sb, [&] { hipLaunchKernelGGL(strm_A, dim3(grid), dim3(256), 0, 0, S, T, n, W); });
    time("stream B grp-plane-major", sb, [&] { hipLaunchKernelGGL(strm_B, dim3(grid), dim3(256), 0, 0, S, T, n, W); });
    time("stream D [x][W][p] x4", sb, [&] { hipLaunchKernelGGL(strm_D, dim3(grid), dim3(256), 0, 0, S, T, n, W); });
    time("copy dwordx4 (2048 blk)", sb, [&] { hipLaunchKernelGGL(strm_C, dim3(2048), dim3(256), 0, 0, (const uint4*)S, (uint4*)T, words / 2); });
    time("copy dwordx4 (full grid)", sb, [&] { hipLaunchKernelGGL(strm_C, dim3((uint32_t)(words / 2 / 256)), dim3(256), 0, 0, (const uint4*)S, (uint4*)T, words / 2); });
    double gb = (double)n * (2 * 96 + 4) + lanes * 8;
    time("gather A (96B contiguous)", gb, [&] { hipLaunchKernelGGL(gath_A, dim3(grid), dim3(256), 0, 0, S, T, tg, n, W); });
    time("gather B (3x32B strided)", gb, [&] { hipLaunchKernelGGL(gath_B, dim3(grid), dim3(256), 0, 0, S, T, tg, n, W); });
    return 0;
}
