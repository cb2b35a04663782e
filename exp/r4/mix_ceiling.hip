// Ceiling of the config-4 round kernel's access mix (experiment, not
// product; VERDICT r3 "state the ceiling or move it").
//
// A synthetic kernel with the dense rounds' memory traffic and nothing else:
// 2^24 nodes of 8 planes x W = 4 words (256 B per node, the engine's layout),
// one lane per (node, word), 256-thread blocks, and per node
//   * its planes read with 16-B coalesced loads (256 B) and written back with
//     16-B nontemporal stores (256 B), as round_kernel stages them;
//   * 52 B of coalesced metadata read (InRec 16, SibRec 16, target 4,
//     Statistics deltas 16) and 16 B written (Statistics deltas);
//   * G random class rows gathered (planes 0-2 of a random node: 96 B, one
//     128-B line): G = 2 per node plus one more for every other node (the
//     dense rounds' ~2.5 rows per node: pushers, t(x), t(x)'s earlier
//     pushers; profiles/r3/pipe_ab).
// i.e. ~5.2 GB streamed reads, ~4.6 GB writes and 2.5 * 2^24 = 42 M random
// lines per launch, the mix round_kernel moves in rounds 14-18 (PMC: 4.9 GB
// streamed, 4.5 GB written, ~5.4 GB of random lines).  The lanes XOR what they
// read into what they write, so nothing is optimised away.
//
// hipcc -O3 --offload-arch=gfx950 -o exp/r4/mix_ceiling exp/r4/mix_ceiling.hip
// ./exp/r4/mix_ceiling [rows_x2 (default 5: 2.5 rows per node)] [reps]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef unsigned long long u64;
#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

constexpr uint32_t kW = 4, kPlanes = 8, kBlock = 256;
constexpr uint32_t kNodesBlk = kBlock / kW;                  // 64 nodes per block
constexpr uint32_t kWordsBlk = kNodesBlk * kPlanes * kW;     // 2048 words = 16 KiB
constexpr uint32_t kV4Blk = kWordsBlk / 2;                   // 1024 16-B chunks

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

__global__ void fill(u64 *p, u64 words) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (u64)gridDim.x * blockDim.x)
        p[i] = i * 0x9E3779B97F4A7C15ull;
}

// metadata record of a node: 16 B "InRec" + 16 B "SibRec" (random ids inside)
struct alignas(16) Rec {
    uint32_t a, b, c, d;
};

__global__ void make_meta(Rec *in, Rec *sib, uint32_t *tg, uint32_t n) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    auto rnd = [&](uint32_t salt) { return (uint32_t)(((u64)hash32((uint32_t)i * 2654435761u + salt) * n) >> 32); };
    in[i] = Rec{rnd(1), rnd(2), rnd(3), 0u};
    sib[i] = Rec{rnd(4), rnd(5), rnd(6), 0u};
    tg[i] = rnd(7);
}

template <uint32_t ROWS2>  // gathered rows per node, times two
__global__ __launch_bounds__(kBlock) void mix(const u64 *__restrict__ S, u64 *__restrict__ N,
                                              const Rec *__restrict__ in, const Rec *__restrict__ sib,
                                              const uint32_t *__restrict__ tg, uint4 *__restrict__ st,
                                              uint32_t n) {
    __shared__ __attribute__((aligned(16))) u64 stage[kWordsBlk];
    const u64 base = (u64)blockIdx.x * kWordsBlk;
    const uint4 *src4 = reinterpret_cast<const uint4 *>(S + base);
    uint4 v0 = src4[threadIdx.x], v1 = src4[threadIdx.x + 256], v2 = src4[threadIdx.x + 512],
          v3 = src4[threadIdx.x + 768];
    const uint32_t x = blockIdx.x * kNodesBlk + threadIdx.x / kW, j = threadIdx.x % kW;
    const Rec r = in[x];
    const Rec s = sib[x];
    const uint32_t t = tg[x];
    const uint4 sv = st[x];
    // the random rows: planes 0-2 of this lane's word (one 128-B line per row)
    u64 acc = 0;
    auto row = [&](uint32_t node) {
        const u64 b = (u64)node * kPlanes * kW + j;
        acc ^= S[b] ^ S[b + kW] ^ S[b + 2 * kW];
    };
    row(r.a);
    row(t);
    if (ROWS2 >= 5 && (x & 1u)) row(s.a);
    if (ROWS2 >= 6) row(r.b);
    if (ROWS2 >= 8) row(s.b);
    uint4 *dst4 = reinterpret_cast<uint4 *>(stage);
    dst4[threadIdx.x] = v0;
    dst4[threadIdx.x + 256] = v1;
    dst4[threadIdx.x + 512] = v2;
    dst4[threadIdx.x + 768] = v3;
    __syncthreads();
    // "transition": mix the gathered rows into the lane's planes
    const uint32_t nl = threadIdx.x / kW;
#pragma unroll
    for (uint32_t p = 0; p < kPlanes; ++p) stage[(nl * kPlanes + p) * kW + j] ^= acc + p;
    __syncthreads();
    uint4 *out4 = reinterpret_cast<uint4 *>(N + base);
#pragma unroll
    for (uint32_t it = 0; it < 4; ++it) {
        const uint32_t i = threadIdx.x + 256u * it;
        __builtin_nontemporal_store(dst4[i].x, &out4[i].x);
        __builtin_nontemporal_store(dst4[i].y, &out4[i].y);
        __builtin_nontemporal_store(dst4[i].z, &out4[i].z);
        __builtin_nontemporal_store(dst4[i].w, &out4[i].w);
    }
    if (j == 0) st[x] = make_uint4(sv.x + (uint32_t)acc, sv.y + r.c, sv.z + s.c, sv.w + 1u);
}

template <uint32_t ROWS2>
float run(const u64 *S, u64 *N, const Rec *in, const Rec *sib, const uint32_t *tg, uint4 *st, uint32_t n, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const uint32_t grid = n / kNodesBlk;
    hipLaunchKernelGGL(mix<ROWS2>, dim3(grid), dim3(kBlock), 0, 0, S, N, in, sib, tg, st, n);  // warm
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(mix<ROWS2>, dim3(grid), dim3(kBlock), 0, 0, (i & 1) ? N : S, (i & 1) ? const_cast<u64 *>(S) : N,
                           in, sib, tg, st, n);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char **argv) {
    const uint32_t rows2 = argc > 1 ? (uint32_t)atoi(argv[1]) : 5u;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const uint32_t n = 1u << 24;
    const u64 words = (u64)n * kPlanes * kW;
    u64 *S, *N;
    Rec *in, *sib;
    uint32_t *tg;
    uint4 *st;
    CK(hipMalloc(&S, words * 8));
    CK(hipMalloc(&N, words * 8));
    CK(hipMalloc(&in, (u64)n * sizeof(Rec)));
    CK(hipMalloc(&sib, (u64)n * sizeof(Rec)));
    CK(hipMalloc(&tg, (u64)n * 4));
    CK(hipMalloc(&st, (u64)n * 16));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, S, words);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, N, words);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<u64 *>(st), (u64)n * 2);
    hipLaunchKernelGGL(make_meta, dim3(n / 256), dim3(256), 0, 0, in, sib, tg, n);
    CK(hipDeviceSynchronize());
    float ms = 0;
    switch (rows2) {
    case 4: ms = run<4>(S, N, in, sib, tg, st, n, reps); break;
    case 5: ms = run<5>(S, N, in, sib, tg, st, n, reps); break;
    case 6: ms = run<6>(S, N, in, sib, tg, st, n, reps); break;
    case 8: ms = run<8>(S, N, in, sib, tg, st, n, reps); break;
    default: printf("rows_x2 in {4,5,6,8}\n"); return 2;
    }
    const double rows = rows2 / 2.0;
    const double stream_rd = (double)n * (256 + 52), wr = (double)n * (256 + 16), lines = rows * n;
    printf("{\"rows_per_node\": %.1f, \"ms\": %.4f, \"stream_read_GB\": %.3f, \"write_GB\": %.3f, "
           "\"random_lines_M\": %.1f, \"hbm_GB_model\": %.3f, \"TBps_model\": %.3f}\n",
           rows, ms, stream_rd / 1e9, wr / 1e9, lines / 1e6, (stream_rd + wr + lines * 128) / 1e9,
           (stream_rd + wr + lines * 128) / (ms * 1e-3) / 1e12);
    return 0;
}
