// Cost of the injected Philox draws on gfx950: peer_of / target_word over
// n nodes (results folded into one word per block so nothing is dead code).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../safe_gossip_amd/csrc/gs_common.h"
using namespace gs;

template <int KIND>
__global__ __launch_bounds__(256) void draw(uint32_t n, uint64_t seed, uint32_t round, Faults f, uint32_t *out) {
    uint32_t acc = 0;
    for (uint32_t x = blockIdx.x * 256 + threadIdx.x; x < n; x += gridDim.x * 256) {
        if (KIND == 0) acc ^= peer_of(seed, 0, round, x, n);
        else if (KIND == 1) acc ^= target_word(seed, 0, round, x, n, f);
        else acc ^= offline_of(seed, 0, round, x, f.churn) ? x : 0u;
    }
    acc = __reduce_add_sync(~0ull, acc);
    if ((threadIdx.x & 63) == 0) atomicXor(&out[blockIdx.x], acc);
}

int main() {
    const uint32_t n = 100000000;
    uint32_t *out;
    hipMalloc(&out, 1 << 20);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    Faults f{42949672u, 42949672u, 42949672u};
    for (int grid : {2048, 8192, 32768}) {
        for (int kind = 0; kind < 3; ++kind) {
            float best = 1e9;
            for (int it = 0; it < 6; ++it) {
                hipEventRecord(a);
                if (kind == 0) hipLaunchKernelGGL(draw<0>, dim3(grid), dim3(256), 0, 0, n, 0x5AFE6055ull, it + 1, f, out);
                if (kind == 1) hipLaunchKernelGGL(draw<1>, dim3(grid), dim3(256), 0, 0, n, 0x5AFE6055ull, it + 1, f, out);
                if (kind == 2) hipLaunchKernelGGL(draw<2>, dim3(grid), dim3(256), 0, 0, n, 0x5AFE6055ull, it + 1, f, out);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                if (it) best = ms < best ? ms : best;
            }
            printf("grid %d kind %s: %.3f ms per %u draws\n", grid,
                   kind == 0 ? "peer_of" : (kind == 1 ? "target_word(faults)" : "offline_of"), best, n);
        }
    }
    return 0;
}
