// Microbenchmark: Philox4x32-10 throughput on gfx950 with the two 32x32
// products formed as mul_hi + mul_lo pairs (gs_common.h) or as one 64-bit
// product each.  Both must agree bit for bit; prints draws/s of each.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

struct P4 { uint32_t a, b, c, d; };

template <int V>
__device__ __forceinline__ P4 ph(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint64_t seed) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint32_t hi0, lo0, hi1, lo1;
        if (V == 0) {
            hi0 = __umulhi(0xD2511F53u, c0); lo0 = 0xD2511F53u * c0;
            hi1 = __umulhi(0xCD9E8D57u, c2); lo1 = 0xCD9E8D57u * c2;
        } else {
            const uint64_t p0 = (uint64_t)c0 * 0xD2511F53u, p1 = (uint64_t)c2 * 0xCD9E8D57u;
            hi0 = (uint32_t)(p0 >> 32); lo0 = (uint32_t)p0;
            hi1 = (uint32_t)(p1 >> 32); lo1 = (uint32_t)p1;
        }
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return {c0, c1, c2, c3};
}

template <int V>
__global__ __launch_bounds__(256) void kern(uint32_t n, uint32_t per, uint64_t seed, uint32_t *out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint32_t acc = 0;
    for (uint32_t j = 0; j < per; ++j) {
        const P4 w = ph<V>(j, i, 3u, 7u, seed);
        acc ^= w.a + w.b * 3u + w.c * 5u + w.d * 7u;
    }
    if (i < n) out[i] = acc;
}

int main() {
    const uint32_t n = 1u << 22, per = 64;
    uint32_t *o0, *o1;
    hipMalloc(&o0, n * 4); hipMalloc(&o1, n * 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int v = 0; v < 2; ++v) {
        float best = 1e9f;
        for (int rep = 0; rep < 5; ++rep) {
            hipEventRecord(e0);
            if (v == 0) hipLaunchKernelGGL(kern<0>, dim3(n / 256), dim3(256), 0, 0, n, per, 0x1234ull, o0);
            else hipLaunchKernelGGL(kern<1>, dim3(n / 256), dim3(256), 0, 0, n, per, 0x1234ull, o1);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
        }
        printf("variant %d: %.3f ms, %.1f G draws/s\n", v, best, (double)n * per / best / 1e6);
    }
    uint32_t *h0 = (uint32_t *)malloc(n * 4), *h1 = (uint32_t *)malloc(n * 4);
    hipMemcpy(h0, o0, n * 4, hipMemcpyDeviceToHost); hipMemcpy(h1, o1, n * 4, hipMemcpyDeviceToHost);
    size_t bad = 0; for (uint32_t i = 0; i < n; ++i) bad += h0[i] != h1[i];
    printf("mismatches %zu\n", bad);
    return bad != 0;
}
