// gs_shard.hip -- kernels of a SHARD engine: one rank's node range of a
// network sharded over G ranks.
//
// Per round t, rank g owns nodes [lo, lo+m).  Data movement between ranks is
// two exchanges of rows (RCCL all-to-allv over xGMI, or device copies when the
// shards share a GPU):
//   A (push rows):  every node x sends its round-t push batch as a 2-plane
//                   class code (2 x W words: 01 counter 1, 10 counter 2, 11
//                   counter 255) to owner(t_t(x)).  Rank g's receive buffer
//                   holds the rows of ALL sources targeting g in ascending
//                   source order (ranks own ascending ranges and each sends its
//                   rows for a destination in ascending order).
//   B (pull rows):  the owner of z returns, for each pusher x of z, the pull
//                   batch Gossip::receive built for x (src/gossip.rs:124-151):
//                   z's live set plus the entries z created from pushers ahead
//                   of x, as a 2-plane class code.  Same row order as A, reversed.
// The plan of a round depends only on the Philox peer stream, so it is built a
// round ahead on the side stream:
//   plan_count  : every source's target (all n; Philox), per 256-source block
//                 the number targeting g and, over the owned blocks, the number
//                 per destination rank
//   plan_scan   : block offsets, send/recv counts per rank
//   plan_emit   : E_id/E_key (the sources targeting g, ascending = receive row
//                 order) and SPOS (stable send row of every owned source)
//   edge_*      : counting sort of E by local target -> per-node in-lists of
//                 receive rows IN[z] = {first, k | zi<<16, e0, e1}, EP[]; zi =
//                 index of t(z) among z's pushers (mutual pair) or 0xFFFF.
#include <algorithm>
#include <cmath>

#include "gs_device.h"
#include "gs_kernels.h"

namespace gs {

constexpr uint32_t kPlanBlock = 256;

// ---------------------------------------------------------------- plan
// Destination rank of a target word; edges that are not delivered (faults)
// have none (G), so they get no row in either exchange.
GS_DEV uint32_t dest_rank(const ShardPlan &P, uint32_t t) {
    return (t & kTgDead) ? P.G : (t & kTgMask) / P.chunk;
}

__global__ __launch_bounds__(kPlanBlock) void plan_count(ShardPlan P, uint64_t seed, uint32_t epoch,
                                                         uint32_t round, Faults f, uint32_t *tg_all,
                                                         uint32_t *bc_me, uint32_t *bc_d) {
    const uint32_t blk = blockIdx.x;
    const u64 x = (u64)blk * kPlanBlock + threadIdx.x;
    const bool valid = x < P.n;
    uint32_t d = P.G;
    if (valid) {
        const uint32_t t = target_word(seed, epoch, round, (uint32_t)x, P.n, f);
        tg_all[x] = t;
        d = dest_rank(P, t);
    }
    const int me = __syncthreads_count(valid && d == P.g);
    if (threadIdx.x == 0) bc_me[blk] = (uint32_t)me;
    if (blk >= P.blk_lo && blk < P.blk_lo + P.nblk_own) {
        const bool own = valid && x >= P.lo && x < (u64)P.lo + P.m;
        for (uint32_t dd = 0; dd < P.G; ++dd) {
            const int c = __syncthreads_count(own && d == dd);
            if (threadIdx.x == 0) bc_d[(u64)(blk - P.blk_lo) * P.G + dd] = (uint32_t)c;
        }
    }
}

// In-place exclusive scan of v[i * stride] for i < count by one block of
// kPlanScanThreads: each thread scans a contiguous chunk serially around a
// single block-wide scan of the chunk sums; returns the total.  The chunk is
// read in unconditional batches of kBatch loads (a bounds test per load made
// the compiler issue them one at a time: 0.2 ms per 2^16-entry scan).
constexpr uint32_t kPlanScanThreads = 1024;
GS_DEV uint32_t chunked_scan(uint32_t *v, uint32_t count, uint32_t stride, uint32_t *lds) {
    constexpr uint32_t kBatch = 16;  // loads in flight per thread
    const uint32_t per = (count + kPlanScanThreads - 1) / kPlanScanThreads;
    const uint32_t lo = min(threadIdx.x * per, count), hi = min(lo + per, count);
    uint32_t sum = 0, i = lo;
    for (; i + kBatch <= hi; i += kBatch) {
        uint32_t t[kBatch];
#pragma unroll
        for (uint32_t q = 0; q < kBatch; ++q) t[q] = v[(u64)(i + q) * stride];
#pragma unroll
        for (uint32_t q = 0; q < kBatch; ++q) sum += t[q];
    }
    for (; i < hi; ++i) sum += v[(u64)i * stride];
    uint32_t tot;
    uint32_t run = block_exclusive_scan_t<kPlanScanThreads>(sum, lds, tot);
    for (i = lo; i + kBatch <= hi; i += kBatch) {
        uint32_t t[kBatch];
#pragma unroll
        for (uint32_t q = 0; q < kBatch; ++q) t[q] = v[(u64)(i + q) * stride];
#pragma unroll
        for (uint32_t q = 0; q < kBatch; ++q) {
            v[(u64)(i + q) * stride] = run;
            run += t[q];
        }
    }
    for (; i < hi; ++i) {
        const uint32_t t = v[(u64)i * stride];
        v[(u64)i * stride] = run;
        run += t;
    }
    return tot;
}

// Exclusive scans in place, one block per scan (G + 1 blocks, independent);
// cnt = {m_in, overflow, scnt[G], rcnt[G]}.
//   block 0     : bc_me (sources targeting this rank, per block of all n) ->
//                 m_in and the receive count from every source rank
//   block 1 + d : bc_d[.][d] over the owned blocks -> scnt[d]
// plan_scan_fix then adds the base of d (prefix of scnt) to bc_d[.][d].
__global__ __launch_bounds__(kPlanScanThreads) void plan_scan(ShardPlan P, uint32_t *bc_me,
                                                              uint32_t *bc_d, uint32_t *cnt) {
    __shared__ uint32_t lds[kPlanScanThreads / 64];
    if (blockIdx.x > 0) {
        const uint32_t dd = blockIdx.x - 1u;
        const uint32_t c2 = chunked_scan(bc_d + dd, P.nblk_own, P.G, lds);
        if (threadIdx.x == 0) cnt[2 + dd] = c2;  // scnt[dd]
        return;
    }
    const uint32_t carry = chunked_scan(bc_me, P.nblk, 1u, lds);
    __syncthreads();
    if (threadIdx.x == 0) {
        cnt[0] = carry;  // m_in: sources targeting this rank
        cnt[1] = carry > P.cap_in ? 1u : 0u;
    }
    // recv counts per source rank: difference of the prefix at rank boundaries
    for (uint32_t s = threadIdx.x; s < P.G; s += blockDim.x) {
        const u64 b0 = (u64)s * P.chunk / kPlanBlock, b1 = (u64)(s + 1) * P.chunk / kPlanBlock;
        const uint32_t p0 = b0 < P.nblk ? bc_me[b0] : carry;
        const uint32_t p1 = b1 < P.nblk ? bc_me[b1] : carry;
        cnt[2 + P.G + s] = p1 - p0;
    }
}

__global__ __launch_bounds__(256) void plan_scan_fix(ShardPlan P, uint32_t *bc_d, const uint32_t *cnt) {
    __shared__ uint32_t sdbase[64];
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (uint32_t dd = 0; dd < P.G; ++dd) {
            sdbase[dd] = run;
            run += cnt[2 + dd];
        }
    }
    __syncthreads();
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (u64)P.nblk_own * P.G) return;
    bc_d[i] += sdbase[(uint32_t)(i % P.G)];
}

__global__ __launch_bounds__(kPlanBlock) void plan_emit(ShardPlan P, const uint32_t *__restrict__ tg_all,
                                                        const uint32_t *__restrict__ off_me,
                                                        const uint32_t *__restrict__ off_d,
                                                        uint32_t *E_id, uint32_t *E_key, uint32_t *SPOS) {
    __shared__ uint32_t lds[kScanBlock / 64];
    __shared__ uint32_t wcnt[64][kPlanBlock / 64];
    const uint32_t blk = blockIdx.x;
    const u64 x = (u64)blk * kPlanBlock + threadIdx.x;
    const bool valid = x < P.n;
    const uint32_t t = valid ? tg_all[x] : 0u;
    const uint32_t d = valid ? dest_rank(P, t) : P.G;
    const bool me = d == P.g;
    uint32_t tot;
    const uint32_t rpos = off_me[blk] + block_exclusive_scan(me ? 1u : 0u, lds, tot);
    if (me && rpos < P.cap_in) {
        E_id[rpos] = (uint32_t)x;
        E_key[rpos] = (t & kTgMask) - P.lo;
    }
    if (blk >= P.blk_lo && blk < P.blk_lo + P.nblk_own) {
        const bool own = valid && x >= P.lo && x < (u64)P.lo + P.m;
        const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
        const u64 lt = (1ull << lane) - 1ull;
        uint32_t myrank = 0;
        for (uint32_t dd = 0; dd < P.G; ++dd) {
            const u64 mk = __ballot(own && d == dd);
            if (lane == 0) wcnt[dd][wid] = (uint32_t)__popcll(mk);
            if (own && d == dd) myrank = (uint32_t)__popcll(mk & lt);
        }
        __syncthreads();
        if (own && d < P.G) {  // a push row is sent (no row for an undelivered edge)
            uint32_t before = 0;
            for (uint32_t w = 0; w < wid; ++w) before += wcnt[d][w];
            SPOS[x - P.lo] = off_d[(u64)(blk - P.blk_lo) * P.G + d] + before + myrank;
        }
    }
}

// ------------------------------------------------ in-lists of receive rows
__global__ __launch_bounds__(256) void edge_bin_count(CsrPlan p, const uint32_t *__restrict__ E_key,
                                                      const uint32_t *__restrict__ cnt, uint32_t *M) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
    for (uint32_t i = threadIdx.x; i < p.nb; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    const uint32_t m_in = min(cnt[0], p.n);
    const u64 lo = (u64)blockIdx.x * p.chunk;
    const u64 hi = min((u64)m_in, lo + p.chunk);
    for (u64 e = lo + threadIdx.x; e < hi; e += blockDim.x) atomicAdd(&hist[E_key[e] >> p.logbin], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < p.nb; i += blockDim.x) M[(u64)blockIdx.x * p.nb + i] = hist[i];
}

__global__ __launch_bounds__(256) void edge_col_scan(uint32_t *M, CsrPlan p, uint32_t *tot) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.nb) return;
    uint32_t run = 0;
    for (uint32_t c = 0; c < p.ba; ++c) {
        const uint32_t v = M[(u64)c * p.nb + b];
        M[(u64)c * p.nb + b] = run;
        run += v;
    }
    tot[b] = run;
}

__global__ __launch_bounds__(kScanBlock) void edge_scan_small(const uint32_t *in, uint32_t *out, uint32_t m) {
    __shared__ uint32_t lds[kScanBlock / 64];
    uint32_t carry = 0;
    for (uint32_t base = 0; base < m; base += kScanBlock) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < m ? in[i] : 0u;
        uint32_t tot;
        const uint32_t ex = block_exclusive_scan(v, lds, tot);
        if (i < m) out[i] = carry + ex;
        carry += tot;
    }
}

__global__ __launch_bounds__(256) void edge_bin_scatter(CsrPlan p, const uint32_t *__restrict__ E_key,
                                                        const uint32_t *__restrict__ cnt,
                                                        const uint32_t *__restrict__ M,
                                                        const uint32_t *__restrict__ base, u64 *pairs) {
    extern __shared__ __attribute__((aligned(16))) uint32_t cur[];
    for (uint32_t i = threadIdx.x; i < p.nb; i += blockDim.x)
        cur[i] = base[i] + M[(u64)blockIdx.x * p.nb + i];
    __syncthreads();
    const uint32_t m_in = min(cnt[0], p.n);
    const u64 lo = (u64)blockIdx.x * p.chunk;
    const u64 hi = min((u64)m_in, lo + p.chunk);
    const uint32_t lm = p.bin - 1u;
    for (u64 e = lo + threadIdx.x; e < hi; e += blockDim.x) {
        const uint32_t t = E_key[e];
        const uint32_t pos = atomicAdd(&cur[t >> p.logbin], 1u);
        pairs[pos] = ((u64)(t & lm) << 32) | (uint32_t)e;
    }
}

// p.n here is the number of local nodes m (bins cover [0, m)).
__global__ __launch_bounds__(256) void edge_bin_sort(const u64 *__restrict__ pairs, CsrPlan p,
                                                     uint32_t nodes_total,
                                                     const uint32_t *__restrict__ base,
                                                     const uint32_t *__restrict__ tot, uint32_t *EP,
                                                     uint4 *IN, uint32_t *IN2,
                                                     const uint32_t *__restrict__ E_id,
                                                     const uint32_t *__restrict__ tg_all, uint32_t lo) {
    extern __shared__ __attribute__((aligned(16))) uint32_t h[];
    uint32_t *lds_scan = h + p.bin;
    const uint32_t b = blockIdx.x;
    const uint32_t start = base[b], cnt = tot[b];
    const uint32_t nb0 = b << p.logbin;
    const uint32_t nodes = min(p.bin, nodes_total - nb0);
    for (uint32_t i = threadIdx.x; i < p.bin; i += blockDim.x) h[i] = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) atomicAdd(&h[pairs[start + i] >> 32], 1u);
    __syncthreads();
    const uint32_t per = p.bin / blockDim.x;
    const uint32_t i0 = threadIdx.x * per;
    uint32_t sum = 0;
    for (uint32_t q = 0; q < per; ++q) sum += h[i0 + q];
    uint32_t total;
    uint32_t run = block_exclusive_scan(sum, lds_scan, total);
    for (uint32_t q = 0; q < per; ++q) {
        const uint32_t v = h[i0 + q];
        h[i0 + q] = run;
        run += v;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) {
        const u64 pr = pairs[start + i];
        const uint32_t pos = atomicAdd(&h[(uint32_t)(pr >> 32)], 1u);
        EP[start + pos] = (uint32_t)pr;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nodes; i += blockDim.x) {
        const uint32_t a = start + (i ? h[i - 1] : 0u), e = start + h[i];
        for (uint32_t q = a + 1; q < e; ++q) {  // receive rows ascending = pushers ascending
            const uint32_t v = EP[q];
            uint32_t r = q;
            while (r > a && EP[r - 1] > v) {
                EP[r] = EP[r - 1];
                --r;
            }
            EP[r] = v;
        }
        const uint32_t k = e - a;
        const uint32_t tz = tg_all[lo + nb0 + i] & kTgMask;  // t(z): did it push to z?
        uint32_t zi = 0xFFFFu;
        for (uint32_t q = a; q < e; ++q)
            if (E_id[EP[q]] == tz) zi = q - a;
        IN[nb0 + i] = make_uint4(a, k | (zi << 16), k > 0 ? EP[a] : 0u, k > 1 ? EP[a + 1] : 0u);
        IN2[nb0 + i] = k > 2 ? EP[a + 2] : 0u;
    }
}

ShardPlan shard_plan(uint32_t n, uint32_t G, uint32_t g) {
    ShardPlan P{};
    P.n = n;
    P.G = G;
    P.g = g;
    u64 chunk = ((u64)n + G - 1) / G;
    chunk = (chunk + kPlanBlock - 1) / kPlanBlock * kPlanBlock;  // whole plan blocks (and words)
    P.chunk = (uint32_t)chunk;
    const u64 lo = std::min<u64>((u64)g * chunk, n);
    const u64 hi = std::min<u64>(lo + chunk, n);
    P.lo = (uint32_t)lo;
    P.m = (uint32_t)(hi - lo);
    P.nblk = (uint32_t)(((u64)n + kPlanBlock - 1) / kPlanBlock);
    P.blk_lo = (uint32_t)(lo / kPlanBlock);
    P.nblk_own = (uint32_t)(((u64)P.m + kPlanBlock - 1) / kPlanBlock);
    // sources targeting this rank ~ Binomial(n, m/n): 16 standard deviations
    const double mean = (double)P.m;
    P.cap_in = (uint32_t)std::min<double>((double)n, mean + 16.0 * std::sqrt(mean + 1.0) + 1024.0);
    // counting sort of the received edges over the m local targets
    CsrPlan &c = P.edges;
    c.n = std::max<uint32_t>(P.cap_in, 1);  // edge capacity (actual count on device)
    uint32_t bin = 4096;
    while ((u64)bin * 16384u < P.m) bin <<= 1;
    c.bin = bin;
    c.logbin = 0;
    while ((1u << c.logbin) < bin) ++c.logbin;
    c.nb = std::max<uint32_t>(1, (uint32_t)(((u64)P.m + bin - 1) / bin));
    const uint32_t ba = (uint32_t)(((u64)c.n + 4095) / 4096);
    c.ba = ba < 256u ? (ba ? ba : 1u) : 256u;
    c.chunk = (uint32_t)(((u64)c.n + c.ba - 1) / c.ba);
    return P;
}

size_t shard_plan_words(const ShardPlan &P, ShardPlanLayout *L) {
    // all u32 words, 16-byte aligned sub-buffers
    size_t off = 0;
    auto take = [&](size_t words) {
        const size_t o = off;
        off += (words + 3) / 4 * 4;
        return o;
    };
    L->tg_all = take(P.n);
    L->bc_me = take(P.nblk);
    L->bc_d = take((size_t)P.nblk_own * P.G);
    L->cnt = take(2 + 2 * (size_t)P.G);
    L->E_id = take(P.cap_in);
    L->E_key = take(P.cap_in);
    L->SPOS = take(P.m);
    L->M = take((size_t)P.edges.ba * P.edges.nb);
    L->tot = take(P.edges.nb);
    L->base = take(P.edges.nb);
    L->EP = take(P.cap_in);
    L->IN = take(4 * (size_t)P.m);
    L->IN2 = take(P.m);
    L->pairs = take(2 * (size_t)P.cap_in);
    return off;
}

hipError_t launch_shard_plan(const ShardPlan &P, const ShardPlanLayout &L, uint32_t *w, uint64_t seed,
                             uint32_t epoch, uint32_t round, const Faults &f, hipStream_t s) {
    uint32_t *tg_all = w + L.tg_all, *bc_me = w + L.bc_me, *bc_d = w + L.bc_d, *cnt = w + L.cnt;
    uint32_t *E_id = w + L.E_id, *E_key = w + L.E_key, *SPOS = w + L.SPOS;
    uint32_t *M = w + L.M, *tot = w + L.tot, *base = w + L.base, *EP = w + L.EP;
    uint4 *IN = reinterpret_cast<uint4 *>(w + L.IN);
    uint32_t *IN2 = w + L.IN2;
    u64 *pairs = reinterpret_cast<u64 *>(w + L.pairs);
    hipLaunchKernelGGL(plan_count, dim3(P.nblk), dim3(kPlanBlock), 0, s, P, seed, epoch, round, f, tg_all,
                       bc_me, bc_d);
    hipLaunchKernelGGL(plan_scan, dim3(P.G + 1), dim3(kPlanScanThreads), 0, s, P, bc_me, bc_d, cnt);
    if (P.nblk_own) {
        const u64 nfix = (u64)P.nblk_own * P.G;
        hipLaunchKernelGGL(plan_scan_fix, dim3((uint32_t)((nfix + 255) / 256)), dim3(256), 0, s, P, bc_d, cnt);
    }
    hipLaunchKernelGGL(plan_emit, dim3(P.nblk), dim3(kPlanBlock), 0, s, P, tg_all, bc_me, bc_d, E_id,
                       E_key, SPOS);
    if (P.m == 0) return hipGetLastError();
    const CsrPlan &c = P.edges;
    const size_t lds_nb = (size_t)c.nb * sizeof(uint32_t);
    hipLaunchKernelGGL(edge_bin_count, dim3(c.ba), dim3(256), lds_nb, s, c, E_key, cnt, M);
    hipLaunchKernelGGL(edge_col_scan, dim3((c.nb + 255) / 256), dim3(256), 0, s, M, c, tot);
    hipLaunchKernelGGL(edge_scan_small, dim3(1), dim3(kScanBlock), 0, s, tot, base, c.nb);
    hipLaunchKernelGGL(edge_bin_scatter, dim3(c.ba), dim3(256), lds_nb, s, c, E_key, cnt, M, base, pairs);
    const size_t lds_sort = ((size_t)c.bin + 16) * sizeof(uint32_t);
    if (lds_sort > 65536) {
        hipError_t e = hipFuncSetAttribute((const void *)edge_bin_sort,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_sort);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(edge_bin_sort, dim3(c.nb), dim3(256), lds_sort, s, pairs, c, P.m, base, tot, EP,
                       IN, IN2, E_id, tg_all, P.lo);
    return hipGetLastError();
}

// ------------------------------------------------------------- pull rows
// Phase 1 at the receiver z (Gossip::receive's response half,
// src/gossip.rs:124-151): for each pusher x_i of z in ascending order, the
// pull batch is z's live set plus the entries z created from x_1..x_{i-1};
// written as a class code into sendB at x_i's receive row.
template <bool SMALL>
__global__ __launch_bounds__(256) void pull_kernel(PullArgs a) {
    const Geometry &g = a.g;
    const u64 seg = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (seg >= g.nseg) return;
    Lane<SMALL> L;
    L.init(g, seg);
    const uint32_t z = L.x;
    const u64 c = SMALL ? (a.S[L.plane_index(0)] >> L.sh) & L.m : a.S[L.plane_index(0)];
    const u64 q0 = SMALL ? (a.S[L.plane_index(1)] >> L.sh) & L.m : a.S[L.plane_index(1)];
    const u64 q1 = SMALL ? (a.S[L.plane_index(2)] >> L.sh) & L.m : a.S[L.plane_index(2)];
    const u64 zB = ~c & (q0 | q1);
    const u64 zB1 = zB & q0 & ~q1, zB2 = zB & q1 & ~q0;
    const u64 zC = c & ~(q0 & q1);
    u64 pnot = ~c & ~q0 & ~q1 & L.m, pB = 0, pC = 0;
    const uint4 in = a.IN[z];
    const uint32_t e2 = a.IN2[z];
    const uint32_t k = in.y & 0xFFFFu;
    for (uint32_t i = 0; i < k; ++i) {
        const uint32_t e = i == 0 ? in.z : (i == 1 ? in.w : (i == 2 ? e2 : a.EP[in.x + i]));
        const u64 pcl = zC | pC;
        a.sendB[L.row_index(e, 2, 0)] = zB1 | pB | pcl;  // code bit 0: counter 1 or 255
        a.sendB[L.row_index(e, 2, 1)] = zB2 | pcl;       // code bit 1: counter 2 or 255
        // a pusher's row matters to the later pull rows only while z lacks rumors
        if (i + 1 < k && pnot) sibling(L.load_push_row(a.recvA, e), pnot, pB, pC);
    }
}

hipError_t launch_pull(const PullArgs &a, hipStream_t s) {
    const u64 grid = (a.g.nseg + 255) / 256;
    if (grid == 0) return hipSuccess;
    if (a.g.small) hipLaunchKernelGGL(pull_kernel<true>, dim3((uint32_t)grid), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(pull_kernel<false>, dim3((uint32_t)grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace gs
