// gs_shard.hip -- kernels of a SHARD engine: one rank's node range of a
// network sharded over G ranks.
//
// Per round t, rank g owns nodes [lo, lo+m), cut into P pipeline parts of mP
// nodes.  Data moves between ranks in two exchanges of FIXED-SIZE blocks (RCCL
// all-to-all with equal splits over xGMI, or device copies when the shards
// share a GPU), so no row count ever has to reach the host and a round is
// enqueued without a host synchronisation.  Both buffers are part-major:
// part h's region holds one sub-block of capP row slots per rank, and each
// part moves in an all-to-all of its own, so the exchanges of one part overlap
// the round kernel of another (gs_shard_round_part):
//   A (push rows):  sub-block (d, h) of rank g's send buffer = g's part-h
//                   sources targeting rank d, ascending, as the 2-plane class
//                   code of their round-t push batch (01 counter 1, 10 counter
//                   2, 11 counter 255); the last part's sub-blocks carry after
//                   their rows the P*capP u32 source ids of round t+1's sources
//                   targeting d (id of (part h, index i) at h*capP + i;
//                   0xFFFFFFFF = empty slot).  Rank g then holds the rows of ALL
//                   sources targeting g; listed in (rank, part, index) order
//                   they are in ascending source order, and the ids of next
//                   round's let it build next round's in-lists while this round
//                   is still being delivered.
//   B (pull rows):  the owner of z returns, for each pusher x of z, the pull
//                   batch Gossip::receive built for x (src/gossip.rs:124-151):
//                   z's live set plus the entries z created from pushers ahead
//                   of x, as a 2-plane class code; sub-block layout of A
//                   without the id rows.
// Capacity: capP = mean + 16 sd + 64 rows per (source rank, destination rank,
// part) sub-block (binomial counts); an overflow raises the device-limit flag.
// Per-rank work is O(m): a plan computes the Philox targets of the OWNED
// sources only; a receiver recomputes the targets of the ids it receives.
//   plan_count / plan_scan / plan_emit / plan_idle : targets, send slots
//       (SPOSA in exchange A, SPOSB in exchange B) and the id blocks of round r
//   edge_bin / edge_sort : the received ids of round r by local target ->
//       per-node in-lists of receive slots IN[z] = {first, k | zi << 16, e0,
//       e1}, IN2[z] = e2, EP[first + i] = pusher i >= 3; zi = index of t(z)
//       among z's pushers (the mutual pair) or 0xFFFF.
#include <algorithm>
#include <cmath>

#include "gs_device.h"
#include "gs_kernels.h"

namespace gs {

constexpr uint32_t kPlanBlock = 256;
constexpr uint32_t kNoId = 0xFFFFFFFFu;

// ---------------------------------------------------------------- plan
// Destination rank of a target word; edges that are not delivered (faults)
// have none (G), so they get no slot in either exchange.
GS_DEV uint32_t dest_rank(const ShardPlan &P, uint32_t t) {
    return (t & kTgDead) ? P.G : (t & kTgMask) / P.chunk;
}

// Id slots of block d inside an exchange-A buffer: the idrows rows after the
// capP row slots of d's sub-block of the last part (P*capP ids; the id of
// next round's source (part h, index i) at h*capP + i).
GS_DEV uint32_t *id_slots(const ShardPlan &P, u64 *bufA, uint32_t d) {
    return reinterpret_cast<uint32_t *>(bufA) + (u64)shard_a_slot(P, d, P.P - 1u, P.capP) * P.rw;
}
GS_DEV const uint32_t *id_slots(const ShardPlan &P, const u64 *bufA, uint32_t d) {
    return reinterpret_cast<const uint32_t *>(bufA) + (u64)shard_a_slot(P, d, P.P - 1u, P.capP) * P.rw;
}

__global__ __launch_bounds__(kPlanBlock) void plan_count(ShardPlan P, uint64_t seed, uint32_t epoch,
                                                         uint32_t round, Faults f, uint32_t *tg,
                                                         uint32_t *bc_d) {
    __shared__ uint32_t hist[kMaxShards];
    for (uint32_t i = threadIdx.x; i < P.G; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    const uint32_t xl = blockIdx.x * kPlanBlock + threadIdx.x;
    if (xl < P.m) {
        const uint32_t t = target_word(seed, epoch, round, P.lo + xl, P.n, f);
        tg[xl] = t;
        const uint32_t d = dest_rank(P, t);
        if (d < P.G) atomicAdd(&hist[d], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < P.G; i += blockDim.x) bc_d[(u64)blockIdx.x * P.G + i] = hist[i];
}

// In-place exclusive scan of v[i * stride] for i < count by one block of
// kPlanScanThreads: each thread scans a contiguous chunk serially around a
// single block-wide scan of the chunk sums; returns the total.  The chunk is
// read in unconditional batches of kBatch loads (a bounds test per load made
// the compiler issue them one at a time).
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

// One block per (destination d, part h): bc_d[.][d] over the part's plan
// blocks -> offsets within sub-block (d, h) of the exchange, cnt[d * P + h] =
// rows part h sends to d.
__global__ __launch_bounds__(kPlanScanThreads) void plan_scan(ShardPlan P, uint32_t *bc_d, uint32_t *cnt,
                                                              uint32_t *flags) {
    __shared__ uint32_t lds[kPlanScanThreads / 64];
    const uint32_t d = blockIdx.x / P.P, h = blockIdx.x - d * P.P;
    const uint32_t b0 = min(h * P.bP, P.nblk_own), b1 = min(b0 + P.bP, P.nblk_own);
    const uint32_t c = chunked_scan(bc_d + (u64)b0 * P.G + d, b1 - b0, P.G, lds);
    if (threadIdx.x == 0) {
        cnt[blockIdx.x] = c;
        if (c > P.capP) atomicOr(&flags[2], 1u);  // more rows than the sub-block holds
    }
}

// Send slots of every owned source (stable: ascending x within each
// sub-block (d, h)) and the ids of block d.
__global__ __launch_bounds__(kPlanBlock) void plan_emit(ShardPlan P, const uint32_t *__restrict__ tg,
                                                        const uint32_t *__restrict__ off_d, uint32_t *SPOSA,
                                                        uint32_t *SPOSB, u64 *bufA) {
    __shared__ uint32_t wcnt[kMaxShards][kPlanBlock / 64];
    const uint32_t xl = blockIdx.x * kPlanBlock + threadIdx.x;
    const bool own = xl < P.m;
    const uint32_t d = own ? dest_rank(P, tg[xl]) : P.G;
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    const u64 lt = (1ull << lane) - 1ull;
    uint32_t myrank = 0;
    for (uint32_t dd = 0; dd < P.G; ++dd) {
        const u64 mk = __ballot(d == dd);
        if (lane == 0) wcnt[dd][wid] = (uint32_t)__popcll(mk);
        if (d == dd) myrank = (uint32_t)__popcll(mk & lt);
    }
    __syncthreads();
    if (!own) return;
    uint32_t sa = kNoId, sb = kNoId;
    if (d < P.G) {  // a push row is sent (no slot for an undelivered edge)
        uint32_t before = 0;
        for (uint32_t w = 0; w < wid; ++w) before += wcnt[d][w];
        const uint32_t i = off_d[(u64)blockIdx.x * P.G + d] + before + myrank;
        const uint32_t h = blockIdx.x / P.bP;  // the part of this plan block
        if (i < P.capP) {  // an overflow is flagged by plan_scan
            sa = shard_a_slot(P, d, h, i);
            sb = shard_b_slot(P, d, h, i);
            if (P.idrows) id_slots(P, bufA, d)[h * P.capP + i] = P.lo + xl;
        }
    }
    SPOSA[xl] = sa;
    SPOSB[xl] = sb;
}

// Empty slots of every sub-block (d, h) (past cnt[d * P + h]): class rows
// mark their id slot, code rows their row's target word (its receiver's
// build skips the slot).
__global__ __launch_bounds__(256) void plan_idle(ShardPlan P, const uint32_t *__restrict__ cnt, u64 *bufA) {
    const uint32_t d = blockIdx.y / P.P, h = blockIdx.y - d * P.P;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.capP || i < cnt[blockIdx.y]) return;
    // (code rows: the receiver of this rank's own block reads its count
    // instead, InListArgs::self_cnt)
    if (P.codes) reinterpret_cast<uint32_t *>(bufA)[(u64)shard_a_slot(P, d, h, i) * 2u + 1u] = kNoId;
    else id_slots(P, bufA, d)[h * P.capP + i] = kNoId;
}

// ------------------------------------------------ in-lists of receive slots
// The ids exchange A of round r-1 delivered (id slot j = (source rank s,
// part h, index i) at id_slots(s)[h*capP + i]: j = (s*P + h)*capP + i is
// also the slot key, ascending = ascending source id) become, per owned node
// z, its pushers of round r in ascending order as receive slots of exchange A
// of round r.  Two launches; no global atomic per edge (one per (chunk, bin)
// run), no global prefix sum:
//   edge_bin  : per chunk of kEdgeChunk id slots: the source's Philox target z
//               (recomputed) and its mutual bit (t(z) is the source: the
//               receiver's pull copy supersedes that push copy,
//               src/message_state.rs:79), an LDS counting sort by bin of
//               kEdgeBin targets, one reservation per non-empty bin in that
//               bin's fixed-capacity region, coalesced runs of (key | mutual,
//               z in the bin) entries
//   edge_sort : per bin: an LDS counting sort by target, per target an
//               insertion sort of its keys (in-degree is Poisson(1)), the
//               mutual pusher's index, IN/IN2 (lanes take consecutive
//               targets: coalesced) and the tails of in-degree > 3 in the
//               bin's own tail region; the fill count is left zeroed
// (round 4 and before: a global counting sort through 6 launches, 0.18 ms
// per 2^21-node shard against 0.074; a per-node fill by one returning global
// atomic per edge measured 0.18 too; DESIGN.md section 7 "Round 5").
constexpr uint32_t kEdgeBinLog = 11;
constexpr uint32_t kEdgeBin = 1u << kEdgeBinLog;           // targets per bin
constexpr uint32_t kEdgeBinCap = kEdgeBin + kEdgeBin / 4;  // region entries per bin (mean kEdgeBin, sd 45)
constexpr uint32_t kEdgeChunk = 4096;                      // id slots per edge_bin block
constexpr uint32_t kEdgeBinThreads = 1024;
constexpr uint32_t kEdgeSortThreads = 256;
constexpr uint32_t kEdgeTails = kEdgeBin / 8;              // tail slots per bin (mean ~48)
constexpr uint32_t kMutual = 1u << 31;                     // key bit: the pusher is the node's own target
static_assert(kEdgeChunk % kEdgeBinThreads == 0, "edge_bin: whole slots per thread");
static_assert(kEdgeChunk <= 0xFFFFu && kEdgeBinCap < 0xFFFFu, "edge_bin: 16-bit offsets and reservations");

__global__ __launch_bounds__(kEdgeBinThreads) void edge_bin(ShardPlan P, const u64 *__restrict__ recvA,
                                                            const uint32_t *__restrict__ tg, uint64_t seed,
                                                            uint32_t epoch, uint32_t round, Faults f, uint32_t nb,
                                                            uint32_t *fill, uint2 *region, uint32_t *flags) {
    constexpr uint32_t kPer = kEdgeChunk / kEdgeBinThreads;
    extern __shared__ __attribute__((aligned(16))) uint32_t sh[];
    uint32_t *skey = sh;                                           // [kEdgeChunk] keys by bin
    uint16_t *sz = reinterpret_cast<uint16_t *>(sh + kEdgeChunk);  // [kEdgeChunk] z in the bin
    uint16_t *sb = sz + kEdgeChunk;                                // [kEdgeChunk] bin of each staged entry
    uint32_t *cnt = sh + 2 * kEdgeChunk;                           // [nb] counts, then cursors
    // [nb] chunk-local start (low 16 bits, < kEdgeChunk) | reserved start in
    // the bin's region << 16 (<= kEdgeBinCap): 8 B of LDS per bin in all
    uint32_t *offres = cnt + nb;
    __shared__ uint32_t lds_scan[kEdgeBinThreads / 64];
    for (uint32_t i = threadIdx.x; i < nb; i += kEdgeBinThreads) cnt[i] = 0u;
    __syncthreads();
    const uint32_t per = P.P * P.capP, slots = P.G * per;
    uint32_t kv[kPer], zv[kPer];
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q) {
        const uint32_t j = blockIdx.x * kEdgeChunk + q * kEdgeBinThreads + threadIdx.x;
        zv[q] = kNoId;
        kv[q] = j;
        if (j >= slots) continue;
        const uint32_t src = j / per;
        const uint32_t id = id_slots(P, recvA, src)[j - src * per];
        if (id == kNoId) continue;
        const uint32_t tw = target_word(seed, epoch, round, id, P.n, f);
        const uint32_t t = tw & kTgMask;
        if (id >= P.n || (tw & kTgDead) || t < P.lo || t - P.lo >= P.m) {
            atomicOr(&flags[2], 1u);  // inconsistent exchange
            continue;
        }
        zv[q] = t - P.lo;
        if ((tg[zv[q]] & kTgMask) == id) kv[q] |= kMutual;
        atomicAdd(&cnt[zv[q] >> kEdgeBinLog], 1u);
    }
    __syncthreads();
    const uint32_t bper = (nb + kEdgeBinThreads - 1) / kEdgeBinThreads, b0 = threadIdx.x * bper;
    uint32_t sum = 0;
    for (uint32_t q = 0; q < bper; ++q)
        if (b0 + q < nb) sum += cnt[b0 + q];
    uint32_t total;
    uint32_t run = block_exclusive_scan_t<kEdgeBinThreads>(sum, lds_scan, total);
    for (uint32_t q = 0; q < bper && b0 + q < nb; ++q) {
        const uint32_t b = b0 + q, c = cnt[b];
        uint32_t r0 = 0;
        if (c) {
            r0 = atomicAdd(&fill[b], c);
            if (r0 + c > kEdgeBinCap) {
                atomicOr(&flags[2], 1u);
                r0 = kEdgeBinCap;  // drop this run; the round reports the limit
            }
        }
        offres[b] = run | (r0 << 16);
        cnt[b] = run;  // cursor
        run += c;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q) {
        if (zv[q] == kNoId) continue;
        const uint32_t b = zv[q] >> kEdgeBinLog;
        const uint32_t pos = atomicAdd(&cnt[b], 1u);
        skey[pos] = kv[q];
        sz[pos] = (uint16_t)(zv[q] & (kEdgeBin - 1u));
        sb[pos] = (uint16_t)b;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < total; i += kEdgeBinThreads) {
        const uint32_t b = sb[i], orb = offres[b], slot = (orb >> 16) + (i - (orb & 0xFFFFu));
        if (slot < kEdgeBinCap) region[(u64)b * kEdgeBinCap + slot] = make_uint2(skey[i], sz[i]);
    }
}

__global__ __launch_bounds__(kEdgeSortThreads) void edge_sort(ShardPlan P, uint32_t *fill,
                                                              const uint2 *__restrict__ region, uint32_t *EP,
                                                              uint4 *IN, uint32_t *IN2, uint32_t *flags) {
    constexpr uint32_t kPer = (kEdgeBinCap + kEdgeSortThreads - 1) / kEdgeSortThreads;
    constexpr uint32_t kTper = kEdgeBin / kEdgeSortThreads;  // targets per thread (scan)
    __shared__ uint32_t h[kEdgeBin];                           // per-target counts -> ends
    __shared__ uint32_t sorted[kEdgeBinCap];
    __shared__ uint32_t lds_scan[kEdgeSortThreads / 64];
    const uint32_t b = blockIdx.x;
    const uint32_t z0 = b << kEdgeBinLog;
    const uint32_t nodes = min(kEdgeBin, P.m - z0);
    const uint32_t cnt = min(fill[b], kEdgeBinCap);
    uint32_t ek[kPer], ez[kPer];
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q) {
        const uint32_t i = threadIdx.x + q * kEdgeSortThreads;
        const uint2 en = i < cnt ? region[(u64)b * kEdgeBinCap + i] : make_uint2(0u, kNoId);
        ek[q] = en.x;
        ez[q] = en.y;
    }
    for (uint32_t i = threadIdx.x; i < kEdgeBin; i += kEdgeSortThreads) h[i] = 0u;
    __syncthreads();
    if (threadIdx.x == 0) fill[b] = 0u;  // (read above by every thread; ready for the set's next build)
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q)
        if (ez[q] != kNoId) atomicAdd(&h[ez[q]], 1u);
    __syncthreads();
    const uint32_t i0 = threadIdx.x * kTper;
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t q = 0; q < kTper; ++q) sum += h[i0 + q];
    uint32_t total;
    uint32_t run = block_exclusive_scan_t<kEdgeSortThreads>(sum, lds_scan, total);
#pragma unroll
    for (uint32_t q = 0; q < kTper; ++q) {
        const uint32_t c = h[i0 + q];
        h[i0 + q] = run;  // start, then (after the scatter) end
        run += c;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q)
        if (ez[q] != kNoId) sorted[atomicAdd(&h[ez[q]], 1u)] = ek[q];
    __syncthreads();
    // the records: lanes take consecutive targets (coalesced IN / IN2 stores);
    // tails (pushers >= 3) go to the bin's own region, in any order
    uint32_t mine = 0;
    for (uint32_t lt = threadIdx.x; lt < nodes; lt += kEdgeSortThreads) {
        const uint32_t k = min(h[lt] - (lt ? h[lt - 1] : 0u), kMaxIn);
        mine += k > 3u ? k - 3u : 0u;
    }
    uint32_t ttot;
    const uint32_t toff = block_exclusive_scan_t<kEdgeSortThreads>(mine, lds_scan, ttot);
    const bool tails_ok = ttot <= kEdgeTails;
    if (!tails_ok && threadIdx.x == 0) atomicOr(&flags[2], 1u);
    uint32_t cur = b * kEdgeTails + toff;
    for (uint32_t lt = threadIdx.x; lt < nodes; lt += kEdgeSortThreads) {
        const uint32_t s = lt ? h[lt - 1] : 0u;
        uint32_t k = h[lt] - s;
        if (k > kMaxIn) {
            // in-degree above the limit (probability ~1e-34 per node, or a
            // corrupted exchange): a device limit, reported by gs_sync
            atomicOr(&flags[2], 1u);
            k = kMaxIn;
        }
        uint32_t *lst = sorted + s;
        for (uint32_t i = 1; i < k; ++i) {  // ascending key = ascending source id
            const uint32_t v = lst[i];
            uint32_t r = i;
            while (r > 0 && (lst[r - 1] & ~kMutual) > (v & ~kMutual)) {
                lst[r] = lst[r - 1];
                --r;
            }
            lst[r] = v;
        }
        uint32_t zi = 0xFFFFu;
        for (uint32_t i = 0; i < k; ++i)
            if (lst[i] & kMutual) zi = i;
        const uint32_t first = tails_ok ? cur : 0u;
        if (tails_ok)
            for (uint32_t i = 3; i < k; ++i) EP[cur + i - 3u] = shard_key_slot(P, lst[i] & ~kMutual);
        if (k > 3u) cur += k - 3u;
        // pushers i >= 3 at EP[in.x + i] (u32 arithmetic: in.x = first - 3)
        const uint32_t z = z0 + lt;
        IN[z] = make_uint4(first - 3u, k | (zi << 16), k > 0 ? shard_key_slot(P, lst[0] & ~kMutual) : 0u,
                           k > 1 ? shard_key_slot(P, lst[1] & ~kMutual) : 0u);
        IN2[z] = k > 2 ? shard_key_slot(P, lst[2] & ~kMutual) : 0u;
    }
}

__host__ __device__ inline uint32_t edge_bins(const ShardPlan &P) {
    return (uint32_t)(((u64)P.m + kEdgeBin - 1) / kEdgeBin);
}

// Dynamic LDS of edge_bin: the staged chunk (key, z, bin) and 8 B per bin.
static size_t edge_bin_lds(uint32_t nb) { return (2 * (size_t)kEdgeChunk + 2 * (size_t)nb) * sizeof(uint32_t); }

bool shard_edges_fit(const ShardPlan &P) {
    // class-row shards only (code rows build no in-lists ahead); the bin of a
    // staged entry is a u16 as well
    return P.codes || (edge_bin_lds(edge_bins(P)) <= kEdgeBinMaxLds && edge_bins(P) <= 0xFFFFu);
}

ShardPlan shard_plan(uint32_t n, uint32_t G, uint32_t g, uint32_t W, uint32_t parts, bool codes) {
    ShardPlan P{};
    P.codes = codes ? 1u : 0u;
    P.rw = codes ? 2u : 4u * W;   // A: (push code, target word) / class code
    P.rwb = codes ? 1u : 4u * W;  // B: pull code / class code
    P.n = n;
    P.G = G;
    P.g = g;
    P.W = W;
    u64 chunk = ((u64)n + G - 1) / G;
    chunk = (chunk + kPlanBlock - 1) / kPlanBlock * kPlanBlock;  // whole plan blocks (and words)
    P.chunk = (uint32_t)chunk;
    const u64 lo = std::min<u64>((u64)g * chunk, n);
    const u64 hi = std::min<u64>(lo + chunk, n);
    P.lo = (uint32_t)lo;
    P.m = (uint32_t)(hi - lo);
    P.nblk_own = (uint32_t)(((u64)P.m + kPlanBlock - 1) / kPlanBlock);
    P.P = std::max<uint32_t>(1, std::min(parts, kMaxParts));
    // (code rows: parts of whole 1024-node blocks, the packed DLV round
    // kernel's blocks at <= 4 nodes per lane)
    const u64 align = codes ? 1024u : kPlanBlock;
    const u64 mp = ((chunk + P.P - 1) / P.P + align - 1) / align * align;
    // parts are whole aligned blocks, so a small rank range holds fewer than
    // asked: the trailing ones would be empty (no overlap, an idle exchange
    // each); P is the number that holds nodes (the same on every rank)
    P.P = (uint32_t)std::max<u64>(1, (chunk + mp - 1) / mp);
    P.mP = (uint32_t)mp;
    P.bP = (uint32_t)(mp / kPlanBlock);
    // rows from one part of one rank to one rank: ~Binomial(mP, chunk/(n-1));
    // 16 standard deviations (the same on every rank: equal exchange splits)
    const double mean = (double)mp * (double)chunk / std::max(1.0, (double)n - 1.0);
    double capd = std::min<double>((double)mp, mean + 16.0 * std::sqrt(mean + 1.0) + 64.0);
    const u64 q = std::max<u64>(64, P.rw);  // P*capP u32 ids fill whole rows of rw u32 words
    P.capP = (uint32_t)(((u64)std::ceil(capd) + q - 1) / q * q);
    P.idrows = codes ? 0u : P.P * P.capP / P.rw;  // (code rows carry their targets: no ids)
    return P;
}

size_t shard_plan_words(const ShardPlan &P, ShardPlanLayout *L) {
    size_t off = 0;  // u32 words, 16-byte aligned sub-buffers
    auto take = [&](size_t words) {
        const size_t o = off;
        off += (words + 3) / 4 * 4;
        return o;
    };
    L->tg = take(P.m);
    L->SPOSA = take(P.m);
    L->SPOSB = take(P.m);
    L->bc_d = take((size_t)P.nblk_own * P.G);
    L->cnt = take((size_t)P.G * P.P);
    return off;
}

size_t shard_edge_words(const ShardPlan &P, ShardEdgeLayout *L) {
    size_t off = 0;
    auto take = [&](size_t words) {
        const size_t o = off;
        off += (words + 3) / 4 * 4;
        return o;
    };
    const size_t nb = edge_bins(P);
    L->fill = take(nb);  // zero between builds (edge_sort leaves it so; cleared at creation)
    L->region = take(2 * nb * kEdgeBinCap);
    L->EP = take(nb * kEdgeTails);
    L->IN = take(4 * (size_t)P.m);
    L->IN2 = take(P.m);
    return off;
}

hipError_t launch_shard_plan(const ShardPlan &P, const ShardPlanLayout &L, uint32_t *w, u64 *bufA,
                             uint64_t seed, uint32_t epoch, uint32_t round, const Faults &f,
                             uint32_t *flags, hipStream_t s) {
    uint32_t *tg = w + L.tg, *bc_d = w + L.bc_d, *cnt = w + L.cnt;
    if (P.nblk_own) {
        hipLaunchKernelGGL(plan_count, dim3(P.nblk_own), dim3(kPlanBlock), 0, s, P, seed, epoch, round, f, tg,
                           bc_d);
        hipLaunchKernelGGL(plan_scan, dim3(P.G * P.P), dim3(kPlanScanThreads), 0, s, P, bc_d, cnt, flags);
        hipLaunchKernelGGL(plan_emit, dim3(P.nblk_own), dim3(kPlanBlock), 0, s, P, tg, bc_d, w + L.SPOSA,
                           w + L.SPOSB, bufA);
    } else {
        hipError_t e = hipMemsetAsync(cnt, 0, (size_t)P.G * P.P * sizeof(uint32_t), s);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(plan_idle, dim3((P.capP + 255) / 256, P.G * P.P), dim3(256), 0, s, P, cnt, bufA);
    return hipGetLastError();
}

hipError_t launch_shard_edges(const ShardPlan &P, const ShardEdgeLayout &L, uint32_t *w, const u64 *recvA,
                              const uint32_t *tg, uint64_t seed, uint32_t epoch, uint32_t round,
                              const Faults &f, uint32_t *flags, hipStream_t s) {
    if (P.m == 0) return hipSuccess;  // no local targets: nothing is received
    const uint32_t nb = edge_bins(P), slots = P.G * P.P * P.capP;
    uint2 *region = reinterpret_cast<uint2 *>(w + L.region);
    if (!shard_edges_fit(P)) return hipErrorInvalidValue;  // (check_config refuses such a rank)
    const size_t lds = edge_bin_lds(nb);
    hipError_t e = hipFuncSetAttribute((const void *)edge_bin, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(edge_bin, dim3((slots + kEdgeChunk - 1) / kEdgeChunk), dim3(kEdgeBinThreads), lds, s, P, recvA,
                       tg, seed, epoch, round, f, nb, w + L.fill, region, flags);
    hipLaunchKernelGGL(edge_sort, dim3(nb), dim3(kEdgeSortThreads), 0, s, P, w + L.fill, region, w + L.EP,
                       reinterpret_cast<uint4 *>(w + L.IN), w + L.IN2, flags);
    return hipGetLastError();
}

// ------------------------------------------------------------- pull rows
// Phase 1 at the receiver z (Gossip::receive's response half,
// src/gossip.rs:124-151): for each pusher x_i of z in ascending order, the
// pull batch is z's live set plus the entries z created from x_1..x_{i-1};
// written as a class code into sendB at x_i's slot of exchange B.
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
        const SlotPos q = shard_a_decode(a.P, e);            // slot e of exchange A
        const uint32_t eb = shard_b_slot(a.P, q.s, q.h, q.i);  // the same slot of exchange B
        const u64 pcl = zC | pC;
        const u64 c0 = zB1 | pB | pcl, c1 = zB2 | pcl;
        a.sendB[L.row_index(eb, 2, 0)] = c0;  // code bit 0: counter 1 or 255
        a.sendB[L.row_index(eb, 2, 1)] = c1;  // code bit 1: counter 2 or 255
        // a pusher's row matters to the later pull rows only while z lacks
        // rumors (and only if it carries something for this word)
        if (i + 1 < k && pnot) sibling(L.load_push_row(a.recvA, e), pnot, pB, pC);
    }
}

// ------------------------------------------------ code rows (R_pad <= 16)
// Observers of a code-row shard: the pull code each node received, in node
// order (its exchange-B slot; none without a delivered push).
__global__ __launch_bounds__(256) void pull_unpack(const uint32_t *__restrict__ spos, const uint32_t *__restrict__ recvB,
                                                   uint32_t *pull, uint32_t m) {
    const uint32_t x = blockIdx.x * 256u + threadIdx.x;
    if (x >= m) return;
    const uint32_t sp = spos[x];
    pull[x] = sp != kNoId ? recvB[sp] : 0u;
}

hipError_t launch_shard_pull_unpack(const uint32_t *spos, const uint32_t *recvB, uint32_t *pull, uint32_t m,
                                    hipStream_t s) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(pull_unpack, dim3((m + 255u) / 256u), dim3(256), 0, s, spos, recvB, pull, m);
    return hipGetLastError();
}

hipError_t launch_pull(const PullArgs &a, hipStream_t s) {
    const u64 grid = (a.g.nseg + 255) / 256;
    if (grid == 0) return hipSuccess;
    if (a.P.codes) return hipErrorInvalidValue;  // code rows: the delivery-record build (gs_inlist.hip)
    if (a.g.small) hipLaunchKernelGGL(pull_kernel<true>, dim3((uint32_t)grid), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(pull_kernel<false>, dim3((uint32_t)grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace gs
