// gs_seq.hip -- the SEQ schedule: the reference harness's literal delivery
// order (src/gossiper.rs:217-234).  Pairs (x, t(x)) are processed by
// ascending x; t(x) answers x's push with its CURRENT live set, computed before
// it absorbs the push (src/gossip.rs:124-151), and x absorbs that pull batch
// at once.  So the pull x gets at "time" x is
//     W(x) = S(z) + { entries z created before time x },   z = t(x),
// where z's events before x are the pushes of z's pushers s < x and, when
// z < x, z's own pull W(z) at time z.  W(x) depends on W(z) only when
// z < x: following x -> t(x) -> ... while ids decrease gives chains whose
// length L has P(L >= l) ~ 1/(l+1)!, i.e. at most ~11 levels at 2^24 nodes.
//
//   seq_levels     : per node, got(x) (it receives a pull: push delivered and
//                    answered -- the second of a mutual pair is not answered,
//                    src/gossip.rs:125-126 -- and the pull not dropped),
//                    dep(x) = got(x) and z < x and got(z), and the chain depth
//   seq_pull_pass  : one launch per level: W(x) for that level's nodes, from
//                    z's class planes, the pushers of z ahead of x (SibRec,
//                    as in the 2P round) and W(z) inserted at time z.
// The round kernel (SEQ variant) then absorbs W(x) at x's own position among
// its pushers.
#include "gs_device.h"
#include "gs_kernels.h"

namespace gs {

namespace {

constexpr uint32_t kMaxSeqLevel = 62;

GS_DEV bool got0(uint32_t tw) { return !(tw & kTgNoPull); }

__global__ __launch_bounds__(256) void seq_levels(SeqArgs a) {
    __shared__ uint32_t bmax, hist[kSeqLists];
    if (threadIdx.x == 0) bmax = 0;
    if (threadIdx.x < kSeqLists) hist[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t y = blockIdx.x * blockDim.x + threadIdx.x;
    if (y < a.g.n) {
        // got(w) = got0(w) and not (t(t(w)) = w, t(w) < w, got0(t(w))).
        // Walk y -> z = t(y) -> t(z) ... while ids decrease, carrying each
        // loaded target word so every level costs one dependent random read;
        // y's in-list record is read up front, beside tg[y].
        const uint32_t ty = a.tg[y];
        const InRec iy = a.IN8[y];
        bool gy = false, dep = false;
        uint32_t lev = 0;
        if (got0(ty)) {
            uint32_t zc = ty & kTgMask, tz = a.tg[zc];  // z = t(y) and its target word
            gy = !((tz & kTgMask) == y && zc < y && got0(tz));
            for (uint32_t cur = y; gy && zc < cur && got0(tz);) {
                const uint32_t w = tz & kTgMask, tw = a.tg[w];
                if ((tw & kTgMask) == zc && w < zc && got0(tw)) break;  // zc gets no pull
                dep = true;
                if (++lev > kMaxSeqLevel) {
                    atomicOr(&a.flags[2], 4u);  // device limit (probability ~n/64!)
                    break;
                }
                cur = zc;
                zc = w;
                tz = tw;
            }
        }
        // W(y) is read by a pass only for a later w > y with t(w) = y that
        // gets a pull, and every such w is in y's in-list (ascending): without
        // a pusher above y, no pass builds W(y) and the round kernel makes it
        // inline from t(y)'s planes, t(y)'s pushers ahead of y and (dep) the
        // W(t(y)) its own pass wrote, t(y) having reader y.
        bool inl = false;
#ifndef GS_SEQ_NO_INLINE
        if (gy) {
            const uint32_t k = iy.k();
            const uint32_t top = k == 0 ? 0u
                                        : (k <= kInline ? pick_inline(iy.s, k - 1u)
                                                        : a.src[iy.first() + (k - 1u - kInline)]);
            inl = k == 0 || top < y;
        }
#endif
        a.sinfo[y] = (uint8_t)((gy ? kSeqGot : 0u) | (dep ? kSeqDep : 0u) |
                               (inl ? kSeqInline : min(lev, kMaxSeqLevel)));
        if (lev) atomicMax(&bmax, lev);
        if (gy && !inl) atomicAdd(&hist[min(lev, kSeqLists - 1u)], 1u);
    }
    __syncthreads();
    if (threadIdx.x < kSeqLists) a.bcnt[(u64)threadIdx.x * gridDim.x + blockIdx.x] = hist[threadIdx.x];
    if (threadIdx.x == 0 && bmax &&
        __hip_atomic_load(&a.flags[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < bmax)
        atomicMax(&a.flags[3], bmax);
}

// Per level list, exclusive prefix of its block counts (bcnt[list][block]):
// one 1024-thread block per list, each thread scanning a contiguous chunk
// (sum, block scan of the sums, rewrite), instead of a serial walk in steps
// of one block width (0.22 ms at 2^16 blocks).
constexpr uint32_t kSeqScanThreads = 1024;
__global__ __launch_bounds__(kSeqScanThreads) void seq_scan(SeqArgs a, uint32_t nblk) {
    __shared__ uint32_t lds[kSeqScanThreads / 64];
    uint32_t *c = a.bcnt + (u64)blockIdx.x * nblk;
    const uint32_t chunk = (nblk + kSeqScanThreads - 1u) / kSeqScanThreads;
    const uint32_t lo = min(threadIdx.x * chunk, nblk), hi = min(lo + chunk, nblk);
    constexpr uint32_t U = 16;  // loads in flight per thread
    uint32_t sum = 0, i = lo;
    for (; i + U <= hi; i += U) {
        uint32_t v[U];
#pragma unroll
        for (uint32_t j = 0; j < U; ++j) v[j] = c[i + j];
#pragma unroll
        for (uint32_t j = 0; j < U; ++j) sum += v[j];
    }
    for (; i < hi; ++i) sum += c[i];
    uint32_t tot;
    uint32_t run = block_exclusive_scan_t<kSeqScanThreads>(sum, lds, tot);
    for (i = lo; i + U <= hi; i += U) {
        uint32_t v[U];
#pragma unroll
        for (uint32_t j = 0; j < U; ++j) v[j] = c[i + j];
#pragma unroll
        for (uint32_t j = 0; j < U; ++j) {
            c[i + j] = run;
            run += v[j];
        }
    }
    for (; i < hi; ++i) {
        const uint32_t v = c[i];
        c[i] = run;
        run += v;
    }
    if (threadIdx.x == 0) a.ltot[blockIdx.x] = tot;
}

// Every node that gets a pull into its level's list (order inside a list
// is irrelevant: each W(x) is computed on its own).
__global__ __launch_bounds__(256) void seq_scatter(SeqArgs a) {
    __shared__ uint32_t cur[kSeqLists], lstart[kSeqLists];
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (uint32_t l = 0; l < kSeqLists; ++l) {
            lstart[l] = run;
            run += a.ltot[l];
        }
    }
    if (threadIdx.x < kSeqLists) cur[threadIdx.x] = a.bcnt[(u64)threadIdx.x * gridDim.x + blockIdx.x];
    __syncthreads();
    const uint32_t y = blockIdx.x * blockDim.x + threadIdx.x;
    if (y >= a.g.n) return;
    const uint32_t si = a.sinfo[y];
    if (!(si & kSeqGot) || (si & kSeqLevelMask) == kSeqInline) return;
    const uint32_t l = min(si & kSeqLevelMask, kSeqLists - 1u);
    a.lists[lstart[l] + atomicAdd(&cur[l], 1u)] = y;
}

template <bool SMALL>
__global__ __launch_bounds__(256) void seq_pull_pass(SeqArgs a, uint32_t level, uint32_t start,
                                                     uint32_t count) {
    const Geometry &g = a.g;
    const u64 lane = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t W = SMALL ? 1u : g.W;
    if (lane >= (u64)count * W) return;
    const uint32_t y0 = a.lists[start + (uint32_t)(lane / W)];
    Lane<SMALL> L;
    L.init(g, SMALL ? (u64)y0 : (u64)y0 * W + (uint32_t)(lane % W));
    const uint32_t y = L.x;
    const uint32_t si = a.sinfo[y];
    if ((si & kSeqLevelMask) != level) return;  // the last list holds every level >= 15
    const uint32_t z = a.tg[y] & kTgMask;
    const SibRec sb = a.SIB8[y];
    const uint32_t r = ((sb.tag >> 8) == (a.serial & kSerialMask)) ? (sb.tag & kSibRankMask) : 0u;
    const bool dep = (si & kSeqDep) != 0;
    const Cls qz = L.load_cls(a.S, z);
    Cls wz = {0, 0, 0};
    if (dep) {  // W(z), absorbed by z at time z: decoded like a push row
        const u64 wi = ((u64)z * 2u) * g.W + L.j;
        const u64 b0 = a.Wb[wi], b1 = a.Wb[wi + g.W];
        wz = Cls{b0 & b1, b0 & ~b1, b1 & ~b0};
    }
    const u64 zB = ~qz.c & (qz.a0 | qz.a1);
    const u64 zC = qz.c & ~(qz.a0 & qz.a1);
    u64 pnot = ~qz.c & ~qz.a0 & ~qz.a1 & L.m, pB = 0, pC = 0;
    bool wdone = !dep;
    InRec zin8 = {};
    if (r > kSibInline) zin8 = a.IN8[z];
    for (uint32_t i = 0; i < r && (pnot || !wdone); ++i) {
        const uint32_t s = i < kSibInline ? pick_sib(sb.e, i)
                                          : (i < kInline ? pick_inline(zin8.s, i)
                                                         : a.src[zin8.first() + (i - kInline)]);
        if (!wdone && s > z) {
            sibling(wz, pnot, pB, pC);
            wdone = true;
        }
        sibling(L.load_cls(a.S, s), pnot, pB, pC);
    }
    if (!wdone) sibling(wz, pnot, pB, pC);
    const u64 pcl = zC | pC;
    const u64 wi = ((u64)y * 2u) * g.W + L.j;
    a.Wb[wi] = ((zB & qz.a0 & ~qz.a1) | pB | pcl) & L.m;  // code bit 0: counter 1 or 255
    a.Wb[wi + g.W] = ((zB & qz.a1 & ~qz.a0) | pcl) & L.m; // code bit 1: counter 2 or 255
}

}  // namespace

hipError_t launch_seq_levels(const SeqArgs &a, hipStream_t s) {
    if (a.g.n == 0) return hipSuccess;
    const uint32_t nblk = seq_blocks(a.g.n);
    hipLaunchKernelGGL(seq_levels, dim3(nblk), dim3(256), 0, s, a);
    hipLaunchKernelGGL(seq_scan, dim3(kSeqLists), dim3(kSeqScanThreads), 0, s, a, nblk);
    hipLaunchKernelGGL(seq_scatter, dim3(nblk), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_seq_pull_pass(const SeqArgs &a, uint32_t level, uint32_t start, uint32_t count,
                                hipStream_t s) {
    const u64 lanes = (u64)count * (a.g.small ? 1u : a.g.W);
    if (lanes == 0) return hipSuccess;
    const uint32_t grid = (uint32_t)((lanes + 255) / 256);
    if (a.g.small) hipLaunchKernelGGL(seq_pull_pass<true>, dim3(grid), dim3(256), 0, s, a, level, start, count);
    else hipLaunchKernelGGL(seq_pull_pass<false>, dim3(grid), dim3(256), 0, s, a, level, start, count);
    return hipGetLastError();
}

}  // namespace gs
