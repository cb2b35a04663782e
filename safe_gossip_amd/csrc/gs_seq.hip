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
    __shared__ uint32_t bmax;
    if (threadIdx.x == 0) bmax = 0;
    __syncthreads();
    const uint32_t y = blockIdx.x * blockDim.x + threadIdx.x;
    if (y < a.g.n) {
        // got(w) = got0(w) and not (t(t(w)) = w, t(w) < w, got0(t(w)))
        auto got = [&](uint32_t w, uint32_t tw) -> bool {
            if (!got0(tw)) return false;
            const uint32_t v = tw & kTgMask;
            const uint32_t tv = a.tg[v];
            return !((tv & kTgMask) == w && v < w && got0(tv));
        };
        const uint32_t ty = a.tg[y];
        const bool gy = got(y, ty);
        uint32_t lev = 0;
        bool dep = false;
        if (gy) {
            uint32_t cur = y, tc = ty;
            for (;;) {
                const uint32_t zc = tc & kTgMask;
                if (zc >= cur) break;
                const uint32_t tz = a.tg[zc];
                if (!got(zc, tz)) break;
                if (lev == 0) dep = true;
                if (++lev > kMaxSeqLevel) {
                    atomicOr(&a.flags[2], 4u);  // device limit (probability ~n/64!)
                    break;
                }
                cur = zc;
                tc = tz;
            }
        }
        a.sinfo[y] = (uint8_t)((gy ? kSeqGot : 0u) | (dep ? kSeqDep : 0u) | min(lev, kMaxSeqLevel));
        if (lev) atomicMax(&bmax, lev);
    }
    __syncthreads();
    if (threadIdx.x == 0 && bmax &&
        __hip_atomic_load(&a.flags[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < bmax)
        atomicMax(&a.flags[3], bmax);
}

template <bool SMALL>
__global__ __launch_bounds__(256) void seq_pull_pass(SeqArgs a, uint32_t level) {
    const Geometry &g = a.g;
    const u64 seg = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (seg >= g.nseg) return;
    Lane<SMALL> L;
    L.init(g, seg);
    const uint32_t y = L.x;
    const uint32_t si = a.sinfo[y];
    if (!(si & kSeqGot) || (si & kSeqLevelMask) != level) return;
    const uint32_t z = a.tg[y] & kTgMask;
    const SibRec sb = a.SIB8[y];
    const uint32_t r = ((sb.tag >> 8) == (a.serial & kSerialMask)) ? (sb.tag & 0xFFu) : 0u;
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
    hipLaunchKernelGGL(seq_levels, dim3((a.g.n + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_seq_pull_pass(const SeqArgs &a, uint32_t level, hipStream_t s) {
    const u64 grid = (a.g.nseg + 255) / 256;
    if (grid == 0) return hipSuccess;
    if (a.g.small) hipLaunchKernelGGL(seq_pull_pass<true>, dim3((uint32_t)grid), dim3(256), 0, s, a, level);
    else hipLaunchKernelGGL(seq_pull_pass<false>, dim3((uint32_t)grid), dim3(256), 0, s, a, level);
    return hipGetLastError();
}

}  // namespace gs
