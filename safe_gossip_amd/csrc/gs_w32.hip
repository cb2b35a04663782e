// gs_w32.hip -- the 2P round kernel of the class-plane gather path with a
// 32-bit lane word (R_pad 32..256, live-filtered gathers, transition modes).
//
// round_kernel (gs_kernels.hip) gives a lane one 64-rumor word of a node and
// keeps every bit-sliced value in a 64-bit register pair: 114 VGPRs, four
// waves per SIMD at config 4 (2^24 x 256).  Its waves spend about half their
// life waiting on memory ("Round 3"), and four waves per
// SIMD cannot keep enough bytes in flight.  Here a lane owns a 32-rumor half
// word: every bit-sliced value is one VGPR, so the same algebra needs about
// half the registers and a SIMD holds more waves (more plane loads and row
// gathers in flight per CU).  The bit-sliced work per node is unchanged (a
// 64-bit logic op is two 32-bit ones); what a lane does per node -- its
// metadata, the gather addresses, the in-list walk, the reductions over the
// node's lanes -- is done by twice as many lanes.
//
// The algebra is round_kernel's 2P filtered path term by term (Gossip::receive
// src/gossip.rs:118-163 for every push batch in ascending pusher order and
// the pull batch, Gossip::new_message src/gossip.rs:71-75, then
// MessageState::next_round src/message_state.rs:86-171 and the Statistics of
// src/gossip.rs:80,103-111,139-163), over the same records (gs_common.h
// InRec / SibRec, the skip flags of the live-filtered gathers), the same
// plane layout ([node][plane][W] u64 words: u32 word 2j / 2j+1 = the low /
// high half of u64 word j) and the same outputs (planes, node maps, any-live
// flag, Statistics deltas, churn votes).  Rounds with external RPCs, the
// observation launches, R_pad > 256 (map bytes shared by two waves) or < 32,
// the unfiltered gathers and the other schedules keep round_kernel.
#include "gs_device.h"
#include "gs_kernels.h"
#include "gs_recv.h"

namespace gs {

#ifndef GS_W32_THREADS
#define GS_W32_THREADS 128u  // lanes per block: 2^24 x 32 1.051 -> 1.037 ms/step against 256 (64: 1.051)
#endif
#ifndef GS_W32_ZSKIP
#define GS_W32_ZSKIP 1  // no plane stores for a block whose new planes are all A
#endif
constexpr uint32_t kW32Threads = GS_W32_THREADS;
#ifndef GS_W32_MINW
#define GS_W32_MINW 1
#endif

using u32 = uint32_t;
using Cls32 = ClsT<u32>;

// u32 word j of plane p of node x: records of 8 planes x W32 words (lw >= 1:
// R_pad 64..256), or, at R_pad 32 (lw = 0), the low / high half of the plane
// words of a unit of two nodes ([unit][plane] u64).
GS_DEV u64 rec32(uint32_t x, uint32_t p, uint32_t j, uint32_t lw) {
    return lw ? ((u64)x << (lw + 3u)) + (p << lw) + j : ((u64)(x >> 1) << 4) + (p << 1) + (x & 1u);
}
// Class planes (isC, a0, a1) of node s for u32 word j.
GS_DEV Cls32 load_cls32(const u32 *__restrict__ S, uint32_t s, uint32_t j, uint32_t lw) {
    if (GS_CLS_VEC && lw <= 1u) {
        // planes 0-2 of the 64-B unit holding s lie in its first 24 bytes
        // (plane p, word sel at 2p + sel): a 16-byte and an 8-byte load
        // instead of three 4-byte ones
        const u64 b0 = lw ? ((u64)s << 4) : ((u64)(s >> 1) << 4);
        const uint32_t sel = lw ? j : (s & 1u);
        const uint4 v = *reinterpret_cast<const uint4 *>(S + b0);
        const uint2 w = *reinterpret_cast<const uint2 *>(S + b0 + 4);
        return Cls32{sel ? v.y : v.x, sel ? v.w : v.z, sel ? w.y : w.x};
    }
    const u64 b = rec32(s, 0, j, lw);
    const uint32_t ps = lw ? (1u << lw) : 2u;  // plane stride
    return Cls32{S[b], S[b + ps], S[b + 2u * ps]};
}

GS_DEV void sibling32(const Cls32 &q, u32 &pnot, u32 &pB, u32 &pC) {
    const u32 vC = q.c & ~(q.a0 & q.a1);
    const u32 sl = (~q.c & (q.a0 | q.a1)) | vC;
    const u32 nc = pnot & sl;
    pB |= nc & ~vC;
    pC |= nc & vC;
    pnot &= ~sl;
}

template <int MODE>
__global__ __launch_bounds__(kW32Threads, GS_W32_MINW) void round_kernel_w32(RoundArgs a) {
    constexpr bool DELIVER = MODE == 1;
    const Geometry &g = a.g;
    if (a.zero_buf || a.zero_rows) zero_for_build(a.zero_buf, a.zero_words, a.zero_rows);
    if (a.zero_buf2) zero_for_build(a.zero_buf2, a.zero_words2, nullptr);
    const uint32_t lw = g.logr - 5u;  // log2 of the u32 words (lanes) per node plane: 0..3
    const uint32_t W32 = 1u << lw;
    const uint32_t bid = blockIdx.x;
    const u64 seg = (u64)bid * kW32Threads + threadIdx.x;
    const u64 nseg = (u64)g.n << lw;
    const bool valid = seg < nseg;
    const uint32_t x = valid ? (uint32_t)(seg >> lw) : 0u;
    const uint32_t j = (uint32_t)seg & (W32 - 1u);
    const u32 *__restrict__ S = reinterpret_cast<const u32 *>(a.Scur);
    __shared__ uint32_t blk_any;  // some node pushes a live rumor in round t+1
    __shared__ uint32_t blk_nz;   // some node is not all-A in round t+1 (GS_W32_ZSKIP)
    if (threadIdx.x == 0) blk_any = 0;
    if (threadIdx.x == 0) blk_nz = 0;

    // ---- own round-t planes: the block's records (kW32Threads / W32 nodes,
    // 8 KiB) with 16-byte coalesced loads, transposed through LDS below
    constexpr uint32_t kBlkWords = kW32Threads * kPlanes;  // u32 words of the block's records
    __shared__ __attribute__((aligned(16))) u32 stage[kBlkWords];
    const u64 blk_base = (u64)bid * kBlkWords;  // u32 word of the block's first record
    const u64 words = g.units * 16u * g.W;      // u32 words of all records
    const uint32_t blk_v4 = (uint32_t)(min((u64)kBlkWords, words - blk_base) >> 2);
    const uint4 *src4 = reinterpret_cast<const uint4 *>(S + blk_base);
    static_assert(kBlkWords / 4u == 2u * kW32Threads, "two uint4 per thread");
    const uint4 st0 = src4[min(threadIdx.x, blk_v4 - 1u)];
    const uint4 st1 = src4[min(threadIdx.x + kW32Threads, blk_v4 - 1u)];

    // ---- coalesced per-node metadata (level 1)
    const bool leader = valid && j == 0;
    uint4 stv = {0u, 0u, 0u, 0u};
    if (leader) stv = reinterpret_cast<const uint4 *>(a.st32)[x];
    uint32_t eadd = 0;  // rumor slice: an earlier round's network empty counts
    if (a.eadd && leader) eadd = reinterpret_cast<const uint16_t *>(a.eadd)[x];
    InRec in8 = {};
    SibRec sb8 = {};
    uint32_t z = x, k = 0, r = 0, tgw = 0;
    uint32_t qskip = 0, eskip = 0;
    bool zneed = false;
    u64 zlw = 0;
    if (DELIVER) {
        in8 = a.IN8[x];  // x = 0 on invalid lanes: a harmless valid address
        tgw = a.tg[x];
        z = tgw & kTgMask;
        k = valid ? in8.k() : 0u;
        sb8 = a.SIB8[x];
        zlw = a.zlm[x >> 6];
        const bool sib_ok = valid && (sb8.tag >> 8) == (a.serial & kSerialMask);
        r = sib_ok ? (sb8.tag & kSibRankMask) : 0u;
        qskip = in8.kf >> kInSkipShift;
        in8.kf &= kInFlagMask;
        eskip = ((sb8.tag >> kSibSkipShift) & 3u) | ((sb8.e[2] >> 31) << 2);
        sb8.e[2] &= kIdMask;
        zneed = sib_ok && (sb8.tag & kSibZNeed) != 0;
    }

    // ---- the random gathers (level 2), issued together: the first kBatchK
    // pushers, t(x), the first kBatchE pushers of t(x) ahead of x; rows the
    // skip flags leave out are not loaded (they would change nothing)
    Cls32 q[kBatchK], e[kBatchE], qz = {0, 0, 0};
    bool gq[kBatchK], ge[kBatchE];
#pragma unroll
    for (uint32_t i = 0; i < kBatchK; ++i) {
        q[i] = {0, 0, 0};
        gq[i] = DELIVER && i < k && !((qskip >> i) & 1u);
        if (gq[i]) q[i] = load_cls32(S, in8.s[i], j, lw);
    }
    const bool gz = DELIVER && valid && !(tgw & kTgNoPull) && (((zlw >> (x & 63u)) & 1ull) != 0 || zneed);
    if (gz) qz = load_cls32(S, z, j, lw);
#pragma unroll
    for (uint32_t i = 0; i < kBatchE; ++i) {
        e[i] = {0, 0, 0};
        ge[i] = DELIVER && i < r && !((eskip >> i) & 1u);
        if (ge[i]) e[i] = load_cls32(S, sb8.e[i], j, lw);
    }
    {
        uint4 *dst4 = reinterpret_cast<uint4 *>(stage);
        dst4[threadIdx.x] = st0;
        dst4[threadIdx.x + kW32Threads] = st1;
    }
    __syncthreads();
    const uint32_t xl = threadIdx.x >> lw;  // node within the block (an even count of them)
    const uint32_t pbase = (uint32_t)rec32(xl, 0, j, lw), pstr = lw ? (1u << lw) : 2u;
    u32 P[kPlanes];
#pragma unroll
    for (int p = 0; p < kPlanes; ++p) P[p] = valid ? stage[pbase + (uint32_t)p * pstr] : 0u;

    const u32 isC = P[0], a0 = P[1], a1 = P[2];
    const u32 A = ~isC & ~a0 & ~a1;
    const u32 B = ~isC & (a0 | a1);
    const u32 C = isC & ~(a0 & a1);
    const u32 liveX = B | C;

    // ---- phases 1 and 2 of round t at x (Gossip::receive)
    const bool off_t = DELIVER && (tgw & kTgOff);
    const bool pulled = !(tgw & kTgNoPull);
    Recv<false, u32> rv;
    rv.init(A, B, B & a0 & ~a1);
    uint32_t psize = 0;
    if (DELIVER && valid && k > 30u) atomicOr(&a.flags[2], 1u);
    if (DELIVER && valid) {
        bool zin = false;
#pragma unroll
        for (uint32_t i = 0; i < kBatchK; ++i) {
            if (i < k) {
                zin |= in8.s[i] == z;
                if (gq[i]) rv.push(q[i], i, k, !(pulled && in8.s[i] == z));
            }
        }
        for (uint32_t i = kBatchK; i < k; ++i) {  // in-degree > kBatchK (1.9% of nodes)
            const uint32_t s = i < kInline ? pick_inline(in8.s, i) : a.src[in8.first() + (i - kInline)];
            zin |= s == z;
            rv.push(load_cls32(S, s, j, lw), i, k, !(pulled && s == z));
        }
        // Pull batch from z: z's live set plus what z created from pushers
        // ahead of x.
        const u32 zB = ~qz.c & (qz.a0 | qz.a1);
        const u32 zC = qz.c & ~(qz.a0 & qz.a1);
        u32 pnot = ~qz.c & ~qz.a0 & ~qz.a1, pB = 0, pC = 0;
#pragma unroll
        for (uint32_t i = 0; i < kBatchE; ++i)
            if (i < r && ge[i]) sibling32(e[i], pnot, pB, pC);
        // (no live sibling ahead of x, or t(x) complete: nothing deeper either)
        if (r > kBatchE && pnot && pulled && zneed) {  // rank > kBatchE (rare)
            for (uint32_t i = kBatchE; i < min(r, kSibInline); ++i)
                if (!((eskip >> i) & 1u)) sibling32(load_cls32(S, pick_sib(sb8.e, i), j, lw), pnot, pB, pC);
            if (r > kSibInline && pnot) {  // rank > 3: 0.2% of nodes
                InRec zin8 = a.IN8[z];
                zin8.kf &= kInFlagMask;
                for (uint32_t i = kSibInline; i < r && pnot; ++i) {
                    const uint32_t s = i < kInline ? pick_inline(zin8.s, i) : a.src[zin8.first() + (i - kInline)];
                    sibling32(load_cls32(S, s, j, lw), pnot, pB, pC);
                }
            }
        }
        u32 pv2 = zB & qz.a1 & ~qz.a0;
        u32 pvB = zB | pB;  // counter 1 (created entries: 1) or 2
        u32 pCl = zC | pC;
        if (!pulled) pv2 = pvB = pCl = 0;
        const u32 pl = pvB | pCl;
        {
            const u32 newc = rv.notyet & pl;
            rv.record(rv.recB & pl, pvB, pv2, pCl);
            rv.create(newc, pCl);
        }
        rv.recv += popcT(pl);
        psize = k + ((pulled && !zin) ? 1u : 0u);  // |peers_in_this_round|
    }

    // ---- node-level statistics of the deliveries
    uint32_t lc = popcT(liveX);
    uint32_t part_cw = rv.part_cw, recv = rv.recv, first_create = rv.first_create;
    if (DELIVER) {
        lc = group_sum(lc, W32);
        part_cw = group_sum(part_cw, W32);
        recv = group_sum(recv, W32);
        first_create = group_min(first_create, W32);
    }
    uint32_t d_full_sent = 0, d_empty_pull = 0;
    if (DELIVER) {
        d_full_sent = k * lc + part_cw;  // pull rows sent by x
        if (k > 0 && lc == 0) d_empty_pull = (first_create == kNone) ? k : first_create + 1u;
    }

    // ---- phase 0 of round t+1 at x: Gossip::new_message for the rumors
    // injected this round, then MessageState::next_round; churn: a node
    // offline in round t+1 keeps its votes in `pend`, a node back from offline
    // (off_t) takes them from there
    u32 inj = 0;
    if (a.n_inj && valid)  // (segment keys: x * W + u64 word; R_pad 32: x, the low bits)
        inj = lw ? (u32)(find_injection(a, ((u64)x << (lw - 1u)) + (j >> 1)) >> ((j & 1u) << 5))
                 : (u32)find_injection(a, x);
    const bool on_next = !(a.f.churn && valid && offline_of(a.seed, a.epoch, a.round_new, a.node_lo + x, a.f.churn));
    u32 *pend32 = reinterpret_cast<u32 *>(a.pend);  // [n][2][W] u64: (bump, anyC) words
    const u64 pidx = lw ? (((u64)x * 2u) << lw) + j : (u64)x * 4u;
    const uint32_t pstep = lw ? W32 : 2u;
    const bool pending = off_t && valid;
    const u32 pb = pending ? pend32[pidx] : 0u, pa = pending ? pend32[pidx + pstep] : 0u;
    NextOutT<u32> o;
    next_round_seg(P, rv, inj, psize, pending, pb, pa, on_next, a.cmax, a.maxc, a.maxr, o);
    if (!on_next) {  // frozen: pre-transition planes + votes (the lane is valid)
        pend32[pidx] = o.bump;
        pend32[pidx + pstep] = o.anyC;
    }

    // ---- node maps of the round-(t+1) planes for the next in-list build:
    // "live" (its push is not empty) and "complete" (no A entry); a wave's
    // 64 / W32 nodes are whole bytes of the maps (W32 <= 8)
    {
        u32 lvw, aw;
        if (a.f.churn == 0u) {
            lvw = o.Bn | o.Cn;
            aw = ~(o.N[0] | o.Bn);
        } else {
            lvw = (o.N[0] & ~(o.N[1] & o.N[2])) | (~o.N[0] & (o.N[1] | o.N[2]));
            aw = ~o.N[0] & ~o.N[1] & ~o.N[2];
        }
        const u64 bl = __ballot(valid && lvw != 0);
        const u64 bc = __ballot(valid && aw == 0);
        const uint32_t lane = threadIdx.x & 63u;
        const u64 seg0 = seg - lane;
        if (lane == 0 && seg0 < nseg) {
            const u64 cl = lw ? compress_stride(group_or_bits(bl, lw), lw) : bl;
            const u64 cc = lw ? compress_stride(group_and_bits(bc, lw), lw) : bc;
            uint8_t *ml = reinterpret_cast<uint8_t *>(a.lvm), *mc = reinterpret_cast<uint8_t *>(a.cpm);
            const u64 byte0 = (seg0 >> lw) >> 3;  // first node of the wave / 8
            if (lw == 0u) {
                *reinterpret_cast<u64 *>(ml + byte0) = cl;
                *reinterpret_cast<u64 *>(mc + byte0) = cc;
            } else if (lw == 1u) {
                *reinterpret_cast<uint32_t *>(ml + byte0) = (uint32_t)cl;
                *reinterpret_cast<uint32_t *>(mc + byte0) = (uint32_t)cc;
            } else if (lw == 2u) {
                *reinterpret_cast<uint16_t *>(ml + byte0) = (uint16_t)cl;
                *reinterpret_cast<uint16_t *>(mc + byte0) = (uint16_t)cc;
            } else {
                ml[byte0] = (uint8_t)cl;
                mc[byte0] = (uint8_t)cc;
            }
        }
        // traffic accounting of timed launches: the class rows this round's
        // build left to gather (counted there, off the kernel's path)
        if (MODE == 1 && a.acct && a.rows_cnt && bid == 0 && threadIdx.x == 0) atomicAdd(a.acct, *a.rows_cnt);
    }

    // ---- write round-(t+1) planes (through LDS, 16-byte coalesced
    // streaming stores)
    uint32_t live_new = (valid && on_next) ? popcT(o.Bn | o.Cn) : 0u;
    live_new = group_sum(live_new, W32);
    if (__ballot(live_new != 0u) != 0ull && (threadIdx.x & 63u) == 0u) blk_any = 1u;
    if (GS_W32_ZSKIP && __ballot(valid && (o.N[0] | o.N[1] | o.N[2]) != 0u) != 0ull && (threadIdx.x & 63u) == 0u)
        blk_nz = 1u;
    __syncthreads();  // also: every lane is done reading stage
    const bool blk_live = blk_any != 0u;
    // a block whose nodes are all-A in round t+1 were all-A in round t-1 (no
    // entry returns to A; clear zeroes both buffers): Snext, which holds round
    // t-1, has its zero planes already
    const bool zskip = GS_W32_ZSKIP && blk_nz == 0u;
    if (valid && !zskip) {
#pragma unroll
        for (int p = 0; p < kPlanes; ++p) stage[pbase + (uint32_t)p * pstr] = o.N[p];
    }
    if (!zskip) __syncthreads();  // (uniform over the block)
    if (!zskip) {
        const uint4 *s4 = reinterpret_cast<const uint4 *>(stage);
        uint4 *dst4 = reinterpret_cast<uint4 *>(reinterpret_cast<u32 *>(a.Snext) + blk_base);
        if (threadIdx.x < blk_v4) nt_store4(s4[threadIdx.x], &dst4[threadIdx.x]);
        if (threadIdx.x + kW32Threads < blk_v4) nt_store4(s4[threadIdx.x + kW32Threads], &dst4[threadIdx.x + kW32Threads]);
    }

    // ---- push list + Statistics (src/gossip.rs:80,103-111)
    mark_any_live(a.live, a.round_new, bid, blk_live);
    if (leader) {
        // rounds is the engine's round count (every node runs every round);
        // the other four are u32 deltas folded into u64 before they can wrap.
        uint4 v = stv;
        const uint32_t d_empty_push = (on_next && live_new == 0u) ? 1u : 0u;
        if (a.emin) {  // rumor slice: empty only if empty in every slice (MIN per byte, caller)
            reinterpret_cast<uint16_t *>(a.emin)[x] = (uint16_t)(min(d_empty_pull, 255u) | (d_empty_push << 8));
            v.x += eadd & 0xFFu;  // an earlier round's network counts (reduced by the caller)
            v.y += eadd >> 8;
        } else {
            v.x += d_empty_pull;  // empty_pull_sent
            v.y += d_empty_push;  // empty_push_sent
        }
        v.z += live_new + d_full_sent;  // full_message_sent
        v.w += recv;                    // full_message_received
        reinterpret_cast<uint4 *>(a.st32)[x] = v;
        if (!on_next) atomicAdd(&a.offc[x], 1u);  // (no return: nothing waits for it)
    }
}

bool w32_eligible(const RoundArgs &a, int mode) {
    const bool geom = a.g.small ? (a.g.rpad == 32u && a.g.lognpu == 1u) : (a.g.logr >= 6u && a.g.logr <= 8u);
    return a.w32 && (mode == 0 || mode == 1) && geom && !a.recvA &&
           !a.Wb && !a.DR && a.zlm && a.lvm && a.cpm && a.n_ext == 0 && a.blk_off == 0 &&
           a.blk_count == 0;
}

hipError_t launch_round_w32(const RoundArgs &a, int mode, hipStream_t s) {
    if (!w32_eligible(a, mode)) return hipErrorInvalidValue;
    const u64 lanes = (u64)a.g.n << (a.g.logr - 5u);
    const u64 grid = (lanes + kW32Threads - 1) / kW32Threads;
    if (grid == 0) return hipSuccess;
    if (mode == 0)
        hipLaunchKernelGGL(round_kernel_w32<0>, dim3((uint32_t)grid), dim3(kW32Threads), 0, s, a);
    else
        hipLaunchKernelGGL(round_kernel_w32<1>, dim3((uint32_t)grid), dim3(kW32Threads), 0, s, a);
    return hipGetLastError();
}

}  // namespace gs
