// gs_dlv4.hip -- the delivery-record (DLV) round kernel with FOUR nodes per
// lane (2P schedule, R_pad <= 16, transition modes 0 and 1).
//
// On the DLV path (gs_common.h DlvRec) every input of a node's round is read
// coalesced: its record (pushers' push codes), its pull batch, its target
// word, its planes.  With one node per lane the bit-sliced algebra of
// gs_kernels.hip ran on R_pad of the 64 bits of every u64 operation (16 of 64
// at config 5) and the kernel was VALU-bound (982 VALU instructions per wave,
// profiles/r2_dlv4).  Here a lane owns four consecutive nodes whose R_pad-bit
// segments sit side by side in one 4*R_pad-bit field of the plane word, so
// MessageState::next_round (src/message_state.rs:86-171) and the absorption of
// push and pull batches (src/gossip.rs:118-163) run once per four nodes; only
// what is per node stays per node: in-degree, the first-creation index,
// |peers_in_this_round|, the median threshold (a per-segment comparator),
// churn, and the five Statistics counters (src/gossip.rs:103-111,139-163).
// The algebra is the per-node kernel's (gs_kernels.hip, round_kernel DLV
// path), term by term; observation launches and rounds with external RPCs
// still run that kernel.
#include <algorithm>

#include "gs_device.h"
#include "gs_kernels.h"

namespace gs {

#ifndef GS_DLV4_THREADS
#define GS_DLV4_THREADS 256u  // lanes per block (A/B builds: 64, 128)
#endif
#ifndef GS_DLV4_ZSKIP
#define GS_DLV4_ZSKIP 1  // no plane stores for a block whose new planes are all A
#endif
constexpr uint32_t kDlv4Threads = GS_DLV4_THREADS;
static_assert(kDlv4Threads == 64u || kDlv4Threads == 128u || kDlv4Threads == 256u, "whole waves, <= 256");
// 4 waves per SIMD (128 VGPRs): 2.63 -> 2.36 ms at config 5 against the
// unconstrained 134-VGPR build (3 waves)
#ifndef GS_DLV4_MINW
#define GS_DLV4_MINW 4
#endif
#ifndef GS_DLV4_TAIL_PRE
#define GS_DLV4_TAIL_PRE 3  // tail codes per node loaded with the metadata (0..3), two nodes per lane or fewer
#endif
static_assert(GS_DLV4_TAIL_PRE <= 3, "tail prefetch depth");
// the config-5 kernel (R_pad 16, two nodes per u32 lane): 7 waves per SIMD
// (72 VGPRs, no spill with three prefetched tail codes; 8 spilled, round 3)
#ifndef GS_DLV4_MINW_R16
#define GS_DLV4_MINW_R16 7
#endif

// The lane word T holds the lane's nodes side by side (u32: two 16-bit or
// four <= 8-bit segments; u64: four 16-bit segments); the bit-sliced helpers
// of gs_device.h (popcT, add5T, ge_uT) take either width.
// "x >= K" with K given per segment: km[i] holds bit i of every segment's K
// spread over that segment.
template <int NB, typename T>
GS_DEV T ge_seg(const T (&x)[NB], const T (&km)[NB]) {
    T b = 0;
#pragma unroll
    for (int i = 0; i < NB; ++i) b = (~x[i] & b) | (km[i] & (~x[i] | b));
    return ~b;
}

// SH: a code-row shard engine (gs_shard.hip, ShardPlan::codes): the pull code
// x received is read from exchange B at x's slot (spos_cur) instead of
// PULL[x], and its next push code goes with its target into its exchange-A
// row (spos_next) instead of PC[x]; blocks [blk_off, blk_off + grid) (a
// pipeline part).
// EXT: the round's external RPCs (gs_handle_received) are applied after the
// internal deliveries, as in round_kernel (gs_kernels.hip, the a.n_ext
// block); a variant of its own, launched only for a round that has some.
template <int MODE, typename T, uint32_t kNpl, bool SH = false, bool EXT = false>
__global__ __launch_bounds__(kDlv4Threads, (kNpl == 2 && sizeof(T) == 4) ? GS_DLV4_MINW_R16 : GS_DLV4_MINW)
void round_kernel_dlv4(RoundArgs a) {
    constexpr bool DELIVER = MODE == 1;
    const Geometry &g = a.g;
    if (a.zero_buf || a.zero_rows) zero_for_build(a.zero_buf, a.zero_words, a.zero_rows);
    if (a.zero_buf2) zero_for_build(a.zero_buf2, a.zero_words2, nullptr);
    const uint32_t n_nodes = g.n;
    const uint32_t rp = g.rpad, lr = g.logr, lognpu = g.lognpu;  // rp <= 16: npu >= 4
    const uint32_t bid = blockIdx.x + a.blk_off;
    const uint32_t lane = bid * kDlv4Threads + threadIdx.x;
    const uint32_t x0 = lane * kNpl;
    const uint32_t nv = x0 < n_nodes ? min(kNpl, n_nodes - x0) : 0u;  // valid nodes of the lane
    const T m1 = (1ull << rp) - 1ull;
    T M[kNpl];  // segment of node x0 + q within the lane's field
    T mV = 0;
#pragma unroll
    for (uint32_t q = 0; q < kNpl; ++q) {
        M[q] = q < nv ? m1 << (q * rp) : (T)0;
        mV |= M[q];
    }
    // the lane's field: bits [shL, shL + 4*rp) of plane word `unit`
    constexpr uint32_t kLogNpl = kNpl == 4 ? 2u : (kNpl == 2 ? 1u : 0u);
    const uint32_t lpw_log = lognpu - kLogNpl;  // lanes per word = npu / kNpl
    const uint32_t shL = (x0 & ((1u << lognpu) - 1u)) << lr;

    __builtin_amdgcn_s_setprio(2);  // the load-issue phase at raised priority (gs_kernels.hip)
    // ---- own round-t planes, staged through LDS (16-byte coalesced loads)
    __shared__ __attribute__((aligned(16))) u64 stage[kDlv4Threads * kNpl * kPlanes / 4];  // >= 8 words per unit
    const uint32_t units_blk = (kDlv4Threads * kNpl) >> lognpu;
    const u64 unit0 = (u64)bid * units_blk;
    const uint32_t blk_units = (uint32_t)min((u64)units_blk, g.units - min(g.units, unit0));
    const uint32_t blk_v4 = blk_units * (kPlanes / 2u);
    {
        const uint4 *src4 = reinterpret_cast<const uint4 *>(a.Scur + unit0 * kPlanes);
        uint4 *dst4 = reinterpret_cast<uint4 *>(stage);
        uint4 v[kNpl];  // at most kNpl uint4 per thread (R_pad 16: 8 words per kNpl nodes)
#pragma unroll
        for (uint32_t it = 0; it < kNpl; ++it) {
            const uint32_t i = threadIdx.x + kDlv4Threads * it;
            v[it] = src4[min(i, blk_v4 - 1u)];  // blk_v4 >= 4: every block owns a unit
        }
#pragma unroll
        for (uint32_t it = 0; it < kNpl; ++it) {
            const uint32_t i = threadIdx.x + kDlv4Threads * it;
            if (i < blk_v4) dst4[i] = v[it];
        }
    }

    // ---- per-node metadata (coalesced: 16-B records, 4-B words, 4 nodes per lane)
    uint32_t kk[kNpl], dzi[kNpl], dfirst[kNpl], c0[kNpl], c1[kNpl], tgw[kNpl], dp[kNpl];
#pragma unroll
    for (uint32_t q = 0; q < kNpl; ++q) kk[q] = dzi[q] = dfirst[q] = c0[q] = c1[q] = tgw[q] = dp[q] = 0u;
    if (DELIVER && SH) {
        // the pull code at x's exchange-B slot (none: x's push was not
        // delivered, so no pull either; kTgNoPull masks it below)
        const uint32_t *rB = reinterpret_cast<const uint32_t *>(a.recvB);
        uint32_t sp[kNpl];
        if (kNpl == 2 && nv == kNpl) {
            const uint2 t2 = *reinterpret_cast<const uint2 *>(a.tg + x0);
            const uint2 s2 = *reinterpret_cast<const uint2 *>(a.spos_cur + x0);
            tgw[0] = t2.x; tgw[1] = t2.y;
            sp[0] = s2.x; sp[kNpl > 1 ? 1 : 0] = s2.y;
        } else {
#pragma unroll
            for (uint32_t q = 0; q < kNpl; ++q) {
                tgw[q] = q < nv ? a.tg[x0 + q] : 0u;
                sp[q] = q < nv ? a.spos_cur[x0 + q] : 0xFFFFFFFFu;
            }
        }
#pragma unroll
        for (uint32_t q = 0; q < kNpl; ++q) dp[q] = sp[q] != 0xFFFFFFFFu ? rB[sp[q]] : 0u;
    } else if (DELIVER) {  // (the delivery flags come with the records below)
        if (kNpl == 4 && nv == kNpl) {
            const uint4 p4 = *reinterpret_cast<const uint4 *>(a.pull + x0);
            dp[0] = p4.x; dp[1] = p4.y; dp[kNpl > 2 ? 2 : 0] = p4.z; dp[kNpl > 3 ? 3 : 0] = p4.w;
        } else if (kNpl == 2 && nv == kNpl) {
            const uint2 p2 = *reinterpret_cast<const uint2 *>(a.pull + x0);
            dp[0] = p2.x; dp[1] = p2.y;
        } else {
#pragma unroll
            for (uint32_t q = 0; q < kNpl; ++q)
                if (q < nv) dp[q] = a.pull[x0 + q];
        }
    }
    if (DELIVER) {
#pragma unroll
        for (uint32_t q = 0; q < kNpl; ++q) {
            const DlvRec r = a.DR[q < nv ? x0 + q : 0u];  // node 0: a harmless valid address
            kk[q] = q < nv ? (r.mf & 31u) : 0u;
            dzi[q] = (r.mf >> 5) & 31u;
            dfirst[q] = ((x0 + q) >> a.dlv_tlog) * a.dlv_tper + (r.mf >> kDlvFirstShift);
            c0[q] = r.c[0];
            c1[q] = r.c[1];
            if (!SH)  // the build put y's own delivery flags in mf (gs_common.h kDlvMeta*)
                tgw[q] = (((r.mf >> kDlvMetaNoPull) & 1u) ? kTgNoPull : 0u) | (((r.mf >> kDlvMetaOff) & 1u) ? kTgOff : 0u);
        }
    }
    // the first kDlvPre tail codes of every node, loaded now rather than in
    // the delivery loop, where each pusher index with a tail was one
    // dependent memory round trip for nearly every wave (its 128 nodes hold
    // a pusher #3 with probability ~1 and a pusher #4 with ~0.9 at in-degree
    // 1): config 5's kernel 1.689 -> 1.62 ms with two codes (one: no
    // change), 1.62 -> 1.59 with three at 7 waves per SIMD.
    // Four nodes per lane (R_pad < 16) measured slower with them.
    constexpr uint32_t kDlvPre = kNpl <= 2 ? GS_DLV4_TAIL_PRE : 0u;
    uint32_t tpre[kDlvPre > 0 ? kDlvPre : 1][kNpl];
#pragma unroll
    for (uint32_t j = 0; j < kDlvPre; ++j)
#pragma unroll
        for (uint32_t q = 0; q < kNpl; ++q) tpre[j][q] = (DELIVER && kk[q] > kDlvInline + j) ? a.dtail[dfirst[q] + j] : 0u;
    // likewise the votes a node back from offline kept (`pend`, the low words:
    // R_pad <= 16 here), which the transition otherwise waited for mid-kernel
    // (at 1 % churn most waves hold such a node; two nodes per lane only,
    // like the tail codes)
    constexpr bool kPendPre = kNpl <= 2;
    uint32_t pv0[kNpl], pv1[kNpl];
#pragma unroll
    for (uint32_t q = 0; q < kNpl; ++q) {
        const uint32_t *pe = reinterpret_cast<const uint32_t *>(a.pend + (u64)(x0 + q) * 2u);
        const bool off = kPendPre && DELIVER && (tgw[q] & kTgOff);
        pv0[q] = off ? pe[0] : 0u;
        pv1[q] = off ? pe[2] : 0u;
    }
    __builtin_amdgcn_s_setprio(0);
    __syncthreads();
    // class planes now; the five b planes only for the transition (still in
    // LDS then: fewer registers live across the deliveries)
    const uint32_t ul = (lane >> lpw_log) - bid * units_blk;  // the lane's word within the block
    T P[kPlanes];
#pragma unroll
    for (int p = 0; p < 3; ++p) P[p] = nv ? (T)(stage[ul * kPlanes + p] >> shL) & mV : (T)0;

    const T isC = P[0], a0 = P[1], a1 = P[2];
    const T A = ~isC & ~a0 & ~a1 & mV;
    const T B = ~isC & (a0 | a1);
    const T C = isC & ~(a0 & a1);
    const T D = isC & a0 & a1;
    const T liveX = B | C;

    // ---- phases 1 and 2 of round t (Gossip::receive), four nodes at once
    T notyet = A, recB = B, oc1r = B & a0 & ~a1, crB = 0, crC = 0, anyC = 0;
    T cv[5] = {0, 0, 0, 0, 0};
    uint32_t part_cw[kNpl], fc[kNpl], recv[kNpl], psize[kNpl];
    T pulledM = 0, offM = 0;
#pragma unroll
    for (uint32_t q = 0; q < kNpl; ++q) {
        part_cw[q] = recv[q] = psize[q] = 0u;
        fc[q] = kNone;
        if (DELIVER && !(tgw[q] & kTgNoPull)) pulledM |= M[q];
        if (DELIVER && (tgw[q] & kTgOff)) offM |= M[q];
    }
    if (DELIVER) {
        uint32_t kmax = 0;
#pragma unroll
        for (uint32_t q = 0; q < kNpl; ++q) {
            kmax = max(kmax, kk[q]);
            if (kk[q] > 30u) atomicOr(&a.flags[2], 1u);
        }
        for (uint32_t i = 0; i < kmax; ++i) {
            // push batch of pusher i of every node that has one (2-plane code:
            // 01 counter 1, 10 counter 2, 11 counter 255); t(x)'s push copy is
            // superseded by its pull copy (message_state.rs:79), so not recorded
            T b0 = 0, b1 = 0, recm = (T)~(T)0;
#pragma unroll
            for (uint32_t q = 0; q < kNpl; ++q) {
                if (i < kk[q]) {
                    uint32_t code;
                    if (i == 0) code = c0[q];
                    else if (i == 1) code = c1[q];
                    else if (kDlvPre > 0 && i == kDlvInline) code = tpre[0][q];
                    else if (kDlvPre > 1 && i == kDlvInline + 1) code = tpre[kDlvPre > 1 ? 1 : 0][q];
                    else if (kDlvPre > 2 && i == kDlvInline + 2) code = tpre[kDlvPre > 2 ? 2 : 0][q];
                    else code = a.dtail[dfirst[q] + i - kDlvInline];
                    b0 |= ((T)code & m1) << (q * rp);
                    b1 |= ((T)(code >> 16) & m1) << (q * rp);
                    if ((pulledM & M[q]) && i == dzi[q]) recm &= ~M[q];
                }
            }
            const T vC = b0 & b1, vB = b0 ^ b1, v2 = b1 & ~b0, sl = b0 | b1;
            const T newc = notyet & sl;           // new_from_peer: not recorded
            const T rec = recB & sl & recm;       // MessageState::receive on B
            anyC |= rec & vC;
            add5T(cv, rec & vB & (v2 | oc1r));
            crB |= newc & ~vC;
            crC |= newc & vC;
            recB |= newc & ~vC;
            oc1r |= newc & ~vC;
            notyet &= ~newc;
#pragma unroll
            for (uint32_t q = 0; q < kNpl; ++q) {
                const uint32_t pc = popcT(newc & M[q]);
                part_cw[q] += (kk[q] - 1u - i) * pc;  // later pushers' pull rows include it
                if (pc && fc[q] == kNone) fc[q] = i;
                recv[q] += popcT(sl & M[q]);
            }
        }
        // the pull batch t(x) returned (built by the in-list build; the slot
        // of a node whose pull is not delivered holds garbage: masked out
        // before it is shifted into place)
        T pb0 = 0, pb1 = 0;
#pragma unroll
        for (uint32_t q = 0; q < kNpl; ++q) {
            pb0 |= ((T)dp[q] & m1) << (q * rp);
            pb1 |= ((T)(dp[q] >> 16) & m1) << (q * rp);
        }
        pb0 &= pulledM;
        pb1 &= pulledM;
        const T pv2 = pb1 & ~pb0, pvB = pb0 ^ pb1, pCl = pb0 & pb1, pl = pb0 | pb1;
        {
            const T newc = notyet & pl;
            const T rec = recB & pl;
            anyC |= rec & pCl;
            add5T(cv, rec & pvB & (pv2 | oc1r));
            crB |= newc & ~pCl;
            crC |= newc & pCl;
            recB |= newc & ~pCl;
            oc1r |= newc & ~pCl;
            notyet &= ~newc;
        }
#pragma unroll
        for (uint32_t q = 0; q < kNpl; ++q) {
            recv[q] += popcT(pl & M[q]);
            const bool pulled = (pulledM & M[q]) != 0;
            psize[q] = kk[q] + ((pulled && dzi[q] == kDlvNoZ) ? 1u : 0u);  // |peers_in_this_round|
        }
    }
    // External RPCs to the lane's nodes (sorted by node, then call order),
    // after every internal delivery (Gossip::receive, src/gossip.rs:118-163):
    // a first RPC from a peer joins peers_in_this_round, a first Push is
    // answered with the node's live set at that point, a copy creates an
    // absent entry or is recorded on a B entry (the last copy per peer).
    uint32_t ext_full[kNpl], ext_empty[kNpl], ext_recv[kNpl];
#pragma unroll
    for (uint32_t q = 0; q < kNpl; ++q) ext_full[q] = ext_empty[q] = ext_recv[q] = 0u;
    if (EXT && DELIVER && a.n_ext && nv) {
        uint32_t lo = 0, hi = a.n_ext;
        const u64 key = (u64)x0 << 32;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (a.ext[mid] < key) lo = mid + 1; else hi = mid;
        }
        for (uint32_t i = lo; i < a.n_ext; ++i) {
            const uint32_t qe = (uint32_t)(a.ext[i] >> 32) - x0;
            if (qe >= nv) break;
            const uint32_t info = (uint32_t)a.ext[i];
            const T Mq = m1 << (qe * rp);
            uint32_t dn = 0, df = 0, de = 0, dr = 0;
            if (info & kExtNew) dn = 1u;
            if ((info & kExtPush) && (info & kExtNew)) {
                const uint32_t cnt = popcT((B | C | crB | crC) & Mq);
                if (cnt) df = cnt; else de = 1u;
            }
            if (!(info & kExtEmpty)) {
                dr = 1u;
                const uint32_t r = info & 0xFFFu, c = (info >> 12) & 0xFFu;
                const T bit = ((T)1 << r) << (qe * rp);
                // a counter >= counter_max acts as C; 0 creates B and votes "less"
                const T vC = c >= a.cmax ? bit : (T)0;
                const T vB = (c >= 1u && c < a.cmax) ? bit : (T)0;
                const T v2 = (c == 2u && c < a.cmax) ? bit : (T)0;
                const T newc = notyet & bit;
                const T rec = recB & bit & ((info & kExtRec) ? (T)~(T)0 : (T)0);
                anyC |= rec & vC;
                add5T(cv, rec & vB & (v2 | oc1r));
                crB |= newc & ~vC;
                crC |= newc & vC;
                recB |= newc & ~vC;
                oc1r |= newc & ~vC;
                notyet &= ~newc;
            }
#pragma unroll
            for (uint32_t q = 0; q < kNpl; ++q)
                if (q == qe) {
                    psize[q] += dn;
                    ext_full[q] += df;
                    ext_empty[q] += de;
                    ext_recv[q] += dr;
                }
        }
    }

    // Statistics deltas of the deliveries
    uint32_t d_empty_pull[kNpl], d_full[kNpl];
#pragma unroll
    for (uint32_t q = 0; q < kNpl; ++q) {
        d_empty_pull[q] = d_full[q] = 0u;
        if (DELIVER) {
            const uint32_t lc = popcT(liveX & M[q]);
            d_full[q] = kk[q] * lc + part_cw[q];  // pull rows sent by x
            if (kk[q] > 0 && lc == 0) d_empty_pull[q] = (fc[q] == kNone) ? kk[q] : fc[q] + 1u;
        }
    }

    // ---- phase 0 of round t+1: injections, MessageState::next_round
    T inj = 0;
    if (a.n_inj && nv) {
        uint32_t lo = 0, hi = a.n_inj;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (a.inj_key[mid] < x0) lo = mid + 1; else hi = mid;
        }
        for (uint32_t i = lo; i < a.n_inj && a.inj_key[i] < (u64)x0 + nv; ++i)
            inj |= ((T)a.inj_mask[i] & m1) << ((uint32_t)(a.inj_key[i] - x0) * rp);
    }
    const T ninj = ~inj;
    const T Bold = B & ninj, Cold = C & ninj, Dold = D & ninj;
    const T cB = crB & ninj, cC = crC & ninj;
    const T Bf = Bold | cB | inj;
    const T Cf = Cold | cC;
    const T oc1 = (Bold & a0 & ~a1) | cB | inj;
    const T oc2 = Bold & a1 & ~a0;
    // median rule with 0-filled peers: bump iff ge >= |P|/2 + 1, per node
    T km[5] = {0, 0, 0, 0, 0}, kbig = 0;
#pragma unroll
    for (uint32_t q = 0; q < kNpl; ++q) {
        const uint32_t thr = psize[q] / 2u + 1u;
#pragma unroll
        for (int i = 0; i < 5; ++i)
            if ((thr >> i) & 1u) km[i] |= M[q];
        if (thr >= 32u) kbig |= M[q];
    }
    T bump = ge_seg<5>(cv, km) & ~kbig & (Bold | cB);
    T anyCe = anyC & ninj;
    if (DELIVER && offM) {  // back from offline: the votes its skipped next_round kept
#pragma unroll
        for (uint32_t q = 0; q < kNpl; ++q)
            if (offM & M[q]) {
                const u64 *pe = a.pend + (u64)(x0 + q) * 2u;
                const T v0 = kPendPre ? (T)pv0[q] : (T)pe[0], v1 = kPendPre ? (T)pv1[q] : (T)pe[1];
                bump = (bump & ~M[q]) | ((v0 & m1) << (q * rp) & Bold);
                anyCe = (anyCe & ~M[q]) | ((v1 & m1) << (q * rp) & ninj);
            }
    }
#pragma unroll
    for (int p = 3; p < kPlanes; ++p) P[p] = nv ? (T)(stage[ul * kPlanes + p] >> shL) & mV : (T)0;
    T nr[6];  // round + 1
    {
        T carry = (T)~(T)0;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const T rb = P[3 + i] & Bold;
            nr[i] = rb ^ carry;
            carry &= rb;
        }
        nr[5] = carry;
    }
    const T toD = ge_uT<6>(nr, a.maxr);
    const T oc1n = oc1 & ~bump;
    const T oc2n = (oc1 & bump) | (oc2 & ~bump);
    const T oc3n = oc2 & bump;
    const T ocge = a.cmax <= 1u ? (T)~(T)0 : (a.cmax == 2u ? (oc2n | oc3n) : oc3n);
    const T toC = anyCe | ocge;
    const T BD = Bf & toD, BC = Bf & ~toD & toC, BB = Bf & ~toD & ~toC;
    const T cr0 = a0 & Cold, cr1 = a1 & Cold;
    const T d[3] = {~cr0, cr1 ^ cr0, cr1 & cr0};
    T rib[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) rib[i] = P[3 + i] & Cold;
    T sum[6];
    {
        T c = 0;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const T di = i < 3 ? d[i] : (T)0;
            sum[i] = rib[i] ^ di ^ c;
            c = (rib[i] & di) | (c & (rib[i] ^ di));
        }
        sum[5] = c;
    }
    const T CtoD = ge_uT<6>(sum, a.maxr) | ge_uT<3>(d, a.maxc);
    const T CD = Cf & CtoD, CC = Cf & ~CtoD;
    const T Dn = BD | CD | Dold;
    const T Cn = BC | CC;
    const T Bn = BB;
    T N[kPlanes];
    N[0] = Cn | Dn;
    N[1] = (Bn & oc1n) | (CC & d[0]) | Dn;
    N[2] = (Bn & oc2n) | (CC & d[1]) | Dn;
#pragma unroll
    for (int i = 0; i < 5; ++i) N[3 + i] = ((Bn | BC) & nr[i]) | (CC & rib[i]);

    // churn: a node offline in round t+1 skips next_round and keeps its
    // pre-transition state and the two votes in `pend`
    T onM = mV;
    if (a.f.churn) {
#pragma unroll
        for (uint32_t q = 0; q < kNpl; ++q)
            if (q < nv && offline_of(a.seed, a.epoch, a.round_new, a.node_lo + x0 + q, a.f.churn)) onM &= ~M[q];
    }
    if (onM != mV) {
        const T fz = mV & ~onM;
        const T F[3] = {(isC & ninj) | cC, (a0 & ninj) | cB | inj, a1 & ninj};
#pragma unroll
        for (int p = 0; p < kPlanes; ++p) {
            const T f = p < 3 ? F[p] : (P[p] & ninj);
            N[p] = (N[p] & onM) | (f & fz);
        }
        const T av = anyCe & (Bold | cB);
#pragma unroll
        for (uint32_t q = 0; q < kNpl; ++q)
            if (fz & M[q]) {
                u64 *pe = a.pend + (u64)(x0 + q) * 2u;
                pe[0] = (u64)((bump >> (q * rp)) & m1);
                pe[1] = (u64)((av >> (q * rp)) & m1);
            }
    }

    // the Statistics counters this round updates (read now: the stores below
    // cover the load's latency)
    uint4 stv[kNpl];
#pragma unroll
    for (uint32_t q = 0; q < kNpl; ++q) stv[q] = q < nv ? load_stats(a.st32, a.st16, x0 + q) : make_uint4(0u, 0u, 0u, 0u);
    // rumor slice: an earlier round's network empty counts (pull | push << 8)
    uint32_t eav[kNpl];
#pragma unroll
    for (uint32_t q = 0; q < kNpl; ++q)
        eav[q] = (a.eadd && q < nv) ? reinterpret_cast<const uint16_t *>(a.eadd)[x0 + q] : 0u;

    // ---- push codes of round t+1 for the in-list build (4 B per node)
    uint32_t pc[kNpl];
    {
        const T vC = N[0] & ~(N[1] & N[2]), vB = ~N[0] & (N[1] | N[2]);
        const T b0 = (vB & N[1] & ~N[2]) | vC, b1 = (vB & N[2] & ~N[1]) | vC;
#pragma unroll
        for (uint32_t q = 0; q < kNpl; ++q)
            pc[q] = (uint32_t)((b0 >> (q * rp)) & m1) | ((uint32_t)((b1 >> (q * rp)) & m1) << 16);
        if (!SH) {
            // the known masks (state != A): with its push code, all a target's
            // planes tell the build about the pull batch it returns (4 + 2 B
            // per node there instead of whole 128-B lines of plane records)
            const T kn = N[0] | N[1] | N[2];
            uint32_t k16[kNpl];
#pragma unroll
            for (uint32_t q = 0; q < kNpl; ++q) k16[q] = (uint32_t)((kn >> (q * rp)) & m1);
            if (kNpl == 4 && nv == kNpl) {
                *reinterpret_cast<uint2 *>(a.kn_out + x0) =
                    make_uint2(k16[0] | (k16[kNpl > 1 ? 1 : 0] << 16), k16[kNpl > 2 ? 2 : 0] | (k16[kNpl > 3 ? 3 : 0] << 16));
            } else if (kNpl == 2 && nv == kNpl) {
                *reinterpret_cast<uint32_t *>(a.kn_out + x0) = k16[0] | (k16[kNpl > 1 ? 1 : 0] << 16);
            } else {
#pragma unroll
                for (uint32_t q = 0; q < kNpl; ++q)
                    if (q < nv) a.kn_out[x0 + q] = (uint16_t)k16[q];
            }
        }
        if (SH) {
            // exchange A of round t+1: to owner(t_{t+1}(x)) (no slot: an
            // undelivered edge, or a capacity overflow, flagged by the plan),
            // the row (push code, target local to that rank | kRowMutual when
            // t_{t+1}(t_{t+1}(x)) = x: x is its target's own target, whose
            // push copy the pull copy supersedes, src/message_state.rs:79)
            // (a row to this rank's own nodes goes straight into the receive
            // buffer's own block, same slot: one rank exchanges nothing; with
            // several the all-to-all still copies the send buffer's own block
            // over it, so the row goes there too)
            uint2 *sA = reinterpret_cast<uint2 *>(a.sendA);
            uint2 *rA = reinterpret_cast<uint2 *>(a.recvA_next);
            const uint32_t me = a.node_lo / a.sp.chunk;
#pragma unroll
            for (uint32_t q = 0; q < kNpl; ++q) {
                const uint32_t sp = q < nv ? a.spos_next[x0 + q] : 0xFFFFFFFFu;
                if (sp == 0xFFFFFFFFu) continue;
                const uint32_t t = a.tg_next[x0 + q] & kTgMask;
                const uint32_t td = t / a.sp.chunk, tl = t - td * a.sp.chunk;
                const bool mutual = peer_of(a.seed, a.epoch, a.round_new, t, a.sp.n) == a.node_lo + x0 + q;
                const uint2 row = make_uint2(pc[q], tl | (mutual ? kRowMutual : 0u));
                if (td == me) rA[sp] = row;
                if (td != me || a.sp.G > 1) sA[sp] = row;
            }
        } else if (kNpl == 4 && nv == kNpl) {
            *reinterpret_cast<uint4 *>(a.pc_out + x0) =
                make_uint4(pc[0], pc[1], pc[kNpl > 2 ? 2 : 0], pc[kNpl > 3 ? 3 : 0]);
        } else if (kNpl == 2 && nv == kNpl) {
            *reinterpret_cast<uint2 *>(a.pc_out + x0) = make_uint2(pc[0], pc[1]);
        } else {
#pragma unroll
            for (uint32_t q = 0; q < kNpl; ++q)
                if (q < nv) a.pc_out[x0 + q] = pc[q];
        }
    }

    // ---- write round-(t+1) planes (lanes of one word OR their fields; LDS
    // stage, 16-byte coalesced nontemporal stores)
    __shared__ uint32_t blk_any, blk_nz;  // (blk_nz: some node not all-A in round t+1, GS_DLV4_ZSKIP)
    if (threadIdx.x == 0) blk_any = 0;
    if (threadIdx.x == 0) blk_nz = 0;
    uint32_t live[kNpl];
    bool any_live = false;
#pragma unroll
    for (uint32_t q = 0; q < kNpl; ++q) {
        live[q] = (onM & M[q]) ? popcT((Bn | Cn) & M[q]) : 0u;
        any_live |= live[q] != 0u;
    }
    __syncthreads();  // every lane is done reading stage; blk_any is cleared
    __builtin_amdgcn_s_setprio(1);
    {
        const uint32_t lpw = 1u << lpw_log;
#pragma unroll
        for (int p = 0; p < kPlanes; ++p) {
            u64 v = (u64)(N[p] & mV) << shL;
            for (uint32_t o = 1; o < lpw; o <<= 1) v |= __shfl_xor(v, (int)o, 64);
            if ((lane & (lpw - 1u)) == 0u && nv) stage[ul * kPlanes + p] = v;
        }
    }
    if (__ballot(any_live) != 0ull && (threadIdx.x & 63u) == 0u) blk_any = 1u;
    if (GS_DLV4_ZSKIP && __ballot(((N[0] | N[1] | N[2]) & mV) != (T)0) != 0ull && (threadIdx.x & 63u) == 0u)
        blk_nz = 1u;
    __syncthreads();
    // a block whose nodes are all-A in round t+1 were all-A in round t-1
    // (no entry returns to A; clear zeroes both buffers): Snext, which holds
    // round t-1, has its zero planes already
    if (!GS_DLV4_ZSKIP || blk_nz != 0u) {
        const uint4 *src4 = reinterpret_cast<const uint4 *>(stage);
        uint4 *dst4 = reinterpret_cast<uint4 *>(a.Snext + unit0 * kPlanes);
#pragma unroll
        for (uint32_t it = 0; it < kNpl; ++it) {
            const uint32_t i = threadIdx.x + kDlv4Threads * it;
            if (i < blk_v4) nt_store4(src4[i], &dst4[i]);
        }
    }

    // ---- any-live flag of round t+1, Statistics (src/gossip.rs:80,103-111)
    mark_any_live(a.live, a.round_new, bid, blk_any != 0u);
#pragma unroll
    for (uint32_t q = 0; q < kNpl; ++q) {
        if (q >= nv) break;
        const bool on = (onM & M[q]) != 0;
        uint4 v = stv[q];
        if (EXT) {
            // u16 deltas hold internal deliveries only (bounded per round):
            // external RPCs go to the totals -- but a rumor slice's empty
            // pulls go through emin (MIN over the slices; the engine bounds
            // them, gs_engine.cpp slice_ext_limit)
            u64 *s64 = const_cast<u64 *>(a.st64) + (u64)(x0 + q) * 4u;
            if (a.emin) d_empty_pull[q] += ext_empty[q];
            else if (ext_empty[q]) s64[0] += ext_empty[q];
            if (ext_full[q]) s64[2] += ext_full[q];
            if (ext_recv[q]) s64[3] += ext_recv[q];
        }
        const uint32_t d_empty_push = (on && live[q] == 0u) ? 1u : 0u;
        if (a.emin) {  // rumor slice: empty only if empty in every slice (MIN per byte, caller)
            reinterpret_cast<uint16_t *>(a.emin)[x0 + q] =
                (uint16_t)(min(d_empty_pull[q], 255u) | (d_empty_push << 8));
            v.x += eav[q] & 0xFFu;
            v.y += eav[q] >> 8;
        } else {
            v.x += d_empty_pull[q];                   // empty_pull_sent
            v.y += d_empty_push;                      // empty_push_sent
        }
        v.z += live[q] + d_full[q];                   // full_message_sent
        v.w += recv[q];                               // full_message_received
        store_stats(a.st32, a.st16, x0 + q, v);
        // (a non-returning atomic: a load + store here left ~3/4 of the waves
        // waiting a memory round trip at their end at 1 % churn)
        if (!on) atomicAdd(&a.offc[x0 + q], 1u);
    }
}

template <typename T, uint32_t NPL>
static hipError_t launch_dlv4_t(const RoundArgs &a, int mode, hipStream_t s) {
    const u64 lanes = ((u64)a.g.n + NPL - 1) / NPL;
    const u64 nblk = (lanes + kDlv4Threads - 1) / kDlv4Threads;
    // a shard part's blocks come in 256-lane units (gs_engine.cpp launch_part)
    constexpr u64 f = 256u / kDlv4Threads;
    const u64 b0 = (u64)a.blk_off * f;
    const u64 b1 = a.blk_count ? std::min<u64>(((u64)a.blk_off + a.blk_count) * f, nblk) : nblk;
    if (b1 <= b0) return hipSuccess;
    const u64 grid = b1 - b0;
    RoundArgs b = a;
    b.blk_off = (uint32_t)b0;
    const dim3 gd((uint32_t)grid), bd(kDlv4Threads);
    // (external RPCs only ever come with a delivery: mode 1)
    const bool ext = mode == 1 && a.n_ext > 0;
    if (ext && !a.ext) return hipErrorInvalidValue;
    if (a.recvA) {  // code-row shard
        if (!a.sp.codes || !a.recvB || !a.sendA || !a.recvA_next || !a.spos_cur || !a.spos_next || !a.tg_next ||
            !a.sp.chunk)
            return hipErrorInvalidValue;
        if (mode == 0) hipLaunchKernelGGL((round_kernel_dlv4<0, T, NPL, true>), gd, bd, 0, s, b);
        else if (ext) hipLaunchKernelGGL((round_kernel_dlv4<1, T, NPL, true, true>), gd, bd, 0, s, b);
        else hipLaunchKernelGGL((round_kernel_dlv4<1, T, NPL, true>), gd, bd, 0, s, b);
    } else {
        if (mode == 0) hipLaunchKernelGGL((round_kernel_dlv4<0, T, NPL>), gd, bd, 0, s, b);
        else if (ext) hipLaunchKernelGGL((round_kernel_dlv4<1, T, NPL, false, true>), gd, bd, 0, s, b);
        else hipLaunchKernelGGL((round_kernel_dlv4<1, T, NPL>), gd, bd, 0, s, b);
    }
    return hipGetLastError();
}

// Lane word per R_pad: u32 holding two 16-bit or four <= 8-bit segments
// (default); dlv_pack == 2 selects u64 words of four 16-bit segments.
hipError_t launch_round_dlv4(const RoundArgs &a, int mode, hipStream_t s) {
    if (a.g.rpad > 16) return hipErrorInvalidValue;
    if (a.g.rpad == 16) {
        if (a.dlv_pack == 2) return launch_dlv4_t<u64, 4>(a, mode, s);
        if (a.dlv_pack == 3) return launch_dlv4_t<uint32_t, 1>(a, mode, s);
        return launch_dlv4_t<uint32_t, 2>(a, mode, s);
    }
    if (a.dlv_pack == 3) return launch_dlv4_t<uint32_t, 1>(a, mode, s);
    return launch_dlv4_t<uint32_t, 4>(a, mode, s);
}

}  // namespace gs
