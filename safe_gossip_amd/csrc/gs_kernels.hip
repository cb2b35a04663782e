// gs_kernels.hip -- hand-written gfx950 kernels of one safe_gossip push-pull
// round over the whole population (2P schedule).
//
// One lane owns one SEGMENT: (node x, 64-rumor word j) when R >= 64, or the
// whole R-bit rumor row of node x when R < 64 (several nodes share a word).
// All per-rumor logic is bit-sliced over the segment (64 rumors per u64
// operation); nothing is per-rumor scalar.
//
// The round kernel fuses, for every node x:
//   phase 1 of round t at x  : Gossip::receive of every push batch x got,
//                              ascending pusher order (src/gossip.rs:118-163)
//   phase 2 of round t at x  : Gossip::receive of the pull batch from t(x)
//   phase 0 of round t+1 at x: Gossip::new_message injections
//                              (src/gossip.rs:71-75), then Gossip::next_round
//                              = MessageState::next_round for every rumor
//                              (src/message_state.rs:86-171) + push list +
//                              Statistics (src/gossip.rs:79-113).
// B.peer_counters are never materialised: the copies x received are
// re-derived from the round-t class planes of its pushers and of t(x), which
// is all MessageState::next_round consumes (anyC + a count of counters >= own).
//
// Latency structure: every per-node metadata read (IN[x], SIB[x], own planes,
// statistics) is coalesced; the only random accesses are the class-plane
// gathers of the pushers, of t(x) and of t(x)'s earlier pushers, and they are
// all issued together, one dependent level after the coalesced reads.
#include "gs_kernels.h"
#include "gs_device.h"
#include "gs_recv.h"

namespace gs {

// Lanes of a round-kernel block (BLK): one wave (64 lanes) for the
// transitions of the gather path and of class-row shards with 64 <= R_pad <=
// 1024 (64 / W nodes; a thread's uint4 steps of 2 BLK words must cover whole
// nodes), 256 otherwise.  The observation launches and the shard parts count
// their blocks in 256 lanes (gs_engine.cpp); launch_mode converts.  A block's
// two barriers wait for no other wave: config 4's round kernel 2.470 ->
// 2.343 ms with two-wave blocks, 2.321 -> 2.222 ms with one-wave blocks
// (2.810 -> 2.693 -> 2.582 ms per step; profiles/r6/ab_blk128/, ab_blk64/).
#ifndef GS_RK_SMALL_BLK
#define GS_RK_SMALL_BLK 64u  // (A/B builds: 128)
#endif
constexpr uint32_t kRkSmallBlk = GS_RK_SMALL_BLK;
static_assert(kRkSmallBlk == 64u || kRkSmallBlk == 128u, "a thread's stage step must cover whole nodes at W <= 16");

#ifndef GS_RK_MINW
#define GS_RK_MINW 1
#endif
#ifndef GS_RK_MINW_SMALL
#define GS_RK_MINW_SMALL 1  // waves per SIMD asked of the small-block transitions (A/B builds)
#endif
#ifndef GS_RK_ZSKIP
#define GS_RK_ZSKIP 1  // one-wave blocks: no plane stores for a wave whose new planes are all A
#endif
#ifndef GS_RK_ZSKIP_BLK
#define GS_RK_ZSKIP_BLK 0  // the same for a whole 256-lane transition block (off: no bench configuration
                           // runs these blocks, and one SEQ harness mismatch, not reproduced, followed it)
#endif

#ifndef GS_RK_TAILPRE
#define GS_RK_TAILPRE 1  // rows of pusher #3 and of t(x)'s sibling #2 issued with the batch (A/B: 0)
#endif

// MODE: 0 transition only (first round), 1 deliver round t + transition to
// t+1, 2 deliver round t + observe, 3 observe only.
// SHARD: this engine owns a node range of a sharded network; pusher class rows
// and the pull row come from the exchange buffers (recvA, recvB) instead of
// gathers, and the new class planes are also written as push rows (sendA).
// SEQ: the literal harness order (gs_seq.hip): x's pull batch W(x) was built
// by the level passes, and it is absorbed at x's own position among its
// pushers (time x), answered pushes included.
// DLV (R_pad <= 16, 2P): a push code (b0 | b1 << 16) as class planes.
GS_DEV Cls decode16(uint32_t code) {
    const u64 b0 = code & 0xFFFFu, b1 = code >> 16;
    return Cls{b0 & b1, b0 & ~b1, b1 & ~b0};
}

// DLV: delivery records (gs_common.h DlvRec) replace every class-plane
// gather: a lane's pushers' push codes are in its own record and its pull
// batch in PULL[x], both read coalesced.
template <bool SMALL, int MODE, bool SHARD, bool SEQ, bool DLV, uint32_t BLK = 256u>
__global__ __launch_bounds__(BLK, BLK == 256u ? GS_RK_MINW : GS_RK_MINW_SMALL) void round_kernel(RoundArgs a) {
    constexpr bool DELIVER = (MODE == 1 || MODE == 2);
    constexpr bool TRANSITION = (MODE == 0 || MODE == 1);
    const Geometry &g = a.g;
    // words of planes one block owns (its records are contiguous), uint4
    // loads per thread, and the stage (padded node strides: <= 10/8)
    constexpr uint32_t kBlk = BLK;
    static_assert(BLK == 256u || (!SMALL && !SEQ && !DLV && (MODE == 0 || MODE == 1)),
                  "smaller blocks: gather-path and class-row shard transitions only");
    constexpr uint32_t kBlockWords = kBlk * kPlanes;
    constexpr uint32_t kStageIters = kBlockWords / 2u / kBlk;
    constexpr uint32_t kStageWords = kBlockWords + kBlockWords / 4u;
    if (a.zero_buf || a.zero_rows) zero_for_build(a.zero_buf, a.zero_words, a.zero_rows);
    if (a.zero_buf2) zero_for_build(a.zero_buf2, a.zero_words2, nullptr);
    const uint32_t bid = (!TRANSITION && a.blk_list) ? a.blk_list[blockIdx.x] : blockIdx.x + a.blk_off;
    const u64 seg = (u64)bid * blockDim.x + threadIdx.x;
    const bool valid = seg < g.nseg;
    Lane<SMALL> L;
    L.init(g, valid ? seg : 0);
    const uint32_t x = L.x;
    const u64 *__restrict__ S = a.Scur;

    __shared__ uint32_t blk_any;  // some node pushes a live rumor in round t+1
    __shared__ uint32_t blk_nz;   // some node is not all-A in round t+1 (256-lane zero skip)
    if (threadIdx.x == 0) blk_any = 0;
    if (threadIdx.x == 0) blk_nz = 0;
    // the load-issue phase at raised priority: a young wave's requests go out
    // ahead of older waves' compute (issue is by priority, then age)
    __builtin_amdgcn_s_setprio(2);

    // ---- own round-t planes: the block's records are one contiguous range
    // (W <= 256), loaded first with 16-byte coalesced loads (clamped, so every
    // load is unconditional) and transposed through LDS below, instead of
    // eight strided 8-byte loads per lane.
    // (W lanes per node, W >= 1: a node's 8 W words sit at a padded stride
    // of 8 W + W words (8 W + 2 at W = 1), so the 32 lanes of a ds_read_b64
    // / ds_write_b64 group -- 32 / W nodes -- fall on distinct banks; at the
    // unpadded stride every node started on bank 0: 8-way conflicts at W = 4,
    // 59 % of the LDS cycles at config 4)
    __shared__ __attribute__((aligned(16))) u64 stage[kStageWords];
    const uint32_t wlog = SMALL ? 0u : g.logr - 6u;
    const uint32_t pst = SMALL ? 0u : (9u << wlog) + (wlog == 0u ? 1u : 0u);  // padded node stride (words)
    auto sidx = [&](uint32_t li) -> uint32_t {  // the block's word li -> its stage index
        return SMALL ? li : (li >> (wlog + 3u)) * pst + (li & ((8u << wlog) - 1u));
    };
    // uint4 i = the block's words 2i, 2i + 1 (one node's, 16-B aligned at the
    // padded stride too): the thread's i = tid + kBlk m sit s4 + m s4d apart
    const uint32_t s4 = sidx(2u * threadIdx.x), s4d = SMALL ? 2u * kBlk : ((kBlk / 4u) >> wlog) * pst;
    const uint32_t npu_blk = SMALL ? (1u << g.lognpu) : 1u;
    const u64 blk_base = (u64)bid * (kBlockWords / npu_blk);
    const uint32_t blk_v4 = (uint32_t)min((u64)(kBlockWords / npu_blk),
                                          g.units * kPlanes * (SMALL ? 1u : g.W) - blk_base) / 2u;
    static_assert(kStageIters == 4, "stage loads are unrolled by hand");
    const uint4 *src4 = reinterpret_cast<const uint4 *>(S + blk_base);
    const uint4 st0 = src4[min(threadIdx.x, blk_v4 - 1u)];
    const uint4 st1 = src4[min(threadIdx.x + kBlk, blk_v4 - 1u)];
    const uint4 st2 = src4[min(threadIdx.x + 2u * kBlk, blk_v4 - 1u)];
    const uint4 st3 = src4[min(threadIdx.x + 3u * kBlk, blk_v4 - 1u)];

    // ---- coalesced per-node metadata (level 1)
    // Statistics deltas of x, loaded with the other level-1 reads so the
    // read-modify-write at the end adds no dependent memory round trip
    uint4 stv = {0u, 0u, 0u, 0u};
    if (TRANSITION && valid && (SMALL || L.j == 0)) stv = load_stats(a.st32, a.st16, x);
    // rumor slice: an earlier round's network empty counts (pull | push << 8)
    uint32_t eadd = 0;
    if (TRANSITION && a.eadd && valid && (SMALL || L.j == 0)) eadd = reinterpret_cast<const uint16_t *>(a.eadd)[x];
    uint4 in = {0, 0, 0, 0};   // SHARD: {first, k|zi<<16, e0, e1}
    InRec in8 = {};            // {first << 5 | k, s0..s2}
    SibRec sb8 = {};           // {serial<<8 | rank of x in in(z), e0..e2}; stale unless rank >= 1
    uint32_t z = x, zi = 0xFFFFu, k = 0, r = 0;
    uint32_t tgw = 0;  // round-t target word: t(x) + delivery flags (gs_common.h)
    uint32_t sinf = 0;  // SEQ: got << 7 | ... (gs_seq.hip)
    bool seq_inl = false;  // SEQ: W(x) built here, not by a pull pass (kSeqInline)
    bool seq_dep = false;  // SEQ: W(x) includes W(t(x)) (kSeqDep)
    DlvRec dr = {};     // DLV: x's record
    uint32_t dpull = 0;  // DLV: x's pull batch
    // live-filtered gathers (2P gather path; gs_common.h kSkipBit)
    const bool filt = !SHARD && !SEQ && !DLV && a.zlm != nullptr;
    u64 zlw = 0;            // the zl word of x: bit x & 63 = t(x) is live
    uint32_t qskip = 0;     // inline pushers that push nothing
    uint32_t eskip = 0;     // inline siblings that cannot pass anything on
    bool zneed = false;     // a live sibling ahead of x and t(x) incomplete
    bool gq[kBatchK], ge[kBatchE], gz = true;  // filtered: rows wanted
#pragma unroll
    for (uint32_t i = 0; i < kBatchK; ++i) gq[i] = true;
#pragma unroll
    for (uint32_t i = 0; i < kBatchE; ++i) ge[i] = true;
    if (DELIVER) {
        if (DLV) {
            dr = a.DR[x];  // x = 0 on invalid lanes: a harmless valid address
            tgw = a.tg[x];
            dpull = a.pull[x];
            z = tgw & kTgMask;
            k = valid ? (dr.mf & 31u) : 0u;
        } else if (SHARD) {
            if (valid) {
                in = a.IN[x];
                zi = in.y >> 16;
                k = in.y & 0xFFFFu;
                if (faults_on(a.f)) tgw = a.tg[x];
            }
        } else {
            in8 = a.IN8[x];  // x = 0 on invalid lanes: a harmless valid address
            tgw = a.tg[x];
            z = tgw & kTgMask;  // t_t(x)
            k = valid ? in8.k() : 0u;
            if (SEQ) sinf = a.sinfo[x];
            sb8 = a.SIB8[x];
            if (filt) zlw = a.zlm[x >> 6];
            const bool sib_ok = valid && (sb8.tag >> 8) == (a.serial & kSerialMask);
            r = sib_ok ? (sb8.tag & kSibRankMask) : 0u;
            if (filt) {
                // live-filtered gathers: the skip flags (gs_common.h)
                qskip = in8.kf >> kInSkipShift;
                in8.kf &= kInFlagMask;
                eskip = ((sb8.tag >> kSibSkipShift) & 3u) | ((sb8.e[2] >> 31) << 2);
                sb8.e[2] &= kIdMask;
                zneed = sib_ok && (sb8.tag & kSibZNeed) != 0;
            }
            if (SEQ) {
                seq_inl = valid && (sinf & kSeqGot) && (sinf & kSeqLevelMask) == kSeqInline;
                seq_dep = seq_inl && (sinf & kSeqDep);
                if (!seq_inl) r = 0;
            }
        }
    }

    // ---- the random gathers (level 2), issued together before the LDS
    // barrier: the first kBatchK pushers, t(x), and the first kBatchE pushers
    // of t(x) ahead of x.  Slots past k / r load x's own row (an L2 hit) so no
    // load is conditional.  Rarer deeper in-lists are walked afterwards.
    Cls q[kBatchK], e[kBatchE], qz = {0, 0, 0}, wz = {0, 0, 0};
    // 2P gather path: the id of pusher #kInline (the first tail entry) read
    // with the batch, so the walk below waits for its row only (a wave's 16
    // nodes at config 4 hold such a pusher with probability ~0.26)
    uint32_t tail0 = 0;
#pragma unroll
    for (uint32_t i = 0; i < kBatchK; ++i) q[i] = {0, 0, 0};
#pragma unroll
    for (uint32_t i = 0; i < kBatchE; ++i) e[i] = {0, 0, 0};
    if (DELIVER) {
        if (DLV) {
            // nothing to gather
        } else if (SHARD) {
            if (valid) {
                static_assert(kBatchK == 3, "shard rows: three batched pushers");
                const uint32_t e2 = a.IN2[x];
                const uint32_t sp = a.spos_cur[x];  // the slot of x's pull row (z's answer)
                // the first three pushers' rows together (unconditional:
                // row 0 stands in for a missing pusher)
                q[0] = L.load_push_row(a.recvA, in.z);
                q[1] = L.load_push_row(a.recvA, in.w);
                q[2] = L.load_push_row(a.recvA, e2);
                gz = !(tgw & kTgNoPull) && sp != 0xFFFFFFFFu;  // no slot: capacity overflow (flagged)
                if (gz) {
                    qz.c = a.recvB[L.row_index(sp, 2, 0)];
                    qz.a0 = a.recvB[L.row_index(sp, 2, 1)];
                    qz.a1 = 0;
                }
            }
        } else if (filt) {
            if (!SEQ && k > kInline) tail0 = a.src[in8.first()];
            // live-filtered: a row that cannot change any result (a pusher with
            // nothing live, a t(x) with nothing live and no live sibling ahead
            // of x to create from, a sibling that is not live or whose target
            // is complete) is not gathered; its place holds the empty row
            // (a skipped load is branched around, not redirected to an L2 hit:
            // with most rows skipped that measured 0.1-0.2 ms faster per launch)
#pragma unroll
            for (uint32_t i = 0; i < kBatchK; ++i) {
                gq[i] = i < k && !((qskip >> i) & 1u);
                if (gq[i]) q[i] = L.load_cls(S, in8.s[i]);
            }
            gz = valid && !(tgw & kTgNoPull) && (((zlw >> (x & 63u)) & 1ull) != 0 || zneed);
            if (gz) qz = L.load_cls(S, z);
#pragma unroll
            for (uint32_t i = 0; i < kBatchE; ++i) {
                ge[i] = i < r && !((eskip >> i) & 1u);
                if (ge[i]) e[i] = L.load_cls(S, sb8.e[i]);
            }
        } else {
            if (!SEQ && k > kInline) tail0 = a.src[in8.first()];
#pragma unroll
            for (uint32_t i = 0; i < kBatchK; ++i) q[i] = L.load_cls(S, i < k ? in8.s[i] : x);
            if (SEQ && !seq_inl) {  // W(x), coalesced (qz holds its code planes)
                if (valid && (sinf & kSeqGot)) {
                    const u64 wi = ((u64)x * 2u) * g.W + L.j;
                    qz.c = a.Wb[wi];
                    qz.a0 = a.Wb[wi + g.W];
                }
            } else {  // 2P, and SEQ nodes without a reader of W(x)
                qz = L.load_cls(S, z);
                if (SEQ && seq_dep) {  // W(z), built by z's pass (z < x has reader x)
                    const u64 wi = ((u64)z * 2u) * g.W + L.j;
                    const u64 b0 = a.Wb[wi], b1 = a.Wb[wi + g.W];
                    wz = Cls{b0 & b1, b0 & ~b1, b1 & ~b0};
                }
            }
            if (!SEQ || seq_inl) {
#pragma unroll
                for (uint32_t i = 0; i < kBatchE; ++i) e[i] = L.load_cls(S, i < r ? sb8.e[i] : x);
            }
        }
    }
    // ... and that pusher's row, issued as soon as the id is in (the batch's
    // rows, issued after it, stay in flight)
    Cls t0 = {0, 0, 0};
    if (GS_RK_TAILPRE && DELIVER && !SEQ && !DLV && !SHARD && k > kInline) t0 = L.load_cls(S, tail0);
    // likewise the row of t(x)'s pusher #kBatchE ahead of x (its id is inline)
    static_assert(kBatchE < kSibInline, "sibling #kBatchE is inline");
    Cls s2 = {0, 0, 0};
    if (GS_RK_TAILPRE && DELIVER && !SEQ && !DLV && !SHARD && r > kBatchE && !(tgw & kTgNoPull) &&
        (!filt || zneed) && !((eskip >> kBatchE) & 1u))
        s2 = L.load_cls(S, pick_sib(sb8.e, kBatchE));
    __builtin_amdgcn_s_setprio(0);
    {
        *reinterpret_cast<uint4 *>(&stage[s4]) = st0;
        *reinterpret_cast<uint4 *>(&stage[s4 + s4d]) = st1;
        *reinterpret_cast<uint4 *>(&stage[s4 + 2u * s4d]) = st2;
        *reinterpret_cast<uint4 *>(&stage[s4 + 3u * s4d]) = st3;
    }
    __syncthreads();
    u64 P[kPlanes];
    // the lane's plane 0 word in the stage (plane p: + p W; SMALL: its unit's)
    const uint32_t sb0 = sidx((uint32_t)(L.plane_index(0) - blk_base));
#pragma unroll
    for (int p = 0; p < kPlanes; ++p) {
        const u64 v = valid ? stage[sb0 + ((uint32_t)p << wlog)] : 0ull;
        P[p] = SMALL ? ((v >> L.sh) & L.m) : v;
    }

    // filtered: a skipped t(x) row stays the empty row it was initialised to;
    // skipped pushers and siblings are not absorbed at all (an empty row
    // changes nothing but |P|, which k counts)

    const u64 isC = P[0], a0 = P[1], a1 = P[2];
    const u64 A = ~isC & ~a0 & ~a1 & L.m;
    const u64 B = ~isC & (a0 | a1);
    const u64 C = isC & ~(a0 & a1);
    const u64 D = isC & a0 & a1;
    const u64 liveX = B | C;

    // ---- phases 1 and 2 of round t at x (Gossip::receive)
    // Faults: a node offline in round t (off_t) has no pushers and no pull; its
    // planes are the frozen pre-transition state of its last online round.  A
    // dropped pull batch (!pulled) is neither absorbed nor counted, so t(x)'s
    // own push copy, if any, stays recorded.
    const bool off_t = DELIVER && (tgw & kTgOff);
    const bool pulled = !(tgw & kTgNoPull);
    Recv<!TRANSITION> rv;
    rv.init(A, B, B & a0 & ~a1);
    uint32_t psize = 0;
    uint32_t ext_new = 0, ext_full = 0, ext_empty = 0, ext_recv = 0;  // external RPCs (node level)
    bool seq_gx = false, seq_skip = false;
    uint32_t seq_px = 0, seq_jz = kNone;
    if (DELIVER && valid && k > 30u) atomicOr(&a.flags[2], 1u);
    if (DELIVER && valid) {
        bool zin = false;
        u64 pv2, pvB, pCl;
        if (DLV) {
            static_assert(kDlvInline == 2, "inline pushers are read by hand");
            const uint32_t dzi = (dr.mf >> 5) & 31u;  // t(x)'s index among x's pushers
            const uint32_t dfirst = (x >> a.dlv_tlog) * a.dlv_tper + (dr.mf >> kDlvFirstShift);
            zin = dzi != kDlvNoZ;
            for (uint32_t i = 0; i < k; ++i) {
                const uint32_t code = i == 0 ? dr.c[0] : (i == 1 ? dr.c[1] : a.dtail[dfirst + i - kDlvInline]);
                rv.push(decode16(code), i, k, !(pulled && i == dzi));
            }
            // the pull batch z returned (built by the in-list build): code
            // (b0, b1) = 01 counter 1, 10 counter 2, 11 counter 255
            const u64 b0 = dpull & 0xFFFFu, b1 = dpull >> 16;
            pv2 = b1 & ~b0;
            pvB = b0 ^ b1;
            pCl = b0 & b1;
            if (!pulled) pv2 = pvB = pCl = 0;
        } else if (SHARD) {
            // zi = index of t(x) among x's pushers (0xFFFF: t(x) did not push to x)
            zin = zi != 0xFFFFu;
            const uint32_t zs = pulled ? zi : 0xFFFFu;  // push copy superseded by the pull copy
#pragma unroll
            for (uint32_t i = 0; i < kBatchK; ++i)
                if (i < k) rv.push(q[i], i, k, zs != i);
            for (uint32_t i = kBatchK; i < k; ++i) {
                rv.push(L.load_push_row(a.recvA, a.src[in.x + i]), i, k, zs != i);
            }
            // pull row code (b0, b1): 01 counter 1, 10 counter 2, 11 counter 255
            pv2 = qz.a0 & ~qz.c;
            pvB = qz.c ^ qz.a0;
            pCl = qz.c & qz.a0;
        } else if (SEQ) {
            // Events at x in time order: pushes from s < x, x's own pair (its
            // pull W(x), if it gets one), pushes from s > x.  x answers every
            // push except z's when x already heard from z (x < z, pulled);
            // of two copies from z the later one is recorded.
            const bool gx = (sinf & kSeqGot) != 0;
            uint32_t px = 0, jz = kNone;
            for (uint32_t i = 0; i < k; ++i) {
                const uint32_t s = i < kInline ? pick_inline(in8.s, i) : a.src[in8.first() + (i - kInline)];
                px += s < x ? 1u : 0u;
                if (s == z) jz = i;
            }
            zin = jz != kNone;
            if (seq_inl) {  // W(x) = S(z) + what z created before time x: from
                            // its pushers s < x and (dep) from W(z) at time z
                const u64 zB = ~qz.c & (qz.a0 | qz.a1);
                const u64 zC = qz.c & ~(qz.a0 & qz.a1);
                u64 pnot = ~qz.c & ~qz.a0 & ~qz.a1 & L.m, pB = 0, pC = 0;
                bool wdone = !seq_dep;
                auto put_w = [&](uint32_t s) {  // W(z) lands between z's pushers < z and > z
                    if (!wdone && s > z) {
                        sibling(wz, pnot, pB, pC);
                        wdone = true;
                    }
                };
#pragma unroll
                for (uint32_t i = 0; i < kBatchE; ++i)
                    if (i < r) {
                        put_w(sb8.e[i]);
                        sibling(e[i], pnot, pB, pC);
                    }
                if (r > kBatchE && (pnot || !wdone)) {
                    for (uint32_t i = kBatchE; i < min(r, kSibInline); ++i) {
                        const uint32_t s = pick_sib(sb8.e, i);
                        put_w(s);
                        sibling(L.load_cls(S, s), pnot, pB, pC);
                    }
                    if (r > kSibInline && (pnot || !wdone)) {
                        const InRec zin8 = a.IN8[z];
                        for (uint32_t i = kSibInline; i < r && (pnot || !wdone); ++i) {
                            const uint32_t s = i < kInline ? pick_inline(zin8.s, i)
                                                           : a.src[zin8.first() + (i - kInline)];
                            put_w(s);
                            sibling(L.load_cls(S, s), pnot, pB, pC);
                        }
                    }
                }
                if (!wdone) sibling(wz, pnot, pB, pC);
                const u64 pcl = zC | pC;  // the 2-plane code seq_pull_pass writes
                const u64 b0 = ((zB & qz.a0 & ~qz.a1) | pB | pcl) & L.m;
                const u64 b1 = ((zB & qz.a1 & ~qz.a0) | pcl) & L.m;
                qz = Cls{b0, b1, 0};
            }
            const bool skip = gx && zin && z > x;
            const uint32_t sk = skip ? 1u : 0u;
            // z's later push (z > x) overwrites the pull's records of the
            // rumors it carries (the pull may also carry entries z created)
            u64 precm = ~0ull;
            if (zin && z > x) {
                Cls qj = L.load_cls(S, z);
                const u64 vCj = qj.c & ~(qj.a0 & qj.a1);
                precm = ~((~qj.c & (qj.a0 | qj.a1)) | vCj);
            }
            pv2 = qz.a0 & ~qz.c;  // W(x) code (b0, b1) = (qz.c, qz.a0)
            pvB = qz.c ^ qz.a0;
            pCl = qz.c & qz.a0;
            bool pdone = !gx;
            for (uint32_t i = 0; i < k; ++i) {
                if (!pdone && i == px) {
                    rv.absorb(pvB, pv2, pCl, k - px - sk, px, precm);
                    pdone = true;
                }
                Cls qi;
                if (i < kBatchK) {
                    qi = q[0];
#pragma unroll
                    for (uint32_t b = 1; b < kBatchK; ++b) qi = (i == b) ? q[b] : qi;
                } else {
                    qi = L.load_cls(S, a.src[in8.first() + (i - kInline)]);
                }
                const uint32_t rafter = (k - 1u - i) - ((skip && jz > i) ? 1u : 0u);
                rv.absorb_cls(qi, rafter, i + ((gx && i >= px) ? 1u : 0u), !(i == jz && gx && z < x));
            }
            if (!pdone) rv.absorb(pvB, pv2, pCl, 0u, px, precm);
            seq_gx = gx;
            seq_px = px;
            seq_jz = jz;
            seq_skip = skip;
            pv2 = pvB = pCl = 0;  // absorbed above
        } else {
#pragma unroll
            for (uint32_t i = 0; i < kBatchK; ++i) {
                if (i < k) {
                    zin |= in8.s[i] == z;
                    if (!filt || gq[i]) rv.push(q[i], i, k, !(pulled && in8.s[i] == z));
                }
            }
            for (uint32_t i = kBatchK; i < k; ++i) {  // in-degree > kBatchK (1.9% of nodes)
                const uint32_t s = i < kInline ? pick_inline(in8.s, i)
                                               : (i == kInline ? tail0 : a.src[in8.first() + (i - kInline)]);
                zin |= s == z;
                rv.push((GS_RK_TAILPRE && i == kInline) ? t0 : L.load_cls(S, s), i, k, !(pulled && s == z));
            }
            // Pull batch from z: z's live set plus what z created from pushers
            // ahead of x.
            const u64 zB = ~qz.c & (qz.a0 | qz.a1);
            const u64 zC = qz.c & ~(qz.a0 & qz.a1);
            u64 pnot = ~qz.c & ~qz.a0 & ~qz.a1 & L.m, pB = 0, pC = 0;
#pragma unroll
            for (uint32_t i = 0; i < kBatchE; ++i)
                if (i < r && (!filt || ge[i])) sibling(e[i], pnot, pB, pC);
            // (filtered: no live sibling ahead of x, or t(x) complete -- nothing
            // deeper can be passed on either)
            if (r > kBatchE && pnot && pulled && (!filt || zneed)) {  // rank > kBatchE (rare)
                auto sib_row = [&](uint32_t s, bool skip) -> Cls {
                    if (skip) return Cls{0, 0, 0};
                    return L.load_cls(S, s);
                };
                for (uint32_t i = kBatchE; i < min(r, kSibInline); ++i) {
                    const bool sk = ((eskip >> i) & 1u) != 0;
                    Cls row;
                    if (GS_RK_TAILPRE && i == kBatchE) {
                        row = s2;
                    } else {
                        row = sib_row(pick_sib(sb8.e, i), sk);
                    }
                    sibling(row, pnot, pB, pC);
                }
                if (r > kSibInline && pnot) {  // rank > 3: 0.2% of nodes
                    InRec zin8 = a.IN8[z];
                    if (filt) zin8.kf &= kInFlagMask;  // (skip flags above the tail start)
                    for (uint32_t i = kSibInline; i < r && pnot; ++i) {
                        const uint32_t s = i < kInline ? pick_inline(zin8.s, i)
                                                       : a.src[zin8.first() + (i - kInline)];
                        sibling(sib_row(s, false), pnot, pB, pC);
                    }
                }
            }
            pv2 = zB & qz.a1 & ~qz.a0;
            pvB = zB | pB;  // counter 1 (created entries: 1) or 2
            pCl = zC | pC;
            if (!pulled) pv2 = pvB = pCl = 0;
        }
        const u64 pl = pvB | pCl;
        {
            const u64 newc = rv.notyet & pl;
            rv.record(rv.recB & pl, pvB, pv2, pCl);
            rv.create(newc, pCl);
        }
        rv.recv += popc(pl);
        if (a.n_ext) {
            // External RPCs to x (gs_handle_received), after every internal
            // delivery of the round, in call order (Gossip::receive,
            // src/gossip.rs:118-163): a first RPC from a peer joins
            // peers_in_this_round; a first Push is answered with x's live set
            // at that point; a copy creates an absent entry (new_from_peer, not
            // recorded) or is recorded on a B entry (the last copy per peer).
            uint32_t lo = 0, hi = a.n_ext;
            const u64 key = (u64)x << 32;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (a.ext[mid] < key) lo = mid + 1; else hi = mid;
            }
            for (uint32_t i = lo; i < a.n_ext && (uint32_t)(a.ext[i] >> 32) == x; ++i) {
                const uint32_t info = (uint32_t)a.ext[i];
                if (info & kExtNew) ++ext_new;
                if ((info & kExtPush) && (info & kExtNew)) {
                    uint32_t cnt = popc((B | C | rv.crB | rv.crC) & L.m);
                    if (!SMALL) cnt = group_sum(cnt, g.W);
                    if (cnt) ext_full += cnt; else ++ext_empty;
                }
                if (info & kExtEmpty) continue;
                ++ext_recv;
                const uint32_t r = info & 0xFFFu, c = (info >> 12) & 0xFFu;
                if ((SMALL ? 0u : (r >> 6)) != L.j) continue;
                const u64 bit = 1ull << (SMALL ? r : (r & 63u));
                // a counter >= counter_max acts as C (anyC); 0 creates B and votes "less"
                const u64 vC = c >= a.cmax ? bit : 0ull;
                const u64 vB = (c >= 1u && c < a.cmax) ? bit : 0ull;
                const u64 v2 = (c == 2u && c < a.cmax) ? bit : 0ull;
                const u64 newc = rv.notyet & bit;
                rv.record(rv.recB & bit & ((info & kExtRec) ? ~0ull : 0ull), vB, v2, vC);
                rv.create(newc, vC);
            }
        }
        const bool gets = SEQ ? seq_gx : pulled;
        psize = k + ((gets && !zin) ? 1u : 0u) + ext_new;  // |peers_in_this_round|
    }
    const u64 crB = rv.crB, crC = rv.crC, anyC = rv.anyC;

    // ---- node-level statistics of the deliveries
    uint32_t lc = popc(liveX);
    uint32_t part_cw = rv.part_cw, recv = rv.recv, first_create = rv.first_create;
    if (DELIVER && !SMALL) {
        lc = group_sum(lc, g.W);
        part_cw = group_sum(part_cw, g.W);
        recv = group_sum(recv, g.W);
        first_create = group_min(first_create, g.W);
    }
    uint32_t d_full_sent = 0, d_empty_pull = 0, d_recv = 0;
    if (DELIVER && SEQ) {
        // pull rows x sends: every answered push gets x's live set plus what x
        // created before it; empty ones until the first creating batch
        const uint32_t nresp = k - (seq_skip ? 1u : 0u);
        d_full_sent = nresp * lc + part_cw;
        if (nresp > 0 && lc == 0) {
            if (first_create == kNone) {
                d_empty_pull = nresp;
            } else {
                uint32_t c = (!seq_gx || first_create < seq_px) ? first_create + 1u : first_create;
                c = min(c, k);
                if (seq_skip && seq_jz + 1u <= first_create) c -= 1u;
                d_empty_pull = c;
            }
        }
        d_recv = recv;
    } else if (DELIVER) {
        d_full_sent = k * lc + part_cw;  // pull rows sent by x
        if (k > 0 && lc == 0) d_empty_pull = (first_create == kNone) ? k : first_create + 1u;
        d_recv = recv;
    }
    d_full_sent += ext_full;
    d_empty_pull += ext_empty;
    d_recv += ext_recv;
    const bool leader = valid && (SMALL || L.j == 0);

    if (!TRANSITION) {
        // ---------------- observation (post phase 2 of round t) -------------
        if (!valid) return;
        if (a.obs_only != 0xFFFFFFFFu || a.obs_list) {  // listed nodes' state codes only
            uint32_t slot = 0;
            if (a.obs_list) {  // (sorted: a binary search)
                uint32_t lo = 0, hi = a.n_obs;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (a.obs_list[mid] < x) lo = mid + 1; else hi = mid;
                }
                if (lo >= a.n_obs || a.obs_list[lo] != x) return;
                slot = lo;
            } else if (x != a.obs_only) {
                return;
            }
            uint16_t *os = a.obs_state + (u64)slot * g.R;
            const uint32_t nb = SMALL ? g.rpad : 64u;
            for (uint32_t b = 0; b < nb; ++b) {
                const uint32_t rr = SMALL ? b : L.j * 64u + b;
                if (rr >= g.R) break;
                const u64 bit = 1ull << b;
                uint32_t bf = 0;
#pragma unroll
                for (int i = 0; i < 5; ++i) bf |= (uint32_t)((P[3 + i] >> b) & 1u) << i;
                const uint32_t af = (uint32_t)((a0 >> b) & 1u) | ((uint32_t)((a1 >> b) & 1u) << 1);
                uint16_t code = 0;
                if (crB & bit) code = (uint16_t)((1u << 14) | (1u << 7));
                else if (crC & bit) code = (uint16_t)(2u << 14);
                else if (B & bit) code = (uint16_t)((1u << 14) | (af << 7) | bf);
                else if (C & bit) code = (uint16_t)((2u << 14) | (af << 7) | bf);
                else if (D & bit) code = (uint16_t)(3u << 14);
                os[rr] = code;
            }
            return;
        }
        const uint32_t KW = (g.R + 63u) >> 6;
        const u64 known = (~A | crB | crC) & L.m;
        if (a.obs_known && (SMALL || L.j < KW)) a.obs_known[(u64)x * KW + L.j] = known;
        if (leader) {
            if (a.obs_stats || a.obs_digest) {
                const uint4 d32 = load_stats(a.st32, a.st16, x);
                const u64 *b64 = a.st64 + (u64)x * 4;
                u64 o[5];
                o[0] = a.obs_rounds - (a.offc ? a.offc[x] : 0u);  // next_round calls
                if (a.emin) a.emin[x] = (uint8_t)min(d_empty_pull, 255u);  // slice: reduced by the caller
                o[1] = b64[0] + d32.x + (a.emin ? 0u : d_empty_pull);
                o[2] = b64[1] + d32.y;
                o[3] = b64[2] + d32.z + d_full_sent;
                o[4] = b64[3] + d32.w + d_recv;
                if (a.obs_stats)
                    for (int i = 0; i < 5; ++i) a.obs_stats[(u64)x * 5 + i] = o[i];
                if (a.obs_digest) a.obs_digest[x] = digest_node(psize, o);  // + the rumor terms below
            }
            if (a.obs_psize) a.obs_psize[x] = psize;
        }
        if (a.obs_dpart) {
            // rumor slice: this lane's word sum, split over the network words
            // it covers (its first rumor is the network's rumor dp_lo + 64 jw)
            const uint32_t jw = SMALL ? 0u : L.j;
            if (64u * jw < g.R) {
                u64 pl[20];
                digest_planes(L.m, B, C, D, crB, crC, a0, a1, &P[3], anyC, rv.c1, rv.c2, pl);
                const uint32_t gb = a.dp_lo + 64u * jw, gw = gb >> 6, sh = gb & 63u;
                u64 *dp = a.obs_dpart + (u64)x * a.dp_words;
                atomicAdd(&dp[gw], digest_sum(pl, sh));
                if (sh && gw + 1u < a.dp_words) {
                    for (int p = 0; p < 20; ++p) pl[p] >>= 64u - sh;
                    atomicAdd(&dp[gw + 1u], digest_sum(pl));
                }
            }
        }
        if (a.obs_digest) {
            // this lane's word (words past ceil(R/64) hold no rumor: no term);
            // the node's lanes add their terms (W adjacent lanes), the leader
            // wrote the node terms above
            const uint32_t jw = SMALL ? 0u : L.j;
            u64 dg = 64u * jw < g.R ? digest_word(jw, L.m, B, C, D, crB, crC, a0, a1, &P[3], anyC, rv.c1, rv.c2) : 0ull;
            if (!SMALL)
                for (uint32_t o = 1; o < g.W; o <<= 1) dg += __shfl_xor(dg, (int)o, 64);
            if (leader) a.obs_digest[x] += dg;
        }
        if (a.obs_state || a.obs_rec) {
            const uint32_t nb = SMALL ? g.rpad : 64u;
            for (uint32_t b = 0; b < nb; ++b) {
                const uint32_t rr = SMALL ? b : L.j * 64u + b;
                if (rr >= g.R) break;
                const u64 bit = 1ull << b;
                uint32_t bf = 0;
#pragma unroll
                for (int i = 0; i < 5; ++i) bf |= (uint32_t)((P[3 + i] >> b) & 1u) << i;
                const uint32_t af = (uint32_t)((a0 >> b) & 1u) | ((uint32_t)((a1 >> b) & 1u) << 1);
                uint16_t code = 0;
                if (crB & bit) code = (uint16_t)((1u << 14) | (1u << 7));
                else if (crC & bit) code = (uint16_t)(2u << 14);
                else if (B & bit) code = (uint16_t)((1u << 14) | (af << 7) | bf);
                else if (C & bit) code = (uint16_t)((2u << 14) | (af << 7) | bf);
                else if (D & bit) code = (uint16_t)(3u << 14);
                if (a.obs_state) a.obs_state[(u64)x * g.R + rr] = code;
                if (a.obs_rec) {
                    uint16_t rvv = 0;
                    if ((B | crB) & bit) {
                        uint32_t v1 = 0, v2 = 0;
#pragma unroll
                        for (int i = 0; i < 5; ++i) {
                            v1 |= (uint32_t)((rv.c1[i] >> b) & 1u) << i;
                            v2 |= (uint32_t)((rv.c2[i] >> b) & 1u) << i;
                        }
                        rvv = (uint16_t)((((anyC >> b) & 1u) << 15) | (v2 << 7) | v1);
                    }
                    a.obs_rec[(u64)x * g.R + rr] = rvv;
                }
            }
        }
        return;
    }

    // ---------------- phase 0 of round t+1 at x ----------------------------
    u64 N[kPlanes];
    u64 Bn = 0, Cn = 0;
    bool on_next = true;
    {
        // Gossip::new_message (insert = replace with MessageState::new, records
        // dropped) for the rumors injected at x this round.
        u64 inj = 0;
        if (a.n_inj && valid) inj = find_injection(a, SMALL ? (u64)x : seg) & L.m;
        // Churn: a node offline in round t+1 skips next_round (its votes go to
        // `pend`); a node returning from offline (off_t) takes them from there.
        on_next = !(a.f.churn && valid && offline_of(a.seed, a.epoch, a.round_new, a.node_lo + x, a.f.churn));
        const u64 pidx = ((u64)x * 2u) * g.W + L.j;
        const bool pending = off_t && valid;
        const u64 pb = pending ? a.pend[pidx] : 0ull, pa = pending ? a.pend[pidx + g.W] : 0ull;
        NextOut o;
        next_round_seg(P, rv, inj, psize, pending, pb, pa, on_next, a.cmax, a.maxc, a.maxr, o);
#pragma unroll
        for (int p = 0; p < kPlanes; ++p) N[p] = o.N[p];
        Bn = o.Bn;
        Cn = o.Cn;
        if (!on_next) {  // frozen: pre-transition planes + votes (the lane is valid)
            a.pend[pidx] = o.bump;
            a.pend[pidx + g.W] = o.anyC;
        }
    }

    // DLV: the push code of round t+1 (b0 | b1 << 16), which the in-list
    // build carries to the receivers (coalesced, 4 B per node)
    if (DLV && valid) {
        const u64 vC = N[0] & ~(N[1] & N[2]), vB = ~N[0] & (N[1] | N[2]);
        const u64 b0 = ((vB & N[1] & ~N[2]) | vC) & L.m, b1 = ((vB & N[2] & ~N[1]) | vC) & L.m;
        a.pc_out[x] = (uint32_t)b0 | ((uint32_t)b1 << 16);
        if (a.kn_out) a.kn_out[x] = (uint16_t)((N[0] | N[1] | N[2]) & L.m);
    }

    // ---- live-filtered gathers: node maps of the round-(t+1) planes, "live"
    // (its push row is not empty) and "complete" (no A entry), for the next
    // in-list build; one ballot per wave (W <= 8: a wave's nodes are whole bytes)
    if (TRANSITION && a.lvm) {
        // live = B | C entries, A = no entry; from the transition's Bn / Cn
        // (N[0] = C | D), or from the stored planes of a frozen offline node
        u64 lvw, aw;
        if (a.f.churn == 0u) {
            lvw = Bn | Cn;
            aw = ~(N[0] | Bn) & L.m;
        } else {
            lvw = ((N[0] & ~(N[1] & N[2])) | (~N[0] & (N[1] | N[2]))) & L.m;
            aw = ~N[0] & ~N[1] & ~N[2] & L.m;
        }
        const u64 bl = __ballot(valid && lvw != 0);
        const u64 bc = __ballot(valid && aw == 0);
        const uint32_t lane = threadIdx.x & 63u;
        const u64 seg0 = seg - lane;
        if (lane == 0 && seg0 < g.nseg) {
            if (SMALL) {  // a lane per node: the wave's 64 nodes are one map word
                a.lvm[seg0 >> 6] = bl;
                a.cpm[seg0 >> 6] = bc;
            } else {
                const uint32_t lw = g.logr - 6u;
                const u64 cl = compress_stride(group_or_bits(bl, lw), lw);
                const u64 cc = compress_stride(group_and_bits(bc, lw), lw);
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
        }
        // traffic accounting of timed launches: the class rows this round's
        // build left to gather (counted there, off the kernel's path)
        if (MODE == 1 && a.acct && a.rows_cnt && bid == 0 && threadIdx.x == 0) atomicAdd(a.acct, *a.rows_cnt);
    }

    // ---- write round-(t+1) planes (through LDS, 16-byte coalesced stores)
    uint32_t live_new = (valid && on_next) ? popc(Bn | Cn) : 0u;
    if (!SMALL) live_new = group_sum(live_new, g.W);
    if (__ballot(live_new != 0u) != 0ull && (threadIdx.x & 63u) == 0u) blk_any = 1u;
    constexpr bool kZBlk = GS_RK_ZSKIP_BLK && TRANSITION && kBlk != 64u;
    const u64 nz_mask = SMALL ? L.m : ~0ull;
    if (kZBlk && __ballot(valid && ((N[0] | N[1] | N[2]) & nz_mask) != 0ull) != 0ull && (threadIdx.x & 63u) == 0u)
        blk_nz = 1u;
    __syncthreads();  // also: every lane is done reading stage
    const bool blk_live = blk_any != 0u;
    __builtin_amdgcn_s_setprio(1);  // the drain: retire the block, free its slot
    // A wave (= block) whose nodes are all-A in round t+1 were all-A in
    // round t-1 as well (no entry ever returns to A; clear zeroes both
    // buffers), and Snext holds round t-1: its zero planes are there already.
    // (a 256-lane block: the same over its four waves, from blk_nz)
    const bool zskip = kZBlk ? blk_nz == 0u
                             : GS_RK_ZSKIP && kBlk == 64u && __ballot(valid && (N[0] | N[1] | N[2]) != 0ull) == 0ull;
    if (zskip) {
        // nothing to store
    } else if (SMALL) {
        const uint32_t npu = 1u << g.lognpu;
#pragma unroll
        for (int p = 0; p < kPlanes; ++p) {
            u64 v = valid ? ((N[p] & L.m) << L.sh) : 0ull;
            for (uint32_t o = 1; o < npu; o <<= 1) v |= __shfl_xor(v, (int)o, 64);
            if (valid && (x & (npu - 1u)) == 0) stage[sidx((uint32_t)(L.plane_index(p) - blk_base))] = v;
        }
    } else if (valid) {
#pragma unroll
        for (int p = 0; p < kPlanes; ++p) stage[sb0 + ((uint32_t)p << wlog)] = N[p];
    }
    if (!zskip) __syncthreads();  // (zskip is uniform over the block)
    if (!zskip) {
        uint4 *dst4 = reinterpret_cast<uint4 *>(a.Snext + blk_base);
        // streaming (nontemporal) stores: 3.11 -> 3.01 ms per round kernel at
        // config 4 (nontemporal plane loads measured slower: 3.27 ms).
        for (uint32_t i = threadIdx.x, si = s4; i < blk_v4; i += blockDim.x, si += s4d)
            nt_store4(*reinterpret_cast<const uint4 *>(&stage[si]), &dst4[i]);
    }
    if (SHARD) {
        // push row of round t+1: the push batch's class code, to owner(t_{t+1}(x))
        // (no slot: an undelivered edge, or a capacity overflow, flagged)
        const uint32_t sp = valid ? a.spos_next[x] : 0xFFFFFFFFu;
        const u64 vC = N[0] & ~(N[1] & N[2]), vB = ~N[0] & (N[1] | N[2]);
        const u64 c0 = ((vB & N[1] & ~N[2]) | vC) & L.m;  // code bit 0
        const u64 c1 = ((vB & N[2] & ~N[1]) | vC) & L.m;  // code bit 1
        if (sp != 0xFFFFFFFFu) {
            a.sendA[L.row_index(sp, 2, 0)] = c0;
            a.sendA[L.row_index(sp, 2, 1)] = c1;
        }
    }

    // ---- push list + Statistics (src/gossip.rs:80,103-111)
    mark_any_live(a.live, a.round_new, bid, blk_live);
    if (leader) {
        // rounds is the engine's round count (every node runs every round);
        // the other four are u32 deltas folded into u64 before they can wrap.
        uint4 v = stv;
        if (a.st16 && (ext_full | ext_empty | ext_recv)) {
            // u16 deltas hold internal deliveries only (bounded per round):
            // external RPCs, as many as the caller sends, go to the totals --
            // but a rumor slice's empty pulls go through emin (MIN over the
            // slices; the engine bounds them, gs_engine.cpp slice_ext_limit)
            u64 *s64 = const_cast<u64 *>(a.st64) + (u64)x * 4u;
            if (!a.emin) {
                s64[0] += ext_empty;
                d_empty_pull -= ext_empty;
            }
            s64[2] += ext_full;
            s64[3] += ext_recv;
            d_full_sent -= ext_full;
            d_recv -= ext_recv;
        }
        const uint32_t d_empty_push = (on_next && live_new == 0u) ? 1u : 0u;
        if (a.emin) {  // rumor slice: empty only if empty in every slice (MIN per byte, caller)
            reinterpret_cast<uint16_t *>(a.emin)[x] = (uint16_t)(min(d_empty_pull, 255u) | (d_empty_push << 8));
            v.x += eadd & 0xFFu;  // an earlier round's network counts (reduced by the caller)
            v.y += eadd >> 8;
        } else {
            v.x += d_empty_pull;                   // empty_pull_sent
            v.y += d_empty_push;                   // empty_push_sent
        }
        v.z += live_new + d_full_sent;             // full_message_sent
        v.w += d_recv;                             // full_message_received
        store_stats(a.st32, a.st16, x, v);
        if (!on_next) atomicAdd(&a.offc[x], 1u);  // (no return: nothing waits for it)
    }
}

template <bool SMALL, bool SHARD, bool SEQ, bool DLV = false>
static hipError_t launch_mode(const RoundArgs &a, int mode, hipStream_t s) {
    if constexpr (!SMALL && !SEQ && !DLV) {
        if ((mode == 0 || mode == 1) && a.g.W <= 16u) {
            if (a.blk_list) return hipErrorInvalidValue;  // (observation launches only)
            // a part's 256-lane blocks [blk_off, blk_off + blk_count) as
            // 128-lane blocks, none past the last segment (a block wholly
            // past it would compute a stage range below zero)
            constexpr u64 f = 256u / kRkSmallBlk;
            const u64 nblk = (a.g.nseg + kRkSmallBlk - 1) / kRkSmallBlk;
            const u64 b0 = std::min<u64>((u64)a.blk_off * f, nblk);
            const u64 b1 = a.blk_count ? std::min<u64>(((u64)a.blk_off + a.blk_count) * f, nblk) : nblk;
            if (b1 <= b0) return hipSuccess;
            RoundArgs b = a;
            b.blk_off = (uint32_t)b0;
            if (mode == 0)
                hipLaunchKernelGGL((round_kernel<false, 0, SHARD, false, false, kRkSmallBlk>), dim3((uint32_t)(b1 - b0)),
                                   dim3(kRkSmallBlk), 0, s, b);
            else
                hipLaunchKernelGGL((round_kernel<false, 1, SHARD, false, false, kRkSmallBlk>), dim3((uint32_t)(b1 - b0)),
                                   dim3(kRkSmallBlk), 0, s, b);
            return hipGetLastError();
        }
    }
    const uint32_t block = 256;
    const u64 grid = a.blk_count ? a.blk_count : (a.g.nseg + block - 1) / block;
    if (grid == 0) return hipSuccess;
    if (a.blk_list && (mode == 0 || mode == 1)) return hipErrorInvalidValue;  // (observation launches only)
    switch (mode) {
    case 0: hipLaunchKernelGGL((round_kernel<SMALL, 0, SHARD, SEQ, DLV>), dim3((uint32_t)grid), dim3(block), 0, s, a); break;
    case 1: hipLaunchKernelGGL((round_kernel<SMALL, 1, SHARD, SEQ, DLV>), dim3((uint32_t)grid), dim3(block), 0, s, a); break;
    case 2: hipLaunchKernelGGL((round_kernel<SMALL, 2, SHARD, SEQ, DLV>), dim3((uint32_t)grid), dim3(block), 0, s, a); break;
    default: hipLaunchKernelGGL((round_kernel<SMALL, 3, SHARD, SEQ, DLV>), dim3((uint32_t)grid), dim3(block), 0, s, a); break;
    }
    return hipGetLastError();
}

hipError_t launch_round(const RoundArgs &a, int mode, hipStream_t s) {
    if (a.recvA) {  // shard engine (2P only)
        // code rows: the packed DLV round kernel for transitions; observers
        // read the unpacked pull codes on the DLV path (gs_engine.cpp observe)
        if (a.sp.codes) return (mode == 0 || mode == 1) ? launch_round_dlv4(a, mode, s) : hipErrorInvalidValue;
        return a.g.small ? launch_mode<true, true, false>(a, mode, s) : launch_mode<false, true, false>(a, mode, s);
    }
    if (a.Wb)     // SEQ schedule
        return a.g.small ? launch_mode<true, false, true>(a, mode, s) : launch_mode<false, false, true>(a, mode, s);
    if (a.DR) {   // delivery records (2P, R_pad <= 16)
        if (!a.g.small || a.g.rpad > 16) return hipErrorInvalidValue;
        if (a.dlv_pack && (mode == 0 || mode == 1)) return launch_round_dlv4(a, mode, s);
        return launch_mode<true, false, false, true>(a, mode, s);
    }
    if (w32_eligible(a, mode)) return launch_round_w32(a, mode, s);                   // gs_w32.hip
    return a.g.small ? launch_mode<true, false, false>(a, mode, s) : launch_mode<false, false, false>(a, mode, s);
}

// Rumor slices: add a round's empty-RPC counts, reduced with MIN over the
// slices by the caller (gs_slice_apply), to the u32 Statistics deltas.
__global__ __launch_bounds__(256) void slice_apply(uint32_t *st32, const uint8_t *__restrict__ emin, uint32_t n,
                                                   uint32_t st16) {
    const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= n) return;
    uint4 v = load_stats(st32, st16, x);
    v.x += emin[2u * (u64)x];       // empty_pull_sent
    v.y += emin[2u * (u64)x + 1u];  // empty_push_sent
    store_stats(st32, st16, x, v);
}

hipError_t launch_slice_apply(uint32_t *st32, const uint8_t *emin, uint32_t n, uint32_t st16, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(slice_apply, dim3((n + 255u) / 256u), dim3(256), 0, s, st32, emin, n, st16);
    return hipGetLastError();
}

// Fold the u32 (u16: st16) statistics deltas into the u64 totals (before they can wrap).
__global__ __launch_bounds__(256) void stats_fold(uint32_t *st32, u64 *st64, u64 words, uint32_t st16) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= words) return;
    if (st16) {
        uint16_t *s16 = reinterpret_cast<uint16_t *>(st32);
        st64[i] += s16[i];
        s16[i] = 0;
    } else {
        st64[i] += st32[i];
        st32[i] = 0u;
    }
}

hipError_t launch_stats_fold(uint32_t *st32, u64 *st64, uint32_t n, uint32_t st16, hipStream_t s) {
    const u64 words = (u64)n * 4;
    if (words == 0) return hipSuccess;
    hipLaunchKernelGGL(stats_fold, dim3((uint32_t)((words + 255) / 256)), dim3(256), 0, s, st32, st64,
                       words, st16);
    return hipGetLastError();
}

// ------------------------------------------------------------ reductions
__global__ __launch_bounds__(256) void known_reduce(const u64 *__restrict__ known, uint32_t n,
                                                    uint32_t KW, uint32_t min_known, u64 *partials) {
    __shared__ u64 s_tot[256], s_cmp[256];
    u64 tot = 0, cmp = 0;
    for (u64 x = (u64)blockIdx.x * blockDim.x + threadIdx.x; x < n; x += (u64)gridDim.x * blockDim.x) {
        uint32_t c = 0;
        for (uint32_t w = 0; w < KW; ++w) c += popc(known[x * KW + w]);
        tot += c;
        cmp += (c >= min_known) ? 1u : 0u;
    }
    s_tot[threadIdx.x] = tot;
    s_cmp[threadIdx.x] = cmp;
    __syncthreads();
    for (uint32_t o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            s_tot[threadIdx.x] += s_tot[threadIdx.x + o];
            s_cmp[threadIdx.x] += s_cmp[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        partials[2 * blockIdx.x] = s_tot[0];
        partials[2 * blockIdx.x + 1] = s_cmp[0];
    }
}

hipError_t launch_known_reduce(const u64 *known, uint32_t n, uint32_t KW, uint32_t min_known,
                               u64 *partials, uint32_t blocks, hipStream_t s) {
    hipLaunchKernelGGL(known_reduce, dim3(blocks), dim3(256), 0, s, known, n, KW, min_known, partials);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void known_popc(const u64 *__restrict__ known, uint32_t n, uint32_t KW,
                                                  uint32_t *counts) {
    const u64 x = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= n) return;
    uint32_t c = 0;
    for (uint32_t w = 0; w < KW; ++w) c += popc(known[x * KW + w]);
    counts[x] = c;
}

hipError_t launch_known_popc(const u64 *known, uint32_t n, uint32_t KW, uint32_t *counts, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(known_popc, dim3((n + 255) / 256), dim3(256), 0, s, known, n, KW, counts);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void obs_pending(const u64 *__restrict__ pairs, uint32_t m, uint32_t R,
                                                   u64 *known, uint16_t *state, uint16_t *rec) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint32_t x = (uint32_t)(pairs[i] >> 32), r = (uint32_t)pairs[i];
    const uint32_t KW = (R + 63u) >> 6;
    atomicOr(&known[(u64)x * KW + (r >> 6)], 1ull << (r & 63u));
    if (state) state[(u64)x * R + r] = (uint16_t)((1u << 14) | (1u << 7));  // B{round 0, counter 1}
    if (rec) rec[(u64)x * R + r] = 0;
}

hipError_t launch_obs_pending(const u64 *pairs, uint32_t m, uint32_t R, u64 *known, uint16_t *state,
                              uint16_t *rec, hipStream_t s) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(obs_pending, dim3((m + 255) / 256), dim3(256), 0, s, pairs, m, R, known, state, rec);
    return hipGetLastError();
}

// Digests of a sliced network from the summed word parts (gs_digest_finish).
__global__ __launch_bounds__(256) void digest_finish(const u64 *__restrict__ dpart, uint32_t n, uint32_t words,
                                                     const uint32_t *__restrict__ psize, const u64 *__restrict__ stats,
                                                     u64 *out) {
    const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= n) return;
    u64 st[5];
    for (int i = 0; i < 5; ++i) st[i] = stats[(u64)x * 5 + i];
    u64 h = digest_node(psize[x], st);
    for (uint32_t j = 0; j < words; ++j) h += digest_fin(j, dpart[(u64)x * words + j]);
    out[x] = h;
}

hipError_t launch_digest_finish(const u64 *dpart, uint32_t n, uint32_t words, const uint32_t *psize,
                                const u64 *stats, u64 *out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(digest_finish, dim3((n + 255u) / 256u), dim3(256), 0, s, dpart, n, words, psize, stats, out);
    return hipGetLastError();
}

// Statistics::add / min / max over [n][5] observed statistics.
__global__ __launch_bounds__(256) void stats_reduce(const u64 *__restrict__ st, uint32_t n, int op,
                                                    u64 *partials) {
    __shared__ u64 sm[5][256];
    u64 acc[5];
    for (int f = 0; f < 5; ++f) acc[f] = (op == 1) ? ~0ull : 0ull;
    for (u64 x = (u64)blockIdx.x * blockDim.x + threadIdx.x; x < n; x += (u64)gridDim.x * blockDim.x) {
        for (int f = 0; f < 5; ++f) {
            const u64 v = st[x * 5 + f];
            acc[f] = op == 0 ? acc[f] + v : (op == 1 ? min(acc[f], v) : max(acc[f], v));
        }
    }
    for (int f = 0; f < 5; ++f) sm[f][threadIdx.x] = acc[f];
    __syncthreads();
    for (uint32_t o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            for (int f = 0; f < 5; ++f) {
                const u64 u = sm[f][threadIdx.x], v = sm[f][threadIdx.x + o];
                sm[f][threadIdx.x] = op == 0 ? u + v : (op == 1 ? min(u, v) : max(u, v));
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0)
        for (int f = 0; f < 5; ++f) partials[5 * blockIdx.x + f] = sm[f][0];
}

hipError_t launch_stats_reduce(const u64 *stats, uint32_t n, int op, u64 *partials,
                               uint32_t blocks, hipStream_t s) {
    hipLaunchKernelGGL(stats_reduce, dim3(blocks), dim3(256), 0, s, stats, n, op, partials);
    return hipGetLastError();
}

}  // namespace gs
