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

namespace gs {


// Receiver-side state of phases 1-2 at x for one segment.  The transition
// path keeps one bit-sliced counter of the recorded counters that vote ">= own"
// (MessageState::next_round's greater_or_equal, src/message_state.rs:118-129);
// the observation path (OBS) keeps the two counters the parity dumps report.
template <bool OBS>
struct Recv {
    u64 notyet;          // still absent: the next live copy creates the entry
    u64 recB;            // entries in state B (existing or created): record copies
    u64 oc1;             // B entries whose our_counter is 1 (created ones included)
    u64 crB, crC;        // created this round as B{0,1} / C{0,0}
    u64 anyC;            // a recorded counter >= counter_max
    u64 cv[5];           // #recorded counters >= our_counter (and < counter_max)
    u64 c1[5];           // OBS only: #recorded counters in [1, counter_max)
    u64 c2[5];           // OBS only: #recorded counters == 2 (< counter_max)
    uint32_t part_cw;    // sum over pushers i of (k-1-i) * |created by i|
    uint32_t first_create;
    uint32_t recv;       // copies received (push rows + pull row)

    GS_DEV void init(u64 A, u64 B, u64 Boc1) {
        notyet = A;
        recB = B;
        oc1 = Boc1;
        crB = crC = anyC = 0;
#pragma unroll
        for (int i = 0; i < 5; ++i) cv[i] = 0;
        if constexpr (OBS) {
#pragma unroll
            for (int i = 0; i < 5; ++i) c1[i] = c2[i] = 0;
        }
        part_cw = 0;
        first_create = kNone;
        recv = 0;
    }
    // Record copies `rec` of class (vB: a B counter, v2: counter 2, vC: 255).
    GS_DEV void record(u64 rec, u64 vB, u64 v2, u64 vC) {
        anyC |= rec & vC;
        add5(cv, rec & vB & (v2 | oc1));
        if constexpr (OBS) {
            add5(c1, rec & vB);
            add5(c2, rec & v2);
        }
    }
    GS_DEV void create(u64 newc, u64 vC) {
        crB |= newc & ~vC;
        crC |= newc & vC;
        recB |= newc & ~vC;
        oc1 |= newc & ~vC;
        notyet &= ~newc;
    }
    // One push batch from pusher i of k (Gossip::receive, src/gossip.rs:153-163);
    // `rec_on` is false for t(x)'s own push, superseded by its pull copy.
    GS_DEV void push(const Cls &q, uint32_t i, uint32_t k, bool rec_on) {
        const u64 vC = q.c & ~(q.a0 & q.a1);   // C: counter 255
        const u64 vB = ~q.c & (q.a0 | q.a1);   // B: counter = our_counter
        const u64 v2 = vB & q.a1 & ~q.a0;      // B with our_counter 2
        const u64 sl = vB | vC;                // the push batch
        const u64 newc = notyet & sl;          // new_from_peer: not recorded
        if (rec_on) record(recB & sl, vB, v2, vC);  // MessageState::receive on B
        create(newc, vC);
        const uint32_t pc = popc(newc);
        part_cw += (k - 1u - i) * pc;  // later pushers' pull rows include it
        if (pc && first_create == kNone) first_create = i;
        recv += popc(sl);
    }
};

#ifndef GS_RK_MINW
#define GS_RK_MINW 1
#endif

// MODE: 0 transition only (first round), 1 deliver round t + transition to
// t+1, 2 deliver round t + observe, 3 observe only.
// SHARD: this engine owns a node range of a sharded network; pusher class rows
// and the pull row come from the exchange buffers (recvA, recvB) instead of
// gathers, and the new class planes are also written as push rows (sendA).
template <bool SMALL, int MODE, bool SHARD>
__global__ __launch_bounds__(256, GS_RK_MINW) void round_kernel(RoundArgs a) {
    constexpr bool DELIVER = (MODE == 1 || MODE == 2);
    constexpr bool TRANSITION = (MODE == 0 || MODE == 1);
    const Geometry &g = a.g;
    const u64 seg = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = seg < g.nseg;
    Lane<SMALL> L;
    L.init(g, valid ? seg : 0);
    const uint32_t x = L.x;
    const u64 *__restrict__ S = a.Scur;

    // ---- coalesced per-node metadata and own round-t planes
    uint4 in = {0, 0, 0, 0}, sb = {0, 0, 0, 0};
    uint32_t z = 0, zi = 0xFFFFu;
    if (DELIVER && valid) {
        in = a.IN[x];   // {first edge, k, s0, s1}  (SHARD: {first, k|zi<<16, e0, e1})
        if (SHARD) {
            zi = in.y >> 16;
            in.y &= 0xFFFFu;
        } else {
            sb = a.SIB[x];  // {serial, rank of x in in(z), e0, e1}; stale unless rank >= 1
            z = a.tg[x];    // t_t(x)
        }
    }
    u64 P[kPlanes];
#pragma unroll
    for (int p = 0; p < kPlanes; ++p) {
        u64 v = valid ? S[L.plane_index(p)] : 0ull;
        P[p] = SMALL ? ((v >> L.sh) & L.m) : v;
    }

    // ---- the random gathers, all issued together
    uint32_t k = 0, r = 0;
    Cls q0 = {0, 0, 0}, q1 = {0, 0, 0}, qz = {0, 0, 0}, e0 = {0, 0, 0}, e1 = {0, 0, 0};
    if (DELIVER && valid) {
        k = in.y;
        r = sb.x == a.serial ? sb.y : 0u;
#ifdef GS_EXP_NO_PUSHERS
        k = 0;
#endif
#ifdef GS_EXP_NO_ZPUSHERS
        r = 0;
#endif
        if (SHARD) {
            if (k > 0) q0 = L.load_row3(a.recvA, in.z);
            if (k > 1) q1 = L.load_row3(a.recvA, in.w);
            const uint32_t sp = a.spos_cur[x];  // the pull row z returned to x
            qz.c = a.recvB[L.row_index(sp, 2, 0)];
            qz.a0 = a.recvB[L.row_index(sp, 2, 1)];
            qz.a1 = 0;
        } else {
            if (k > 0) q0 = L.load_cls(S, in.z);
            if (k > 1) q1 = L.load_cls(S, in.w);
            qz = L.load_cls(S, z);
            if (r > 0) e0 = L.load_cls(S, sb.z);
            if (r > 1) e1 = L.load_cls(S, sb.w);
        }
    }

    const u64 isC = P[0], a0 = P[1], a1 = P[2];
    const u64 A = ~isC & ~a0 & ~a1 & L.m;
    const u64 B = ~isC & (a0 | a1);
    const u64 C = isC & ~(a0 & a1);
    const u64 D = isC & a0 & a1;
    const u64 liveX = B | C;

    // ---- phases 1 and 2 of round t at x (Gossip::receive)
    Recv<!TRANSITION> rv;
    rv.init(A, B, B & a0 & ~a1);
    uint32_t psize = 0;
    if (DELIVER && valid) {
        if (k > 30u) atomicOr(&a.flags[2], 1u);
        bool zin = false;
        u64 pv2, pvB, pCl;
        if (SHARD) {
            // zi = index of t(x) among x's pushers (0xFFFF: t(x) did not push to x)
            zin = zi != 0xFFFFu;
            if (k > 0) rv.push(q0, 0, k, zi != 0);
            if (k > 1) rv.push(q1, 1, k, zi != 1);
            for (uint32_t i = 2; i < k; ++i) rv.push(L.load_row3(a.recvA, a.src[in.x + i]), i, k, zi != i);
            // pull row code (b0, b1): 01 counter 1, 10 counter 2, 11 counter 255
            pv2 = qz.a0 & ~qz.c;
            pvB = qz.c ^ qz.a0;
            pCl = qz.c & qz.a0;
        } else {
            if (k > 0) {
                zin |= in.z == z;
                rv.push(q0, 0, k, in.z != z);
            }
            if (k > 1) {
                zin |= in.w == z;
                rv.push(q1, 1, k, in.w != z);
            }
            for (uint32_t i = 2; i < k; ++i) {  // in-degree >= 3 (8% of nodes)
                const uint32_t s = a.src[in.x + i];
                zin |= s == z;
                rv.push(L.load_cls(S, s), i, k, s != z);
            }
            // Pull batch from z: z's live set plus what z created from pushers
            // ahead of x.
            const u64 zB = ~qz.c & (qz.a0 | qz.a1);
            const u64 zC = qz.c & ~(qz.a0 & qz.a1);
            u64 pnot = ~qz.c & ~qz.a0 & ~qz.a1 & L.m, pB = 0, pC = 0;
            if (r > 0) sibling(e0, pnot, pB, pC);
            if (r > 1) sibling(e1, pnot, pB, pC);
            if (r > 2 && pnot) {
                const uint32_t zb = a.IN[z].x;  // rare: rank >= 3
                for (uint32_t i = 2; i < r && pnot; ++i) sibling(L.load_cls(S, a.src[zb + i]), pnot, pB, pC);
            }
            pv2 = zB & qz.a1 & ~qz.a0;
            pvB = zB | pB;  // counter 1 (created entries: 1) or 2
            pCl = zC | pC;
        }
        const u64 pl = pvB | pCl;
        {
            const u64 newc = rv.notyet & pl;
            rv.record(rv.recB & pl, pvB, pv2, pCl);
            rv.create(newc, pCl);
        }
        rv.recv += popc(pl);
        psize = k + (zin ? 0u : 1u);  // |peers_in_this_round|
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
    if (DELIVER) {
        d_full_sent = k * lc + part_cw;  // pull rows sent by x
        if (k > 0 && lc == 0) d_empty_pull = (first_create == kNone) ? k : first_create + 1u;
        d_recv = recv;
    }
    const bool leader = valid && (SMALL || L.j == 0);

    if (!TRANSITION) {
        // ---------------- observation (post phase 2 of round t) -------------
        if (!valid) return;
        const uint32_t KW = (g.R + 63u) >> 6;
        const u64 known = (~A | crB | crC) & L.m;
        if (a.obs_known && (SMALL || L.j < KW)) a.obs_known[(u64)x * KW + L.j] = known;
        if (leader) {
            if (a.obs_stats) {
                const uint4 d32 = reinterpret_cast<const uint4 *>(a.st32)[x];
                const u64 *b64 = a.st64 + (u64)x * 4;
                u64 *o = a.obs_stats + (u64)x * 5;
                o[0] = a.obs_rounds;
                o[1] = b64[0] + d32.x + d_empty_pull;
                o[2] = b64[1] + d32.y;
                o[3] = b64[2] + d32.z + d_full_sent;
                o[4] = b64[3] + d32.w + d_recv;
            }
            if (a.obs_psize) a.obs_psize[x] = psize;
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
    // Gossip::new_message (insert = replace with MessageState::new, records
    // dropped) for the rumors injected at x this round.
    u64 inj = 0;
    if (a.n_inj && valid) {
        const u64 key = SMALL ? (u64)x : seg;
        uint32_t lo = 0, hi = a.n_inj;
        while (lo < hi) {
            uint32_t mid = (lo + hi) >> 1;
            if (a.inj_key[mid] < key) lo = mid + 1; else hi = mid;
        }
        if (lo < a.n_inj && a.inj_key[lo] == key) inj = a.inj_mask[lo] & L.m;
    }
    const u64 ninj = ~inj;
    const u64 Bold = B & ninj, Cold = C & ninj, Dold = D & ninj;
    const u64 cB = crB & ninj, cC = crC & ninj;
    const u64 Bf = Bold | cB | inj;  // entries in state B entering next_round
    const u64 Cf = Cold | cC;        // entries in state C entering next_round

    // B (src/message_state.rs:94-147).  0-filled peers vote "less", so with
    // no C copy the median rule is: bump iff 2*ge > |P| iff ge >= |P|/2+1.
    const u64 oc1 = (Bold & a0 & ~a1) | cB | inj;
    const u64 oc2 = Bold & a1 & ~a0;
    const uint32_t thr = psize / 2u + 1u;
    const u64 bump = ge_k<5>(rv.cv, thr) & (Bold | cB);  // cv counts only B entries' votes
    const u64 anyCe = anyC & ninj;
    u64 nr[6];  // round + 1
    {
        u64 carry = ~0ull;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const u64 rb = P[3 + i] & Bold;
            nr[i] = rb ^ carry;
            carry &= rb;
        }
        nr[5] = carry;
    }
    const u64 toD = ge_u<6>(nr, a.maxr);
    const u64 oc1n = oc1 & ~bump;
    const u64 oc2n = (oc1 & bump) | (oc2 & ~bump);
    const u64 oc3n = oc2 & bump;
    const u64 ocge = a.cmax <= 1u ? ~0ull : (a.cmax == 2u ? (oc2n | oc3n) : oc3n);
    const u64 toC = anyCe | ocge;
    const u64 BD = Bf & toD, BC = Bf & ~toD & toC, BB = Bf & ~toD & ~toC;

    // C (src/message_state.rs:148-168): round+1; D if round+rib >= max_rounds
    // or round >= max_c_rounds.
    const u64 cr0 = a0 & Cold, cr1 = a1 & Cold;
    const u64 d[3] = {~cr0, cr1 ^ cr0, cr1 & cr0};
    u64 rib[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) rib[i] = P[3 + i] & Cold;
    u64 sum[6];
    {
        u64 c = 0;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const u64 di = i < 3 ? d[i] : 0ull;
            sum[i] = rib[i] ^ di ^ c;
            c = (rib[i] & di) | (c & (rib[i] ^ di));
        }
        sum[5] = c;
    }
    const u64 CtoD = ge_u<6>(sum, a.maxr) | ge_u<3>(d, a.maxc);
    const u64 CD = Cf & CtoD, CC = Cf & ~CtoD;

    const u64 Dn = BD | CD | Dold;
    const u64 Cn = BC | CC;
    const u64 Bn = BB;
    u64 N[kPlanes];
    N[0] = Cn | Dn;
    N[1] = (Bn & oc1n) | (CC & d[0]) | Dn;
    N[2] = (Bn & oc2n) | (CC & d[1]) | Dn;
#pragma unroll
    for (int i = 0; i < 5; ++i) N[3 + i] = ((Bn | BC) & nr[i]) | (CC & rib[i]);

    // ---- write round-(t+1) planes
    if (SMALL) {
        const uint32_t npu = 1u << g.lognpu;
#pragma unroll
        for (int p = 0; p < kPlanes; ++p) {
            u64 v = valid ? ((N[p] & L.m) << L.sh) : 0ull;
            for (uint32_t o = 1; o < npu; o <<= 1) v |= __shfl_xor(v, (int)o, 64);
            if (valid && (x & (npu - 1u)) == 0) a.Snext[L.plane_index(p)] = v;
        }
    } else {
        if (valid) {
#pragma unroll
            for (int p = 0; p < kPlanes; ++p) a.Snext[L.plane_index(p)] = N[p];
        }
    }
    if (SHARD && valid) {  // push row of round t+1: the class planes, to owner(t_{t+1}(x))
        const uint32_t sp = a.spos_next[x];
#pragma unroll
        for (int p = 0; p < kClsPlanes; ++p) a.sendA[L.row_index(sp, 3, p)] = N[p] & L.m;
    }

    // ---- push list + Statistics (src/gossip.rs:80,103-111)
    uint32_t live_new = valid ? popc(Bn | Cn) : 0u;
    if (!SMALL) live_new = group_sum(live_new, g.W);
    const int blk_live = __syncthreads_or(live_new != 0u);
    if (blockIdx.x == 0 && threadIdx.x == 0)  // slot of round t, read by the host already
        __hip_atomic_store(&a.flags[(a.round_new + 1u) & 1u], 0u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0 && blk_live) {
        uint32_t *f = &a.flags[a.round_new & 1u];
        if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
            atomicOr(f, 1u);
    }
    if (leader) {
#ifndef GS_EXP_NO_STATS
        // rounds is the engine's round count (every node runs every round);
        // the other four are u32 deltas folded into u64 before they can wrap.
        uint4 *st = reinterpret_cast<uint4 *>(a.st32) + x;
        uint4 v = *st;
        v.x += d_empty_pull;                       // empty_pull_sent
        v.y += (live_new == 0u) ? 1u : 0u;         // empty_push_sent
        v.z += live_new + d_full_sent;             // full_message_sent
        v.w += d_recv;                             // full_message_received
        *st = v;
#endif
    }
}

template <bool SMALL, bool SHARD>
static hipError_t launch_mode(const RoundArgs &a, int mode, hipStream_t s) {
    const uint32_t block = 256;
    const u64 grid = (a.g.nseg + block - 1) / block;
    if (grid == 0) return hipSuccess;
    switch (mode) {
    case 0: hipLaunchKernelGGL((round_kernel<SMALL, 0, SHARD>), dim3((uint32_t)grid), dim3(block), 0, s, a); break;
    case 1: hipLaunchKernelGGL((round_kernel<SMALL, 1, SHARD>), dim3((uint32_t)grid), dim3(block), 0, s, a); break;
    case 2: hipLaunchKernelGGL((round_kernel<SMALL, 2, SHARD>), dim3((uint32_t)grid), dim3(block), 0, s, a); break;
    default: hipLaunchKernelGGL((round_kernel<SMALL, 3, SHARD>), dim3((uint32_t)grid), dim3(block), 0, s, a); break;
    }
    return hipGetLastError();
}

hipError_t launch_round(const RoundArgs &a, int mode, hipStream_t s) {
    if (a.recvA)  // shard engine
        return a.g.small ? launch_mode<true, true>(a, mode, s) : launch_mode<false, true>(a, mode, s);
    return a.g.small ? launch_mode<true, false>(a, mode, s) : launch_mode<false, false>(a, mode, s);
}

// Fold the u32 statistics deltas into the u64 totals (before they can wrap).
__global__ __launch_bounds__(256) void stats_fold(uint32_t *st32, u64 *st64, u64 words) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= words) return;
    st64[i] += st32[i];
    st32[i] = 0u;
}

hipError_t launch_stats_fold(uint32_t *st32, u64 *st64, uint32_t n, hipStream_t s) {
    const u64 words = (u64)n * 4;
    if (words == 0) return hipSuccess;
    hipLaunchKernelGGL(stats_fold, dim3((uint32_t)((words + 255) / 256)), dim3(256), 0, s, st32, st64,
                       words);
    return hipGetLastError();
}

// ------------------------------------------------------------ in-edge lists
// Two-stage counting sort of the n edges (x -> tg[x]) by target, with no
// global atomics (targets are uniform, so fixed-width target bins balance):
//   bin_count   : per source chunk, an LDS histogram over target bins
//                 -> M[chunk][bin]
//   col_scan    : per bin, exclusive prefix over chunks; bin totals
//   scan (1 blk): exclusive prefix of the bin totals -> bin bases
//   bin_scatter : (local target, source) pairs into their bin's range
//                 (runs of ~chunk/nb pairs per chunk and bin)
//   bin_sort    : per bin, LDS counting sort by local target -> src[] with each
//                 node's sources ascending (the order Gossip::receive sees its
//                 pushers in, src/gossiper.rs:217), then the per-node records
//                 IN[y] = {first edge, in-degree, s0, s1}          (node order)
//                 SIB[x] = {serial, rank of x in in(t(x)), e0, e1}  (per source,
//                          written only when rank >= 1; stale serial = rank 0)
CsrPlan csr_plan(uint32_t n) {
    CsrPlan p{};
    p.n = n;
    uint32_t bin = 4096;
    while ((u64)bin * 16384u < n) bin <<= 1;  // <= 16384 bins: bin_count LDS <= 64 KiB
    p.bin = bin;
    p.logbin = 0;
    while ((1u << p.logbin) < bin) ++p.logbin;
    p.nb = (uint32_t)(((u64)n + bin - 1) / bin);
    uint32_t ba = (uint32_t)(((u64)n + 4095) / 4096);
    p.ba = ba < 256u ? (ba ? ba : 1u) : 256u;
    p.chunk = (uint32_t)(((u64)n + p.ba - 1) / p.ba);
    return p;
}

size_t csr_scratch_words(const CsrPlan &p) {
    // M[ba][nb] + tot[nb] + base[nb] (u32 words); pairs are separate (u64 [n])
    return (size_t)p.ba * p.nb + 2 * (size_t)p.nb;
}

// Also draws the round's peer choices (Gossiper::next_round's
// thread_rng().choose, src/gossiper.rs:71, as the injected Philox stream).
__global__ __launch_bounds__(256) void csr_bin_count(uint32_t *__restrict__ tg, CsrPlan p,
                                                     uint32_t *M, uint64_t seed, uint32_t epoch,
                                                     uint32_t round) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
    for (uint32_t i = threadIdx.x; i < p.nb; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    const u64 lo = (u64)blockIdx.x * p.chunk;
    const u64 hi = min((u64)p.n, lo + p.chunk);
    for (u64 x = lo + threadIdx.x; x < hi; x += blockDim.x) {
        const uint32_t t = peer_of(seed, epoch, round, (uint32_t)x, p.n);
        tg[x] = t;
        atomicAdd(&hist[t >> p.logbin], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < p.nb; i += blockDim.x) M[(u64)blockIdx.x * p.nb + i] = hist[i];
}

__global__ __launch_bounds__(256) void csr_col_scan(uint32_t *M, CsrPlan p, uint32_t *tot) {
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

// Exclusive scan of a small array (one block).
__global__ __launch_bounds__(kScanBlock) void scan_small(const uint32_t *in, uint32_t *out, uint32_t m) {
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

__global__ __launch_bounds__(256) void csr_bin_scatter(const uint32_t *__restrict__ tg, CsrPlan p,
                                                       const uint32_t *__restrict__ M,
                                                       const uint32_t *__restrict__ base, u64 *pairs) {
    extern __shared__ __attribute__((aligned(16))) uint32_t cur[];
    for (uint32_t i = threadIdx.x; i < p.nb; i += blockDim.x)
        cur[i] = base[i] + M[(u64)blockIdx.x * p.nb + i];
    __syncthreads();
    const u64 lo = (u64)blockIdx.x * p.chunk;
    const u64 hi = min((u64)p.n, lo + p.chunk);
    const uint32_t lm = p.bin - 1u;
    for (u64 x = lo + threadIdx.x; x < hi; x += blockDim.x) {
        const uint32_t t = tg[x];
        const uint32_t pos = atomicAdd(&cur[t >> p.logbin], 1u);
        pairs[pos] = ((u64)(t & lm) << 32) | (uint32_t)x;
    }
}

__global__ __launch_bounds__(256) void csr_bin_sort(const u64 *__restrict__ pairs, CsrPlan p,
                                                    const uint32_t *__restrict__ base,
                                                    const uint32_t *__restrict__ tot, uint32_t *src,
                                                    uint4 *IN, uint4 *SIB, uint32_t serial) {
    extern __shared__ __attribute__((aligned(16))) uint32_t h[];  // [bin] + 16 scan words
    uint32_t *lds_scan = h + p.bin;
    const uint32_t b = blockIdx.x;
    const uint32_t start = base[b], cnt = tot[b];
    const uint32_t nb0 = b << p.logbin;
    const uint32_t nodes = min(p.bin, p.n - nb0);
    for (uint32_t i = threadIdx.x; i < p.bin; i += blockDim.x) h[i] = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) atomicAdd(&h[pairs[start + i] >> 32], 1u);
    __syncthreads();
    // exclusive scan of h[0..bin): each thread owns bin/256 consecutive counters
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
        src[start + pos] = (uint32_t)pr;
    }
    __syncthreads();
    // h[i] is now the end of node i's bucket: sort each (Poisson(1)-sized)
    // bucket, then emit IN[] and SIB[].
    for (uint32_t i = threadIdx.x; i < nodes; i += blockDim.x) {
        const uint32_t a = start + (i ? h[i - 1] : 0u), e = start + h[i];
        for (uint32_t q = a + 1; q < e; ++q) {
            const uint32_t v = src[q];
            uint32_t r = q;
            while (r > a && src[r - 1] > v) {
                src[r] = src[r - 1];
                --r;
            }
            src[r] = v;
        }
        const uint32_t k = e - a;
        const uint32_t s0 = k > 0 ? src[a] : 0u, s1 = k > 1 ? src[a + 1] : 0u;
        const uint32_t y = nb0 + i;
        IN[y] = make_uint4(a, k, s0, s1);
        (void)y;
        for (uint32_t q = a + 1; q < e; ++q) {
            const uint32_t rank = q - a;
            SIB[src[q]] = make_uint4(serial, rank, s0, rank > 1 ? s1 : 0u);
        }
    }
}

hipError_t launch_build_csr(uint32_t *tg, const CsrPlan &p, uint32_t *scratch, u64 *pairs,
                            uint32_t *src, uint4 *IN, uint4 *SIB, uint32_t serial,
                            uint64_t seed, uint32_t epoch, uint32_t round, hipStream_t s) {
    uint32_t *M = scratch;
    uint32_t *tot = M + (size_t)p.ba * p.nb;
    uint32_t *base = tot + p.nb;
    const size_t lds_nb = (size_t)p.nb * sizeof(uint32_t);
    hipLaunchKernelGGL(csr_bin_count, dim3(p.ba), dim3(256), lds_nb, s, tg, p, M, seed, epoch, round);
    hipLaunchKernelGGL(csr_col_scan, dim3((p.nb + 255) / 256), dim3(256), 0, s, M, p, tot);
    hipLaunchKernelGGL(scan_small, dim3(1), dim3(kScanBlock), 0, s, tot, base, p.nb);
    hipLaunchKernelGGL(csr_bin_scatter, dim3(p.ba), dim3(256), lds_nb, s, tg, p, M, base, pairs);
    const size_t lds_sort = ((size_t)p.bin + 16) * sizeof(uint32_t);
    if (lds_sort > 65536) {  // n > 2^28: bins of 32768 nodes need 128 KiB of the 160 KiB LDS
        hipError_t e = hipFuncSetAttribute((const void *)csr_bin_sort,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_sort);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(csr_bin_sort, dim3(p.nb), dim3(256), lds_sort, s, pairs, p, base, tot, src, IN,
                       SIB, serial);
    return hipGetLastError();
}

// ------------------------------------------------------------ reductions
__global__ __launch_bounds__(256) void known_reduce(const u64 *__restrict__ known, uint32_t n,
                                                    uint32_t KW, uint32_t R, u64 *partials) {
    __shared__ u64 s_tot[256], s_cmp[256];
    u64 tot = 0, cmp = 0;
    for (u64 x = (u64)blockIdx.x * blockDim.x + threadIdx.x; x < n; x += (u64)gridDim.x * blockDim.x) {
        uint32_t c = 0;
        for (uint32_t w = 0; w < KW; ++w) c += popc(known[x * KW + w]);
        tot += c;
        cmp += (c == R) ? 1u : 0u;
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

hipError_t launch_known_reduce(const u64 *known, uint32_t n, uint32_t KW, uint32_t R,
                               u64 *partials, uint32_t blocks, hipStream_t s) {
    hipLaunchKernelGGL(known_reduce, dim3(blocks), dim3(256), 0, s, known, n, KW, R, partials);
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
