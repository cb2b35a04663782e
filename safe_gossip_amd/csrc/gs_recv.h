// gs_recv.h -- receiver-side bit-sliced state of phases 1-2 of a round at
// one node (Gossip::receive, src/gossip.rs:118-163), shared by the round
// kernels (gs_kernels.hip, gs_pipe.hip).
#pragma once
#include "gs_device.h"
#include "gs_kernels.h"

namespace gs {

// Gathers issued in the first batch: pushers (in-degree is Poisson(1): <= 3
// for 98% of nodes) and pushers of t(x) ahead of x (rank <= 2 for 98.6%).
#ifndef GS_BATCH_K
#define GS_BATCH_K 3
#endif
#ifndef GS_BATCH_E
#define GS_BATCH_E 2
#endif
static_assert(GS_BATCH_E <= kSibInline, "SIB records hold kSibInline pushers");
constexpr uint32_t kBatchK = GS_BATCH_K;
constexpr uint32_t kBatchE = GS_BATCH_E;

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
    // One batch x absorbs (Gossip::receive, src/gossip.rs:153-163) with
    // copies of class vB (counter < counter_max; v2: counter 2) or vC (255).
    // `rafter` = pull rows x sends after it (they include what it creates),
    // `ev` = its position among x's batches; `recm` masks out the rumors whose
    // copy a later copy from the same peer overwrites (message_state.rs:79).
    GS_DEV void absorb(u64 vB, u64 v2, u64 vC, uint32_t rafter, uint32_t ev, u64 recm) {
        const u64 sl = vB | vC;                // the batch
        const u64 newc = notyet & sl;          // new_from_peer: not recorded
        record(recB & sl & recm, vB, v2, vC);  // MessageState::receive on B
        create(newc, vC);
        const uint32_t pc = popc(newc);
        part_cw += rafter * pc;
        if (pc && first_create == kNone) first_create = ev;
        recv += popc(sl);
    }
    // Push batch of pusher i of k (2P: pushers in ascending order, all
    // answered; `rec_on` is false for t(x)'s own push, superseded by its pull).
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
    GS_DEV void absorb_cls(const Cls &q, uint32_t rafter, uint32_t ev, bool rec_on) {
        const u64 vC = q.c & ~(q.a0 & q.a1);   // C: counter 255
        const u64 vB = ~q.c & (q.a0 | q.a1);   // B: counter = our_counter
        const u64 v2 = vB & q.a1 & ~q.a0;      // B with our_counter 2
        absorb(vB, v2, vC, rafter, ev, rec_on ? ~0ull : 0ull);
    }
};

// Rumors injected at segment `key` this round (Gossip::new_message,
// src/gossip.rs:71-75): binary search of the sorted injection keys.
GS_DEV u64 find_injection(const RoundArgs &a, u64 key) {
    uint32_t lo = 0, hi = a.n_inj;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.inj_key[mid] < key) lo = mid + 1; else hi = mid;
    }
    return (lo < a.n_inj && a.inj_key[lo] == key) ? a.inj_mask[lo] : 0ull;
}

// Phase 0 of round t+1 at one segment, bit-sliced: Gossip::new_message for
// the injected rumors `inj` (insert = replace with MessageState::new,
// src/gossip.rs:71-75), then MessageState::next_round for every rumor
// (src/message_state.rs:86-171) from the round-t planes P, the entries the
// deliveries created (rv.crB / rv.crC), the recorded votes (rv.cv, rv.anyC)
// and |peers_in_this_round| = psize.  A node returning from churn (`pending`)
// takes its votes from the pend words (pbump, panyC) instead; a node going
// offline (!on_next) keeps its pre-transition planes and leaves its votes in
// bump / anyC for the caller to store.
struct NextOut {
    u64 N[kPlanes];  // round-(t+1) planes
    u64 Bn, Cn;      // entries in state B / C after the transition
    u64 bump, anyC;  // !on_next: the votes next_round will use
};
template <typename RV>
GS_DEV void next_round_seg(const u64 (&P)[kPlanes], const RV &rv, u64 inj, uint32_t psize, bool pending,
                           u64 pbump, u64 panyC, bool on_next, uint32_t cmax, uint32_t maxc,
                           uint32_t maxr, NextOut &o) {
    const u64 isC = P[0], a0 = P[1], a1 = P[2];
    const u64 B = ~isC & (a0 | a1);
    const u64 C = isC & ~(a0 & a1);
    const u64 D = isC & a0 & a1;
    const u64 ninj = ~inj;
    const u64 Bold = B & ninj, Cold = C & ninj, Dold = D & ninj;
    const u64 cB = rv.crB & ninj, cC = rv.crC & ninj;
    const u64 Bf = Bold | cB | inj;  // entries in state B entering next_round
    const u64 Cf = Cold | cC;        // entries in state C entering next_round

    // B (src/message_state.rs:94-147).  0-filled peers vote "less", so with
    // no C copy the median rule is: bump iff 2*ge > |P| iff ge >= |P|/2+1.
    const u64 oc1 = (Bold & a0 & ~a1) | cB | inj;
    const u64 oc2 = Bold & a1 & ~a0;
    u64 bump, anyCe;
    if (pending) {
        bump = pbump & Bold;
        anyCe = panyC & ninj;
    } else {
        bump = ge_k<5>(rv.cv, psize / 2u + 1u) & (Bold | cB);  // cv counts only B entries' votes
        anyCe = rv.anyC & ninj;
    }
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
    const u64 toD = ge_u<6>(nr, maxr);
    const u64 oc1n = oc1 & ~bump;
    const u64 oc2n = (oc1 & bump) | (oc2 & ~bump);
    const u64 oc3n = oc2 & bump;
    const u64 ocge = cmax <= 1u ? ~0ull : (cmax == 2u ? (oc2n | oc3n) : oc3n);
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
    const u64 CtoD = ge_u<6>(sum, maxr) | ge_u<3>(d, maxc);
    const u64 CD = Cf & CtoD, CC = Cf & ~CtoD;

    const u64 Dn = BD | CD | Dold;
    o.Cn = BC | CC;
    o.Bn = BB;
    o.N[0] = o.Cn | Dn;
    o.N[1] = (BB & oc1n) | (CC & d[0]) | Dn;
    o.N[2] = (BB & oc2n) | (CC & d[1]) | Dn;
#pragma unroll
    for (int i = 0; i < 5; ++i) o.N[3 + i] = ((BB | BC) & nr[i]) | (CC & rib[i]);
    o.bump = bump;
    o.anyC = anyCe & (Bold | cB);
    if (!on_next) {  // frozen: pre-transition planes, entries created folded in
        o.N[0] = (isC & ninj) | cC;
        o.N[1] = (a0 & ninj) | cB | inj;
        o.N[2] = a1 & ninj;
#pragma unroll
        for (int i = 0; i < 5; ++i) o.N[3 + i] = P[3 + i] & ninj;
    }
}

}  // namespace gs
