// gs_recv.h -- receiver-side bit-sliced state of phases 1-2 of a round at
// one node (Gossip::receive, src/gossip.rs:118-163), shared by the round
// kernels (gs_kernels.hip, gs_w32.hip).
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
// T is the lane word: u64 (64 rumors per lane) or u32 (gs_w32.hip).
template <bool OBS, typename T = u64>
struct Recv {
    T notyet;            // still absent: the next live copy creates the entry
    T recB;              // entries in state B (existing or created): record copies
    T oc1;               // B entries whose our_counter is 1 (created ones included)
    T crB, crC;          // created this round as B{0,1} / C{0,0}
    T anyC;              // a recorded counter >= counter_max
    T cv[5];             // #recorded counters >= our_counter (and < counter_max)
    T c1[5];             // OBS only: #recorded counters in [1, counter_max)
    T c2[5];             // OBS only: #recorded counters == 2 (< counter_max)
    uint32_t part_cw;    // sum over pushers i of (k-1-i) * |created by i|
    uint32_t first_create;
    uint32_t recv;       // copies received (push rows + pull row)

    GS_DEV void init(T A, T B, T Boc1) {
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
    GS_DEV void record(T rec, T vB, T v2, T vC) {
        anyC |= rec & vC;
        add5T(cv, rec & vB & (v2 | oc1));
        if constexpr (OBS) {
            add5T(c1, rec & vB);
            add5T(c2, rec & v2);
        }
    }
    GS_DEV void create(T newc, T vC) {
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
    GS_DEV void absorb(T vB, T v2, T vC, uint32_t rafter, uint32_t ev, T recm) {
        const T sl = vB | vC;                  // the batch
        const T newc = notyet & sl;            // new_from_peer: not recorded
        record(recB & sl & recm, vB, v2, vC);  // MessageState::receive on B
        create(newc, vC);
        const uint32_t pc = popcT(newc);
        part_cw += rafter * pc;
        if (pc && first_create == kNone) first_create = ev;
        recv += popcT(sl);
    }
    // Push batch of pusher i of k (2P: pushers in ascending order, all
    // answered; `rec_on` is false for t(x)'s own push, superseded by its pull).
    GS_DEV void push(const ClsT<T> &q, uint32_t i, uint32_t k, bool rec_on) {
        const T vC = q.c & ~(q.a0 & q.a1);     // C: counter 255
        const T vB = ~q.c & (q.a0 | q.a1);     // B: counter = our_counter
        const T v2 = vB & q.a1 & ~q.a0;        // B with our_counter 2
        const T sl = vB | vC;                  // the push batch
        const T newc = notyet & sl;            // new_from_peer: not recorded
        if (rec_on) record(recB & sl, vB, v2, vC);  // MessageState::receive on B
        create(newc, vC);
        const uint32_t pc = popcT(newc);
        part_cw += (k - 1u - i) * pc;  // later pushers' pull rows include it
        if (pc && first_create == kNone) first_create = i;
        recv += popcT(sl);
    }
    GS_DEV void absorb_cls(const ClsT<T> &q, uint32_t rafter, uint32_t ev, bool rec_on) {
        const T vC = q.c & ~(q.a0 & q.a1);     // C: counter 255
        const T vB = ~q.c & (q.a0 | q.a1);     // B: counter = our_counter
        const T v2 = vB & q.a1 & ~q.a0;        // B with our_counter 2
        absorb(vB, v2, vC, rafter, ev, rec_on ? (T)~(T)0 : (T)0);
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
template <typename T>
struct NextOutT {
    T N[kPlanes];  // round-(t+1) planes
    T Bn, Cn;      // entries in state B / C after the transition
    T bump, anyC;  // !on_next: the votes next_round will use
};
using NextOut = NextOutT<u64>;
template <typename RV, typename T>
GS_DEV void next_round_seg(const T (&P)[kPlanes], const RV &rv, T inj, uint32_t psize, bool pending,
                           T pbump, T panyC, bool on_next, uint32_t cmax, uint32_t maxc,
                           uint32_t maxr, NextOutT<T> &o) {
    const T isC = P[0], a0 = P[1], a1 = P[2];
    const T B = ~isC & (a0 | a1);
    const T C = isC & ~(a0 & a1);
    const T D = isC & a0 & a1;
    const T ninj = ~inj;
    const T Bold = B & ninj, Cold = C & ninj, Dold = D & ninj;
    const T cB = rv.crB & ninj, cC = rv.crC & ninj;
    const T Bf = Bold | cB | inj;  // entries in state B entering next_round
    const T Cf = Cold | cC;        // entries in state C entering next_round

    // B (src/message_state.rs:94-147).  0-filled peers vote "less", so with
    // no C copy the median rule is: bump iff 2*ge > |P| iff ge >= |P|/2+1.
    const T oc1 = (Bold & a0 & ~a1) | cB | inj;
    const T oc2 = Bold & a1 & ~a0;
    T bump, anyCe;
    if (pending) {
        bump = pbump & Bold;
        anyCe = panyC & ninj;
    } else {
        bump = ge_kT<5>(rv.cv, psize / 2u + 1u) & (Bold | cB);  // cv counts only B entries' votes
        anyCe = rv.anyC & ninj;
    }
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
    const T toD = ge_uT<6>(nr, maxr);
    const T oc1n = oc1 & ~bump;
    const T oc2n = (oc1 & bump) | (oc2 & ~bump);
    const T oc3n = oc2 & bump;
    const T ocge = cmax <= 1u ? (T)~(T)0 : (cmax == 2u ? (oc2n | oc3n) : oc3n);
    const T toC = anyCe | ocge;
    const T BD = Bf & toD, BC = Bf & ~toD & toC, BB = Bf & ~toD & ~toC;

    // C (src/message_state.rs:148-168): round+1; D if round+rib >= max_rounds
    // or round >= max_c_rounds.
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
    const T CtoD = ge_uT<6>(sum, maxr) | ge_uT<3>(d, maxc);
    const T CD = Cf & CtoD, CC = Cf & ~CtoD;

    const T Dn = BD | CD | Dold;
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
