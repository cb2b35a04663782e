// gs_common.h -- host/device helpers shared by the engine and its kernels:
// the injected Philox4x32-10 peer schedule and the packed state layout.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gs {

typedef unsigned long long u64;

// Philox4x32-10 (Salmon et al., Random123), the generator rocrand's
// philox4x32_10 engine implements; KATs in tests/test_philox.py.
constexpr uint32_t kPhM0 = 0xD2511F53u, kPhM1 = 0xCD9E8D57u;
constexpr uint32_t kPhW0 = 0x9E3779B9u, kPhW1 = 0xBB67AE85u;

// Counter word 2 selects the stream.
constexpr uint32_t kStreamPeer = 0, kStreamOrigin = 1, kStreamCoin = 2, kStreamFault = 3;

__host__ __device__ __forceinline__ uint32_t mulhi32(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umulhi(a, b);
#else
    return (uint32_t)(((uint64_t)a * b) >> 32);
#endif
}

struct Ph4 {
    uint32_t w0, w1, w2, w3;
};

__host__ __device__ __forceinline__ Ph4 philox4(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                uint64_t seed) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
#ifdef GS_PHILOX_MULHI
        uint32_t hi0 = mulhi32(kPhM0, c0), lo0 = kPhM0 * c0;
        uint32_t hi1 = mulhi32(kPhM1, c2), lo1 = kPhM1 * c2;
#else
        // one v_mad_u64_u32 per product instead of a mul_hi + mul_lo pair
        const uint64_t p0 = (uint64_t)kPhM0 * c0, p1 = (uint64_t)kPhM1 * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
#endif
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += kPhW0; k1 += kPhW1;
    }
    return {c0, c1, c2, c3};
}

__host__ __device__ __forceinline__ u64 philox_u64(uint32_t c0, uint32_t c1, uint32_t c2,
                                                   uint32_t c3, uint64_t seed) {
    const Ph4 w = philox4(c0, c1, c2, c3, seed);
    return ((u64)w.w1 << 32) | w.w0;
}

// floor(v * m / 2^64): uniform index in [0, m).
__host__ __device__ __forceinline__ uint32_t mulhi64(u64 v, uint32_t m) {
    u64 lo = (u64)(uint32_t)v * m;
    u64 hi = (u64)(uint32_t)(v >> 32) * m;
    return (uint32_t)((hi + (lo >> 32)) >> 32);
}

// Gossiper::next_round's rand::thread_rng().choose(&self.peers)
// (src/gossiper.rs:71) over create_network's peer order
// (src/gossiper.rs:157-171: node k's peers are [0..k-1, k+1..n-1]).
__host__ __device__ __forceinline__ uint32_t peer_of(uint64_t seed, uint32_t epoch,
                                                    uint32_t round, uint32_t node, uint32_t n) {
    uint32_t u = mulhi64(philox_u64(round, node, kStreamPeer, epoch, seed), n - 1u);
    return u + (u >= node ? 1u : 0u);
}

__host__ __device__ __forceinline__ uint32_t origin_of(uint64_t seed, uint32_t epoch,
                                                      uint32_t rumor, uint32_t n) {
    return mulhi64(philox_u64(rumor, 0u, kStreamOrigin, epoch, seed), n);
}

__host__ __device__ __forceinline__ uint32_t coin_of(uint64_t seed, uint32_t epoch,
                                                    uint32_t round, uint32_t node) {
    return (uint32_t)(philox_u64(round, node, kStreamCoin, epoch, seed) & 1u);
}

// Harness-injected faults, thresholds over
// 2^32: churn = the node is offline for the round (no next_round, every RPC to
// or from it dropped, state kept), push = its push batch is dropped (and so
// never answered), pull = the pull batch answering it is dropped.  One Philox
// draw per (round, node) on stream kStreamFault: word 0 churn, 1 push, 2 pull.
struct Faults {
    uint32_t churn, push, pull;
};

__host__ __device__ __forceinline__ bool faults_on(const Faults &f) {
    return (f.churn | f.push | f.pull) != 0u;
}

__host__ __device__ __forceinline__ bool offline_of(uint64_t seed, uint32_t epoch, uint32_t round,
                                                   uint32_t node, uint32_t churn) {
    return churn != 0u && philox4(round, node, kStreamFault, epoch, seed).w0 < churn;
}

// Target word of (round, node): t(x) in the low 29 bits (n < 2^29 is implied
// by the state layout's n < e^(e^3)) plus the delivery flags of x's edge.
constexpr uint32_t kTgDead = 1u << 31;    // x's push batch is not delivered
constexpr uint32_t kTgNoPull = 1u << 30;  // no pull batch reaches x
constexpr uint32_t kTgOff = 1u << 29;     // x is offline this round
constexpr uint32_t kTgMask = kTgOff - 1u;

// SEQ schedule, per-node info byte (gs_seq.hip): x receives a pull at time x,
// its pull depends on t(x)'s pull (t(x) < x), and the level of that chain.
constexpr uint32_t kSeqGot = 0x80u, kSeqDep = 0x40u, kSeqLevelMask = 0x3Fu;
// Level code of a node whose pull no later node reads (no pusher above it):
// the round kernel builds its pull inline, so it is in no pass list.
constexpr uint32_t kSeqInline = kSeqLevelMask;

__host__ __device__ __forceinline__ uint32_t target_word(uint64_t seed, uint32_t epoch,
                                                        uint32_t round, uint32_t node, uint32_t n,
                                                        const Faults &f) {
    const uint32_t t = peer_of(seed, epoch, round, node, n);
    if (!faults_on(f)) return t;
    const Ph4 w = philox4(round, node, kStreamFault, epoch, seed);
    if (w.w0 < f.churn) return t | kTgDead | kTgNoPull | kTgOff;
    if (w.w1 < f.push || offline_of(seed, epoch, round, t, f.churn)) return t | kTgDead | kTgNoPull;
    if (w.w2 < f.pull) return t | kTgNoPull;
    return t;
}

// ---------------------------------------------------------------------------
// Packed per-(node, rumor) state: 8 bit-planes ("State layout").
//   plane 0  isC        plane 1,2  a = f2 (2 bits)    planes 3..7  b = f1 (5 bits)
//   A: isC=0 a=0        B: isC=0 a=our_counter (1|2)  b=round
//   C: isC=1 a=round (0..2) b=rounds_in_state_b       D: isC=1 a=3 b=0
// Valid while counter_max <= 3, max_c_rounds <= 3, max_rounds <= 32.
constexpr int kPlanes = 8;
constexpr int kClsPlanes = 3;   // isC, a0, a1: everything a neighbour reads

struct Geometry {
    uint32_t n;         // nodes
    uint32_t R;         // rumors
    uint32_t rpad;      // next pow2 >= R
    uint32_t W;         // 64-bit words per node (rpad >= 64), else 1
    uint32_t small;     // rpad < 64: several nodes per word
    uint32_t lognpu;    // log2(nodes per unit word) when small
    uint32_t logr;      // log2(rpad)
    uint64_t units;     // records of kPlanes*W words
    uint64_t nseg;      // lanes: n*W (big) or n (small)
};

// In-edge records of one round (gs_inlist.hip):
//   InRec[y]  = {first << 5 | k, s0, s1, s2} (16 B): y's k pushers in
//               ascending index order (the order Gossip::receive sees them);
//               pushers i >= kInline are at src[first + i - kInline] (tails of
//               the 1.9% of nodes with in-degree > 3).  k <= kMaxIn: a larger
//               in-degree (probability ~1e-34 per node) is a device limit.
//   SibRec[x] = {serial << 8 | rank, e0, e1, e2} (16 B): x's rank among the
//               pushers of t(x) and the first kSibInline pushers ahead of it
//               (the rest are InRec[t(x)].s / its tail); valid iff the serial
//               is the round build's (stale records are never cleared).
// Both are read coalesced by the round kernel, so every gather of a node with
// in-degree <= kInline is issued from one level of metadata reads.
constexpr uint32_t kInline = 3;
constexpr uint32_t kSibInline = 3;
constexpr uint32_t kSerialMask = 0xFFFFFFu;
constexpr uint32_t kMaxIn = 30;      // in-degree limit (5-bit k field)
constexpr uint32_t kFirstShift = 5;  // tails: first < 2^27
struct alignas(16) InRec {
    uint32_t kf, s[kInline];
    __host__ __device__ uint32_t k() const { return kf & ((1u << kFirstShift) - 1u); }
    __host__ __device__ uint32_t first() const { return kf >> kFirstShift; }
};
struct alignas(16) SibRec {
    uint32_t tag, e[kSibInline];
};
// Live-filtered gathers (2P gather path, binned in-lists): the build of round
// t's lists reads two node maps of round t's planes, "live" (some B or C
// entry: its push row is not empty) and "complete" (no A entry: it creates
// nothing), and marks the class rows the round kernel may skip because they
// cannot change a result, in bits the records do not otherwise use:
//   InRec.kf bits 28-30  pusher i = 0..2 pushes nothing (binned tails:
//                        first < 2^23)
//   SibRec.tag bits 5-6  sibling i = 0, 1 is not live or t(x) is complete
//                        (no creation to pass on); rank < 32
//   SibRec.e[2] bit 31   the same for sibling 2 (node ids are < 2^29)
//   SibRec.tag bit 7     some earlier sibling is live and t(x) incomplete
//                        (t(x)'s A-set is needed)
// and a per-source bit map zl = t(x) is live.
constexpr uint32_t kInSkipShift = 28;
constexpr uint32_t kInFlagMask = (1u << kInSkipShift) - 1u;
constexpr uint32_t kSibSkipShift = 5;
constexpr uint32_t kSkipBit = 1u << 31;
constexpr uint32_t kIdMask = kSkipBit - 1u;
constexpr uint32_t kSibZNeed = 1u << 7;
constexpr uint32_t kSibRankMask = 0x1Fu;

// Delivery records (R_pad <= 16, 2P, binned in-lists; gs_inlist.hip): the
// in-list build carries every pusher's push code to its receiver and returns
// every pull batch to its pusher, both in node order, so a round kernel lane
// reads only coalesced per-node data -- no class-plane gathers (the gather
// path fetches three random 128-B lines per node: pushers, t(x), t(x)'s
// earlier pushers).
//   DlvRec[y] = {mf = k | zi << 5 (index of t(y) among y's pushers, 31 =
//               none) | flags << 10 | f << 12, c[0], c[1]} (12 B): the push
//               codes (b0 | b1 << 16: 01 counter 1, 10 counter 2, 11 counter
//               255) of y's pushers in ascending order, pushers i >= kDlvInline
//               at dtail[first + i - 2], first = (y >> tlog) * tper + f: the
//               tails of y's sort part (2^tlog targets) own a fixed region of
//               tper slots (RoundArgs::dlv_tlog / dlv_tper, dlv_tail_parts)
//   PULL[x]   = the pull batch t(x) returned to x, the same 2-plane code
constexpr uint32_t kDlvInline = 2;
constexpr uint32_t kDlvNoZ = 31u;
// single-engine records also carry y's own delivery flags (kTgNoPull, kTgOff)
// in meta bits 10 and 11, so the packed round kernel reads no target words
constexpr uint32_t kDlvMetaNoPull = 10u, kDlvMetaOff = 11u;
static_assert(kTgNoPull == 1u << 30 && kTgOff == 1u << 29, "meta flag bits mirror the target-word flags");
constexpr uint32_t kDlvFirstShift = 12u;  // mf bits 12..31: the tail offset within y's part
struct alignas(4) DlvRec {
    uint32_t mf, c[kDlvInline];
};
static_assert(sizeof(DlvRec) == 12, "one delivery record is 12 bytes");

// State digest (gs_state_digest; oracle/gs_dense.c and tests/oracle_lib.py
// digest_of compute the same): per node, the sum mod 2^64 of
//   * per 64-rumor word j < ceil(R/64), one term mixing the 20 bit-planes
//     of what gs_dump_state and gs_dump_records report for those rumors
//     (state code bits 14, 15, 7, 8, 0..4, then record bits 15, 0..4,
//     7..11; bit b of plane p = that bit of rumor 64j + b): mix(sum_p
//     plane_p * K_p ^ mix(j + C));
//   * one term for |peers_in_this_round| and one per Statistics counter.
// Order-free, so the lanes holding the words of a node add their terms.
__host__ __device__ inline u64 digest_mix(u64 z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// odd multipliers of the 20 planes (SplitMix64's golden-ratio increments)
__host__ __device__ inline u64 digest_plane_k(uint32_t p) { return 0x9E3779B97F4A7C15ull * (2ull * p + 1ull); }
// The 20 observation planes of word j (m: its valid rumor bits) from the
// post-delivery bit-sliced state: entries in A/B/C/D before the deliveries
// (B, C, D; a0, a1 and the five b planes bp), the entries the deliveries
// created (crB: B{0,1}, crC: C{0,0}), and the record counters of B entries
// (anyC; c1: #counters in [1, counter_max); c2: #counters == 2).
__host__ __device__ inline void digest_planes(u64 m, u64 B, u64 C, u64 D, u64 crB, u64 crC, u64 a0, u64 a1,
                                              const u64 *bp, u64 anyC, const u64 *c1, const u64 *c2, u64 pl[20]) {
    const u64 BC = B | C, E = B | crB;
    pl[0] = crB | B | D;          // code bit 14 (tag 1 or 3)
    pl[1] = crC | C | D;          // code bit 15 (tag 2 or 3)
    pl[2] = crB | (BC & a0);      // code bit 7 (f2 bit 0; a created B has our_counter 1)
    pl[3] = BC & a1;              // code bit 8
    for (int i = 0; i < 5; ++i) pl[4 + i] = BC & bp[i];  // code bits 0..4 (f1)
    pl[9] = E & anyC;             // record bit 15
    for (int i = 0; i < 5; ++i) {
        pl[10 + i] = E & c1[i];   // record bits 0..4
        pl[15 + i] = E & c2[i];   // record bits 7..11
    }
    for (int p = 0; p < 20; ++p) pl[p] &= m;
}
// The word's sum before the final mix, and the mix (word j of the network).
// The sum is linear over disjoint rumor bits, so engines holding parts of one
// word (rumor slices) add their parts' sums (gs_state_digest_part).
__host__ __device__ inline u64 digest_sum(const u64 pl[20], uint32_t shl = 0) {
    u64 h = 0;
    for (uint32_t p = 0; p < 20; ++p) h += (pl[p] << shl) * digest_plane_k(p);
    return h;
}
__host__ __device__ inline u64 digest_fin(uint32_t j, u64 h) { return digest_mix(h ^ digest_mix((u64)j + 0x632BE59BD9B4E019ull)); }
__host__ __device__ inline u64 digest_word(uint32_t j, u64 m, u64 B, u64 C, u64 D, u64 crB, u64 crC, u64 a0,
                                           u64 a1, const u64 *bp, u64 anyC, const u64 *c1, const u64 *c2) {
    u64 pl[20];
    digest_planes(m, B, C, D, crB, crC, a0, a1, bp, anyC, c1, c2, pl);
    return digest_fin(j, digest_sum(pl));
}
__host__ __device__ inline u64 digest_node(uint32_t psize, const u64 *st5) {
    u64 h = digest_mix((1ull << 63) | psize);
    for (int i = 0; i < 5; ++i) h += digest_mix(st5[i] ^ (0x9E3779B97F4A7C15ull * (u64)(i + 1)));
    return h;
}

}  // namespace gs
