// gs_inlist.hip -- the in-edge lists of one round: every node's peer choice
// (Gossiper::next_round's thread_rng().choose, src/gossiper.rs:71, replaced by
// the injected Philox stream) inverted into, per receiver y, its pushers in
// ascending index order -- the order in which the reference harness delivers
// push batches (src/gossiper.rs:217-231 walks (src, dst) pairs by src Id) --
// and, per source x, the pushers of t(x) ahead of x (what t(x) created from
// them before it answered x, src/gossip.rs:124-151).  Output records: InRec /
// SibRec (gs_common.h).
//
// Targets are uniform and independent of the source, so the inversion is a
// bucket sort with a known distribution; no global prefix sum is needed:
//
//   binned path (n <= kBinnedMaxNodes), two launches, no atomics on HBM
//   except one returning add per (chunk, bin) run:
//     inl_bin  : per chunk of kChunk sources: Philox targets (-> tg), an LDS
//                counting sort of the chunk by target bin, one reservation
//                per non-empty bin in that bin's fixed-capacity region, and
//                coalesced stores of the chunk's sources, bin-run by bin-run
//     inl_sort : per bin of kBin targets: LDS counting sort by target (16-bit
//                packed counters), per-target insertion sort by source, and
//                the InRec / SibRec records (+ the rare in-degree > kInline
//                tails)
//   generic path (larger n): the two-stage LDS counting sort through an exact
//   global CSR (csr_*), same records.
//
// Region capacity is kBin + kBin/4 sources per bin (the mean is kBin, the
// standard deviation sqrt(kBin) = 128): an overflow, like an in-degree > 30,
// is reported as GS_ERR_DEVICE_LIMIT (flags[2]) rather than handled.
#include <cstdlib>

#include "gs_kernels.h"
#include "gs_device.h"

namespace gs {

namespace {

#ifndef GS_INL_BINLOG
#define GS_INL_BINLOG 14
#endif
constexpr uint32_t kBinLog = GS_INL_BINLOG;
constexpr uint32_t kBin = 1u << kBinLog;          // targets per bin
constexpr uint32_t kBinCap = kBin + kBin / 4;     // region capacity per bin
#ifndef GS_INL_CHUNK
#define GS_INL_CHUNK 8192
#endif
constexpr uint32_t kChunk = GS_INL_CHUNK;         // sources per inl_bin block
constexpr uint32_t kInlThreads = 1024;
static_assert(kChunk % kInlThreads == 0, "inl_bin: whole sources per thread");
constexpr uint32_t kChunkSmall = 2048;            // sources per inl_bin block below 2^22 nodes
static_assert(kChunkSmall % kInlThreads == 0, "inl_bin: whole sources per thread");
constexpr uint32_t kBinnedMaxBins = 1u << (27 - kBinLog);  // n <= 2^27 (per-bin LDS state is 6 B)
#ifndef GS_SORT_OWN_TAILS
#define GS_SORT_OWN_TAILS 1  // A/B: 0 = one shared tail counter (reserve_tails)
#endif
#ifndef GS_DLV_OWN_TAILS
#define GS_DLV_OWN_TAILS 1  // A/B: 0 = one shared tail counter (reserve_tails)
#endif
constexpr uint32_t kFlagLimit = 2u;               // flags[2] bit: a device limit was hit

// Target word (target + delivery flags, gs_common.h); edges flagged kTgDead
// carry no push batch and are left out of the lists.
GS_DEV uint32_t target_of(const InListArgs &a, uint32_t x) {
    return target_word(a.seed, a.epoch, a.round, x, a.p.n, a.f);
}

// A source of the DLV build: its target word, push code and source field.
// On the single engine source x is node x (Philox target, written to tg for
// the round kernel; push code from the transition launch).  On a code-row
// shard it is slot key x of exchange A, read from its row (empty slot: no
// edge); its source field carries kRowMutual when the pusher is its target's
// own target (the receiver's t(y), src/message_state.rs:79).
template <bool SH>
GS_DEV void dlv_source(const InListArgs &a, uint32_t x, uint32_t &t, uint32_t &code, uint32_t &src) {
    if constexpr (SH) {
        t = kTgDead;
        code = 0u;
        src = x;
        // (this rank's own block: slots past the plan's count are empty)
        const uint32_t per = a.sr.P * a.sr.capP, ks = x / per, kr = x - ks * per, kh = kr / a.sr.capP;
        if (x < a.nkeys && (ks != a.self_rank || kr - kh * a.sr.capP < a.self_cnt[kh])) {
            const uint2 r = reinterpret_cast<const uint2 *>(a.rowsA)[shard_key_slot(a.sr, x)];
            if (r.y != 0xFFFFFFFFu) {
                t = r.y & ~kRowMutual;
                code = r.x;
                src = x | (r.y & kRowMutual);
            }
        }
    } else {
        t = target_of(a, x);
        a.tg[x] = t;
        code = a.PC[x];
        src = x;
    }
}

// A code-row shard's pull for slot key `key` into exchange B: the send
// buffer, and for this rank's own block also the receive buffer (one rank
// exchanges nothing; with several the all-to-all copies the send buffer's own
// block over the same slots).
GS_DEV void shard_pull_store(const InListArgs &a, uint32_t key, uint32_t v) {
    const uint32_t b = shard_key_bslot(a.sr, key);
    const bool own = key / (a.sr.P * a.sr.capP) == a.self_rank;
    if (own) a.pullB_self[b] = v;
    if (!own || a.sr.G > 1) a.pullB[b] = v;
}

// Per-target record emission, shared by both paths.  `lst` holds y's k
// sources ascending (LDS or global); `first` is where lst[kInline..k) are
// (already) stored in a.src.  Live-filtered gathers (a.lvm, binned path
// only): bit 31 of each lst entry is the source's live bit (kLiveTag, set by
// inl_sort), `yc` = y is complete, `yl` = y is live.  Returns the node class
// rows the records leave the round kernel to gather for y's pushers and their
// pull rows (pushers' rows, siblings' rows, t(x) rows the siblings force;
// traffic accounting, 0 unfiltered).
constexpr uint32_t kLiveTag = 1u << 31;
GS_DEV uint32_t emit_target(const InListArgs &a, uint32_t y, const uint32_t *lst, uint32_t k,
                            uint32_t first, bool yc = false, bool yl = true) {
    InRec r;
    if (k > kMaxIn) {
        atomicOr(&a.flags[2], kFlagLimit);
        k = kMaxIn;
    }
    r.kf = (first << kFirstShift) | k;
    // Live-filtered gathers (gs_common.h kSkipBit): the live bits of y's
    // first pushers; y complete (yc) creates nothing to pass on
    const bool filt = a.lvm != nullptr;
    uint32_t lv = 0;  // live bits of the first kInline pushers
    if (filt) {
#pragma unroll
        for (uint32_t i = 0; i < kInline; ++i)
            if (i < k && (lst[i] & kLiveTag)) lv |= 1u << i;
    }
#pragma unroll
    for (uint32_t i = 0; i < kInline; ++i) r.s[i] = i < k ? (lst[i] & kIdMask) : 0u;
    if (filt) r.kf |= (~lv & 7u) << kInSkipShift;  // skip flags of pushers 0..2
    a.IN8[y] = r;
    uint32_t rows = filt ? (uint32_t)__popc(lv) + (k > kInline ? k - kInline : 0u) : 0u;
    bool any_live = false;  // some pusher ahead of lst[j] is live
    for (uint32_t j = 1; j < k; ++j) {
        const uint32_t prev = j - 1u;
        any_live |= filt && (lst[prev] & kLiveTag) != 0;
        // filtered and nothing ahead of lst[j] to pass on (no live sibling, or y
        // complete): the round kernel would gather nothing from the record, so
        // it is not written (a stale serial reads as rank 0, the same result)
        const bool zneed = any_live && !yc;
        if (filt && !zneed) continue;
        if (filt)  // live siblings among the first kSibInline, the deeper ones, t(x) if forced
            rows += (uint32_t)__popc(lv & ((1u << min(j, kSibInline)) - 1u)) +
                    (j > kSibInline ? j - kSibInline : 0u) + (yl ? 0u : 1u);
        SibRec sr;
        // (filtered and written: y is incomplete, so sibling i is skipped iff
        // it is not live)
        sr.tag = ((a.serial & kSerialMask) << 8) | j | (zneed ? kSibZNeed : 0u) |
                 (filt ? ((~lv & 3u) << kSibSkipShift) : 0u);
#pragma unroll
        for (uint32_t i = 0; i < kSibInline; ++i) sr.e[i] = i < j ? (lst[i] & kIdMask) : 0u;
        if (filt && !((lv >> 2) & 1u)) sr.e[2] |= kSkipBit;
        a.SIB8[lst[j] & kIdMask] = sr;
    }
    return rows;
}

// Pushers i >= kInline of a target go to the tail array.  The binned sorts
// give every part a fixed region of it (GS_SORT_OWN_TAILS / GS_DLV_OWN_TAILS:
// tail_len per target and a block scan, no atomic); otherwise a block
// reserves the tail words of all its targets with ONE atomic (same-address
// atomics serialise at the memory side) -- then emit_tail at the thread's
// running cursor.
template <uint32_t INL = kInline>
GS_DEV uint32_t tail_len(uint32_t k) { return k > INL ? min(k, kMaxIn) - INL : 0u; }

template <uint32_t NT>
GS_DEV uint32_t reserve_tails(const InListArgs &a, uint32_t mine, uint32_t *tailcnt, uint32_t *lds_scan) {
    __shared__ uint32_t blk_first;
    uint32_t total;
    const uint32_t off = block_exclusive_scan_t<NT>(mine, lds_scan, total);
    if (threadIdx.x == 0) {
        uint32_t f = total ? atomicAdd(tailcnt, total) : 0u;
        if (f + total > a.p.tailcap) {
            atomicOr(&a.flags[2], kFlagLimit);
            f = kNone;  // no tails this round (reported as a device limit)
        }
        blk_first = f;
    }
    __syncthreads();
    return blk_first == kNone ? kNone : blk_first + off;
}

// Writes a target's tail at *cur (kNone: none reserved); returns its start.
GS_DEV uint32_t emit_tail(const InListArgs &a, const uint32_t *lst, uint32_t k, uint32_t &cur) {
    const uint32_t m = tail_len<>(k);
    if (m == 0 || cur == kNone) return 0u;
    const uint32_t first = cur;
    for (uint32_t j = 0; j < m; ++j) a.src[first + j] = lst[kInline + j] & kIdMask;
    cur += m;
    return first;
}

// ------------------------------------------------------------ binned path
// Region of bin b: 8-byte records (source, target relative to the bin) at
// region[b*kBinCap ...] (one store stream per run).  Each target is drawn once, here:
// a Philox4x32-10 draw is ~40 quarter-rate multiplies, so redrawing it in
// inl_sort would cost more than carrying 2 bytes.
template <uint32_t CHUNK>
__global__ __launch_bounds__(kInlThreads) void inl_bin(InListArgs a) {
    constexpr uint32_t kChunk = CHUNK;                 // sources of this block
    constexpr uint32_t kBinPer = kChunk / kInlThreads;  // per thread
    extern __shared__ __attribute__((aligned(16))) uint32_t sh[];
    const CsrPlan &p = a.p;
    // Per-bin state is 16-bit (every count, start and cursor is <= kChunk,
    // every reserved slot <= kBinCap): counts / cursors packed two per word for
    // LDS atomics, so 8192 bins fit beside the stage.
    uint32_t *stage = sh;                                      // [kChunk] sources by bin
    uint16_t *stage_lt = reinterpret_cast<uint16_t *>(sh + kChunk);  // [kChunk]
    // partitions: bins, or 2^sub parts per bin (small networks)
    const uint32_t np = p.nb << p.sub, plog = kBinLog - p.sub, pcap = kBinCap >> p.sub;
    uint32_t *fill = a.scratch + p.fill_off;
    uint32_t *cnt = sh + kChunk + kChunk / 2;  // [np/2] counts, then cursors (2 x u16 per word)
    uint16_t *cnt16 = reinterpret_cast<uint16_t *>(cnt);
    uint16_t *off = reinterpret_cast<uint16_t *>(cnt + (np + 1) / 2);  // [np] chunk-local starts
    uint16_t *res = off + np;                  // [np] reserved start in the part's region
    uint16_t *stage_b = res + np;              // [kChunk] part of each stage entry
    __shared__ uint32_t lds_scan[kInlThreads / 64];
    __shared__ uint32_t zrows;  // filtered: t(x) rows the zl bits leave to gather
    if (blockIdx.x == 0 && threadIdx.x == 0) a.scratch[p.nb] = 0u;  // tail count; inl_sort runs after
    if (threadIdx.x == 0) zrows = 0u;
    for (uint32_t i = threadIdx.x; i < (np + 1) / 2; i += kInlThreads) cnt[i] = 0u;
    __syncthreads();
    const uint32_t lo = blockIdx.x * kChunk;
    const uint32_t hi = min(p.n, lo + kChunk);
    // the thread's kBinPer sources lo + threadIdx.x + q * kInlThreads: targets
    // kept in registers (kTgDead past hi) for the stage pass below
    uint32_t tq[kBinPer];
#pragma unroll
    for (uint32_t q = 0; q < kBinPer; ++q) {
        const uint32_t x = lo + threadIdx.x + q * kInlThreads;
        tq[q] = kTgDead;
        if (x < hi) {
            tq[q] = target_of(a, x);
            a.tg[x] = tq[q];
            if (!(tq[q] & kTgDead)) {
                const uint32_t b = (tq[q] & kTgMask) >> plog;
                atomicAdd(&cnt[b >> 1], 1u << ((b & 1u) << 4));
            }
        }
    }
    if (a.zl) {
        // live-filtered gathers: "t(x) is live", a word per 64 sources (the
        // map lookups, L2 hits, issued together)
        bool lq[kBinPer];
#pragma unroll
        for (uint32_t q = 0; q < kBinPer; ++q) lq[q] = !(tq[q] & kTgDead) && map_test(a.lvm, tq[q] & kTgMask);
        uint32_t zr = 0;  // (wave-uniform)
#pragma unroll
        for (uint32_t q = 0; q < kBinPer; ++q) {
            const uint32_t x0 = lo + (threadIdx.x & ~63u) + q * kInlThreads;  // the wave's first source
            const u64 b = __ballot(lq[q]);
            if ((threadIdx.x & 63u) == 0u && x0 < hi) a.zl[x0 >> 6] = b;
            if (a.rows) zr += (uint32_t)__popcll(__ballot(lq[q] && !(tq[q] & kTgNoPull)));
        }
        if (a.rows && (threadIdx.x & 63u) == 0u && zr) atomicAdd(&zrows, zr);
    }
    __syncthreads();
    if (a.rows && threadIdx.x == 0 && zrows) atomicAdd(a.rows, (u64)zrows);
    // exclusive scan of the bin counts: thread i owns bins [i*per, i*per + per)
    const uint32_t per = (np + kInlThreads - 1) / kInlThreads;
    const uint32_t b0 = threadIdx.x * per;
    uint32_t sum = 0;
    for (uint32_t q = 0; q < per; ++q)
        if (b0 + q < np) sum += cnt16[b0 + q];
    uint32_t total;
    uint32_t run = block_exclusive_scan_t<kInlThreads>(sum, lds_scan, total);
    for (uint32_t q = 0; q < per; ++q) {
        const uint32_t b = b0 + q;
        if (b >= np) break;
        const uint32_t c = cnt16[b];
        off[b] = (uint16_t)run;
        uint32_t r0 = 0;
        if (c) {
            r0 = atomicAdd(&fill[b], c);
            if (r0 + c > pcap) {
                atomicOr(&a.flags[2], kFlagLimit);
                r0 = pcap;  // drop this run; the round reports the limit
            }
        }
        res[b] = (uint16_t)r0;
        cnt16[b] = (uint16_t)run;  // cursor
        run += c;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < kBinPer; ++q) {
        const uint32_t t = tq[q];
        if (t & kTgDead) continue;  // (also every slot past hi)
        const uint32_t b = (t & kTgMask) >> plog, sh16 = (b & 1u) << 4;
        const uint32_t pos = (atomicAdd(&cnt[b >> 1], 1u << sh16) >> sh16) & 0xFFFFu;
        stage[pos] = lo + threadIdx.x + q * kInlThreads;
        stage_lt[pos] = (uint16_t)(t & (kBin - 1u));  // (relative to the bin)
        stage_b[pos] = (uint16_t)b;
    }
    __syncthreads();
    // Consecutive stage entries of one part go to consecutive region slots
    // (the part of each entry is kept beside it: no search over the starts).
    for (uint32_t i = threadIdx.x; i < total; i += kInlThreads) {  // delivered edges of the chunk
        const uint32_t b = stage_b[i];
        const uint32_t slot = res[b] + (i - off[b]);
        if (slot < pcap) {
            reinterpret_cast<uint2 *>(a.region)[(u64)b * pcap + slot] = make_uint2(stage[i], stage_lt[i]);
        }
    }
}

// Packed 16-bit counter `i` of h (two per word).
GS_DEV uint32_t half_of(const uint32_t *h, uint32_t i) { return (h[i >> 1] >> ((i & 1u) << 4)) & 0xFFFFu; }

// inl_sort blocks per bin = 2^split: one while there are enough bins to fill
// the chip (two per bin measured slower at 1024 bins: every block reads the
// whole bin region), more for small networks (2^20 nodes = 64 bins), whose
// regions stay in L2.  GS_SORT_SPLIT_LOG forces one value (A/B).
#ifndef GS_SORT_THREADS
#define GS_SORT_THREADS 1024
#endif
constexpr uint32_t kSortThreads = GS_SORT_THREADS;
#ifndef GS_SORT_SMALL_LOG
#define GS_SORT_SMALL_LOG 2u  // sort blocks per bin = 2^this below 128 bins (2^21 nodes)
#endif
inline uint32_t sort_split_log(uint32_t nb) {
#ifdef GS_SORT_SPLIT_LOG
    (void)nb;
    return GS_SORT_SPLIT_LOG;
#else
    return nb >= 512u ? 0u : (nb >= 128u ? 1u : GS_SORT_SMALL_LOG);
#endif
}

// SPLITLOG > 0: 2^SPLITLOG blocks per bin (blockIdx.y = part), each sorting the
// targets of its part from the whole bin region; half the LDS, so two blocks
// share a CU (the fill counts are then cleared by the launcher, not here).
// NT threads per block (GS_SORT_THREADS, A/B): 512-thread blocks of half bins
// let two share a CU (a whole bin's 112 KiB of LDS takes one)
template <uint32_t SPLITLOG, uint32_t NT = kInlThreads>
__global__ __launch_bounds__(NT, NT == kInlThreads ? 1 : 2 * NT / 256) void inl_sort(InListArgs a) {
    constexpr uint32_t kPartLog = kBinLog - SPLITLOG;
    constexpr uint32_t kPart = 1u << kPartLog;             // targets per block
    constexpr uint32_t kPartCap = kBinCap >> SPLITLOG;     // sorted entries per block
    // SPLITLOG > 0: inl_bin wrote this part's own region (p.sub == SPLITLOG)
    constexpr bool own = SPLITLOG > 0;
    constexpr uint32_t kPer = (kPartCap + NT - 1) / NT;  // region entries per thread
    extern __shared__ __attribute__((aligned(16))) uint32_t sh[];
    const CsrPlan &p = a.p;
    uint32_t *h = sh;                   // [kPart/2] packed per-target counters
    uint32_t *sorted = sh + kPart / 2;  // [kPartCap]
    __shared__ uint32_t lds_scan[NT / 64];
    const uint32_t b = blockIdx.x, hh = blockIdx.y;
    const uint32_t cnt = own ? min(a.scratch[p.fill_off + (b << SPLITLOG) + hh], kPartCap) : min(a.scratch[b], kBinCap);
    const u64 rb = own ? (u64)((b << SPLITLOG) + hh) * kPartCap : (u64)b * kBinCap;
    const uint32_t t0 = (b << kBinLog) + (hh << kPartLog);
    const uint32_t nodes = t0 < p.n ? min(kPart, p.n - t0) : 0u;
    if (nodes == 0) return;  // a part past the last node (uniform per block)
    // the bin's entries of this part, held in registers (coalesced loads, issued first)
    uint32_t ex[kPer], el[kPer];
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q) {
        const uint32_t i = threadIdx.x + q * NT;
        const bool ok = i < cnt;
        const uint2 en = ok ? reinterpret_cast<const uint2 *>(a.region)[rb + i] : make_uint2(0u, 0u);
        ex[q] = en.x;
        const uint32_t lt = ok ? en.y : kNone;
        el[q] = (ok && (lt >> kPartLog) == hh) ? (lt & (kPart - 1u)) : kNone;
    }
    for (uint32_t i = threadIdx.x; i < kPart / 2; i += NT) h[i] = 0u;
    // live-filtered gathers: the part's "complete" bits (coalesced) and the
    // live bit of every entry (L2-resident map lookups, issued together),
    // carried as bit 31 of the sorted ids (kLiveTag)
    __shared__ uint32_t cpl[kPart / 32], lvl[kPart / 32];
    const bool filt = a.lvm != nullptr;
    uint32_t lt_tag[kPer];
    if (filt) {
        for (uint32_t i = threadIdx.x; i < kPart / 32; i += NT) {
            const bool in = t0 + 32u * i < p.n;
            cpl[i] = in ? reinterpret_cast<const uint32_t *>(a.cpm)[(t0 >> 5) + i] : 0u;
            lvl[i] = in ? reinterpret_cast<const uint32_t *>(a.lvm)[(t0 >> 5) + i] : 0u;
        }
#pragma unroll
        for (uint32_t q = 0; q < kPer; ++q)
            lt_tag[q] = (el[q] != kNone && map_test(a.lvm, ex[q])) ? kLiveTag : 0u;
    }
    __syncthreads();
    if (SPLITLOG == 0 && threadIdx.x == 0) a.scratch[b] = 0u;  // ready for the next build of this set
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q)
        if (el[q] != kNone) atomicAdd(&h[el[q] >> 1], 1u << ((el[q] & 1u) << 4));
    __syncthreads();
    // exclusive scan over the kPart targets, kPart/NT per thread
    constexpr uint32_t per = kPart / NT;
    static_assert(per >= 2 && per % 2 == 0, "the scan walks packed counter pairs: >= 2048 targets");
    const uint32_t i0 = threadIdx.x * per;
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t q = 0; q < per; ++q) sum += half_of(h, i0 + q);
    uint32_t total;
    uint32_t run = block_exclusive_scan_t<NT>(sum, lds_scan, total);
#pragma unroll
    for (uint32_t q = 0; q < per; q += 2) {
        const uint32_t c0 = half_of(h, i0 + q), c1 = half_of(h, i0 + q + 1);
        h[(i0 + q) >> 1] = run | ((run + c0) << 16);
        run += c0 + c1;
    }
    __syncthreads();
    if (SPLITLOG > 0 && threadIdx.x == 0 && total > kPartCap) atomicOr(&a.flags[2], kFlagLimit);
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q) {
        if (el[q] != kNone) {
            const uint32_t shf = (el[q] & 1u) << 4;
            const uint32_t old = atomicAdd(&h[el[q] >> 1], 1u << shf);
            const uint32_t pos = (old >> shf) & 0xFFFFu;
            if (pos < kPartCap) sorted[pos] = ex[q] | (filt ? lt_tag[q] : 0u);
        }
    }
    __syncthreads();
    // counters are now the ends of each target's run; lanes take consecutive
    // targets so the InRec stores are coalesced (an overflowing part, flagged
    // above, keeps only the entries that fit)
    auto end_of = [&](uint32_t lt) { return min(half_of(h, lt), kPartCap); };
    uint32_t mine = 0;
    for (uint32_t lt = threadIdx.x; lt < nodes; lt += NT)
        mine += tail_len<>(end_of(lt) - (lt ? end_of(lt - 1) : 0u));
    uint32_t cur;
    if (GS_SORT_OWN_TAILS) {
        // the part's own tail region (kPart / 8 slots: pushers beyond kInline
        // average 0.023 per target, so the cap is >= 25 standard deviations
        // above the mean for >= 2 K-target parts): a block scan, no atomic
        constexpr uint32_t kPartTails = kPart / 8u;
        uint32_t tot;
        const uint32_t offs = block_exclusive_scan_t<NT>(mine, lds_scan, tot);
        if (tot > kPartTails && threadIdx.x == 0) atomicOr(&a.flags[2], kFlagLimit);
        cur = tot > kPartTails ? kNone : ((b << SPLITLOG) + hh) * kPartTails + offs;
    } else {
        cur = reserve_tails<NT>(a, mine, &a.scratch[p.nb], lds_scan);
    }
    uint32_t rows = 0;  // filtered: class rows left to gather (traffic accounting)
    for (uint32_t lt = threadIdx.x; lt < nodes; lt += NT) {
        const uint32_t e = end_of(lt);
        const uint32_t s = lt ? end_of(lt - 1) : 0u;
        uint32_t *lst = sorted + s;
        const uint32_t k = e - s;
        for (uint32_t q = 1; q < k; ++q) {  // Poisson(1)-sized: insertion sort (by id)
            const uint32_t v = lst[q];
            uint32_t r = q;
            while (r > 0 && (lst[r - 1] & kIdMask) > (v & kIdMask)) {
                lst[r] = lst[r - 1];
                --r;
            }
            lst[r] = v;
        }
        const bool yc = filt && ((cpl[lt >> 5] >> (lt & 31u)) & 1u) != 0;
        const bool yl = filt && ((lvl[lt >> 5] >> (lt & 31u)) & 1u) != 0;
        rows += emit_target(a, t0 + lt, lst, k, emit_tail(a, lst, k, cur), yc, yl);
    }
    if (a.rows) {
        uint32_t total;
        (void)block_exclusive_scan_t<NT>(rows, lds_scan, total);
        if (threadIdx.x == 0 && total) atomicAdd(a.rows, (u64)total);
    }
}

// ------------------------------------------------------------ DLV path
// The delivery-record build partitions (source, local target, push code)
// entries in two levels, so every partition writes long runs (a single level
// over ~6000 bins of 16 K targets wrote ~3-entry runs, twice the bytes):
//   dl_coarse : per chunk of kPartChunk sources: Philox targets (-> tg), push
//               codes (coalesced), an LDS counting sort into coarse buckets of
//               2^kCoarseLog targets (kCoarseBins bins each), runs of ~170
//   dl_fine   : per chunk of a coarse bucket: an LDS counting sort into its
//               kCoarseBins bins of kBin targets, runs of ~64, into the bin
//               regions inl_sort_dlv reads
#ifndef GS_COARSE_BINS
#define GS_COARSE_BINS 128
#endif
constexpr uint32_t kCoarseBins = GS_COARSE_BINS;  // bins per coarse bucket (a power of two)
constexpr uint32_t ilog2c(uint32_t v) { return v <= 1u ? 0u : 1u + ilog2c(v >> 1); }
static_assert((kCoarseBins & (kCoarseBins - 1u)) == 0 && kCoarseBins <= 256, "coarse bins: a power of two <= 256");
constexpr uint32_t kCoarseLog = kBinLog + ilog2c(kCoarseBins);
constexpr uint32_t kCoarseCap = (1u << kCoarseLog) + (1u << (kCoarseLog - 4));
// Each coarse bucket is split into kCoarseShards sub-regions with fill
// counters of their own (the partitioning block b reserves in shard b % S):
// every block makes one returning atomic per bucket, and on one counter word
// those serialise at the memory side (~88 per us, MI355X_MICROARCH.md
// "dequeue").  dl_coarse's ~24 K blocks showed no queueing on 48 words (A/B
// with 1 / 4 / 8 shards within noise); the transition launch that partitions
// in its epilogue has 8x more blocks.
#ifndef GS_COARSE_SHARDS
#define GS_COARSE_SHARDS 8
#endif
constexpr uint32_t kCoarseShards = GS_COARSE_SHARDS;
constexpr uint32_t kShardCap = kCoarseCap / kCoarseShards;
static_assert(kCoarseCap % kCoarseShards == 0, "whole shards");
#ifndef GS_PART_CHUNK
#define GS_PART_CHUNK 4096
#endif
constexpr uint32_t kPartChunk = GS_PART_CHUNK;
#ifndef GS_COARSE_THREADS
#define GS_COARSE_THREADS 1024
#endif
constexpr uint32_t kCoarseThreads = GS_COARSE_THREADS;
constexpr uint32_t kPartPer = kPartChunk / kInlThreads;
constexpr uint32_t kMaxCoarse = 1u << (27 - kCoarseLog);  // n <= 2^27

__host__ __device__ inline uint32_t n_coarse(uint32_t nb) { return (nb + kCoarseBins - 1) / kCoarseBins; }
// DLV scratch: fill[nb], tail count, pull coarse fills [nc], pull bin fills
// [nb], the part fills (fill_off, when sub > 0), then the coarse shard fills
// [nc * S] last: the transition launch that partitions into a set reserves in
// them while it clears the rest of that set's counters (RoundArgs::cp_*).
__host__ __device__ inline uint32_t pcfill_off(uint32_t nb) { return nb + 1u; }
__host__ __device__ inline uint32_t pffill_off(uint32_t nb) { return pcfill_off(nb) + n_coarse(nb); }
__host__ __device__ inline uint32_t dlv_head_words(uint32_t nb) { return pffill_off(nb) + nb; }
__host__ __device__ inline uint32_t cfill_off(const CsrPlan &p) {
    return dlv_head_words(p.nb) + (p.sub ? (p.nb << p.sub) : 0u);
}
__host__ __device__ inline uint32_t dlv_scratch_words(const CsrPlan &p) {
    return cfill_off(p) + n_coarse(p.nb) * kCoarseShards;
}

#ifndef GS_DLV_SPLIT_LOG
#define GS_DLV_SPLIT_LOG 2
#endif
// sort blocks per bin = 2^kSplitLog (n >= 2^21): quarter bins, whose 48 KiB of
// LDS let two 1024-thread blocks share a CU (half bins took 96 KiB, so a CU's
// loads and LDS work took turns: inl_sort_dlv 1.52 -> 1.09 ms, config 5
// 5.19 -> 4.76 ms/step, profiles/r3/cfg5_build)
constexpr uint32_t kSplitLog = GS_DLV_SPLIT_LOG;
#ifndef GS_DLV_SMALL_LOG
#define GS_DLV_SMALL_LOG (kSplitLog + 1u)  // below 128 bins (one coarse bucket, cache-resident)
#endif
constexpr uint32_t kDlvSmallLog = GS_DLV_SMALL_LOG;
// DLV partition entries are 12-byte records, one store stream per run: a
// coarse entry (source, target, push code), a part entry (source, push code,
// target within the bin).  (Three u32 / u16 arrays made three scattered
// segments per run: dl_fine's runs are ~8 entries.)
struct PEnt {
    uint32_t a, b, c;
};
// The bin (part) regions: [nb * kBinCap] part entries at the region base.
__host__ __device__ inline PEnt *part_entries(uint32_t *region) { return reinterpret_cast<PEnt *>(region); }
constexpr size_t kDlvRegionWords = 3;  // u32 words per part slot
// The single engine's entries are 8 bytes, (source, push code): a consumer
// draws the source's target again (one Philox draw, peer_of) instead of
// reading it -- the target is a counter-based function of (round, source).
// Code-row shards keep 12-byte entries (their targets come with the rows).
[[maybe_unused]] __host__ __device__ inline uint2 *part_entries8(uint32_t *region) { return reinterpret_cast<uint2 *>(region); }
// Coarse-bucket entries inside the region buffer, after the bin regions.
__host__ __device__ inline PEnt *coarse_entries(uint32_t *region, uint32_t nb) {
    return reinterpret_cast<PEnt *>(region + (size_t)nb * kBinCap * kDlvRegionWords);
}
__host__ __device__ inline uint2 *coarse_entries8(uint32_t *region, uint32_t nb) {
    return reinterpret_cast<uint2 *>(region + (size_t)nb * kBinCap * kDlvRegionWords);
}

// Pull pass-back arrays, after the coarse buckets: per coarse source bucket
// 2^kCoarseLog (pusher, pull) slots (a source appears at most once), then per
// source bin kBin (local pusher u16, pull) slots.
struct PullArrays {
    uint32_t *x, *v;
    uint16_t *fx;
    uint32_t *fv;
};
__host__ __device__ inline size_t pull_words(uint32_t nb) {
    const size_t nc = (nb + kCoarseBins - 1) / kCoarseBins;
    return 2 * (nc << kCoarseLog) + (size_t)nb * kBin * 3 / 2;
}
__host__ __device__ inline PullArrays pull_arrays(uint32_t *region, uint32_t nb) {
    const size_t nc = (nb + kCoarseBins - 1) / kCoarseBins;
    uint32_t *base = region + (size_t)nb * kBinCap * kDlvRegionWords + 3 * nc * kCoarseCap;
    const size_t pc = nc << kCoarseLog;
    return PullArrays{base, base + pc, reinterpret_cast<uint16_t *>(base + 2 * pc),
                      base + 2 * pc + (size_t)nb * kBin / 2};
}

// NT threads per block (GS_COARSE_THREADS): 512 lets three blocks share a CU;
// SH: a code-row shard's build (sources = slot keys, dlv_source)
template <uint32_t NT, bool SH = false>
__global__ __launch_bounds__(NT) void dl_coarse(InListArgs a) {
    constexpr uint32_t kPer = kPartChunk / NT;
    static_assert(kPartChunk % NT == 0 && kMaxCoarse <= NT, "dl_coarse: whole sources, a scan slot per bucket");
    extern __shared__ __attribute__((aligned(16))) uint32_t sh[];
    uint32_t *sx = sh, *st = sh + kPartChunk, *sc = sh + 2 * kPartChunk;
    __shared__ uint32_t cnt[kMaxCoarse], off[kMaxCoarse], res[kMaxCoarse + 1];
    const CsrPlan &p = a.p;
    const uint32_t nc = n_coarse(p.nb);
    const uint32_t shard = blockIdx.x % kCoarseShards;
    uint32_t *cfill = a.scratch + cfill_off(p);
    PEnt *ce = coarse_entries(a.region, p.nb);
    for (uint32_t i = threadIdx.x; i < nc; i += NT) cnt[i] = 0u;
    __syncthreads();
    const uint32_t lo = blockIdx.x * kPartChunk;
    uint32_t tv[kPer], cv[kPer], xs[kPer];
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q) {
        const uint32_t x = lo + threadIdx.x + q * NT;
        tv[q] = kTgDead;
        cv[q] = 0u;
        xs[q] = x;
        if (x < p.n) {
            dlv_source<SH>(a, x, tv[q], cv[q], xs[q]);
            if (!(tv[q] & kTgDead)) atomicAdd(&cnt[(tv[q] & kTgMask) >> kCoarseLog], 1u);
        }
    }
    __syncthreads();
    {  // exclusive scan of the nc <= 64 bucket counts; one reservation per bucket
        __shared__ uint32_t lds_scan[NT / 64];
        const uint32_t c = threadIdx.x < nc ? cnt[threadIdx.x] : 0u;
        uint32_t total;
        const uint32_t ex = block_exclusive_scan_t<NT>(c, lds_scan, total);
        if (threadIdx.x < nc) {
            off[threadIdx.x] = ex;
            uint32_t r0 = c ? atomicAdd(&cfill[threadIdx.x * kCoarseShards + shard], c) : 0u;
            if (r0 + c > kShardCap) {
                atomicOr(&a.flags[2], kFlagLimit);
                r0 = kShardCap;
            }
            res[threadIdx.x] = r0;
            cnt[threadIdx.x] = ex;  // cursor
        }
        if (threadIdx.x == 0) res[kMaxCoarse] = total;  // entries of the chunk
    }
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q) {
        if (tv[q] & kTgDead) continue;
        const uint32_t t = tv[q] & kTgMask;
        const uint32_t pos = atomicAdd(&cnt[t >> kCoarseLog], 1u);
        sx[pos] = SH ? xs[q] : lo + threadIdx.x + q * NT;
        st[pos] = t;
        sc[pos] = cv[q];
    }
    __syncthreads();
    const uint32_t total = res[kMaxCoarse];
    for (uint32_t i = threadIdx.x; i < total; i += NT) {
        const uint32_t b = st[i] >> kCoarseLog;
        const uint32_t slot = res[b] + (i - off[b]);
        if (slot < kShardCap) {
            const u64 o = (u64)(b * kCoarseShards + shard) * kShardCap + slot;
            if constexpr (SH) ce[o] = PEnt{sx[i], st[i], sc[i]};
            else coarse_entries8(a.region, p.nb)[o] = make_uint2(sx[i], sc[i]);
        }
    }
}

constexpr uint32_t kMaxFineSub = 2;
#ifndef GS_FINE_THREADS
#define GS_FINE_THREADS 1024
#endif
constexpr uint32_t kFineThreads = GS_FINE_THREADS;
#ifndef GS_FINE_CHUNK
#define GS_FINE_CHUNK 4096  // coarse-bucket entries per dl_fine block
#endif
constexpr uint32_t kFineChunk = GS_FINE_CHUNK;
constexpr uint32_t kFineParts = kCoarseBins << kMaxFineSub;  // parts per coarse bucket (sub <= 2)
// NT threads per block (GS_FINE_THREADS): 512 lets three blocks share a CU
template <uint32_t NT, bool SH = false>
__global__ __launch_bounds__(NT) void dl_fine(InListArgs a) {
    constexpr uint32_t kPer = kFineChunk / NT;
    static_assert(kFineChunk % NT == 0 && kFineParts <= NT, "dl_fine: whole entries, a scan slot per part");
    extern __shared__ __attribute__((aligned(16))) uint32_t sh[];
    uint32_t *sx = sh, *sc = sh + kFineChunk;
    uint16_t *slt = reinterpret_cast<uint16_t *>(sh + 2 * kFineChunk);
    uint16_t *sb = slt + kFineChunk;  // part of each stage entry
    __shared__ uint32_t cnt[kFineParts];
    __shared__ uint16_t off[kFineParts], res[kFineParts];  // (<= kFineChunk, <= pcap: 16 bits)
    static_assert(kFineChunk <= 65535u && kBinCap <= 65535u, "16-bit starts");
    __shared__ uint32_t lds_scan[NT / 64];
    const CsrPlan &p = a.p;
    // the 2^sub parts of each bin inl_sort_dlv sorts: a coarse bucket's
    // kCoarseBins << sub parts, each in its own region of kBinCap >> sub slots
    const uint32_t fp = kCoarseBins << p.sub, plog = kBinLog - p.sub, pcap = kBinCap >> p.sub;
    uint32_t *pfill = p.sub ? a.scratch + p.fill_off : a.scratch;
    const uint32_t cs = blockIdx.y, cb = cs / kCoarseShards;  // (coarse bucket, shard)
    const uint32_t fill = min(a.scratch[cfill_off(p) + cs], kShardCap);
    const uint32_t lo = blockIdx.x * kFineChunk;
    if (lo >= fill) return;  // uniform per block
    const uint32_t hi = min(fill, lo + kFineChunk);
    const PEnt *ce = coarse_entries(a.region, p.nb);
    PEnt *pe = part_entries(a.region);
    if (threadIdx.x < fp) cnt[threadIdx.x] = 0u;
    __syncthreads();
    uint32_t xv[kPer], tv[kPer], cv[kPer];
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q) {
        const uint32_t i = lo + threadIdx.x + q * NT;
        const bool ok = i < hi;
        const u64 o = (u64)cs * kShardCap + (ok ? i : lo);
        if constexpr (SH) {
            const PEnt en = ce[o];
            xv[q] = en.a;
            tv[q] = ok ? en.b : kNone;
            cv[q] = en.c;
        } else {  // (source, push code): the target drawn again
            const uint2 en = coarse_entries8(const_cast<uint32_t *>(a.region), p.nb)[o];
            xv[q] = en.x;
            cv[q] = en.y;
            tv[q] = ok ? peer_of(a.seed, a.epoch, a.round, en.x, p.n) : kNone;
        }
        if (ok) atomicAdd(&cnt[(tv[q] >> plog) & (fp - 1u)], 1u);
    }
    __syncthreads();
    {  // exclusive scan of the part counts, reservations in the part regions
        const uint32_t c = threadIdx.x < fp ? cnt[threadIdx.x] : 0u;
        uint32_t total;
        const uint32_t ex = block_exclusive_scan_t<NT>(c, lds_scan, total);
        if (threadIdx.x < fp) {
            const uint32_t b = cb * fp + threadIdx.x;
            off[threadIdx.x] = (uint16_t)ex;
            uint32_t r0 = c ? atomicAdd(&pfill[b], c) : 0u;
            if (r0 + c > pcap) {
                atomicOr(&a.flags[2], kFlagLimit);
                r0 = pcap;
            }
            res[threadIdx.x] = (uint16_t)r0;
            cnt[threadIdx.x] = ex;  // cursor
        }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q) {
        if (tv[q] == kNone) continue;
        const uint32_t fb = (tv[q] >> plog) & (fp - 1u);
        const uint32_t pos = atomicAdd(&cnt[fb], 1u);
        sx[pos] = xv[q];
        sc[pos] = cv[q];
        slt[pos] = (uint16_t)(tv[q] & (kBin - 1u));  // (relative to the bin)
        sb[pos] = (uint16_t)fb;
    }
    __syncthreads();
    const uint32_t n_here = hi - lo;
    for (uint32_t i = threadIdx.x; i < n_here; i += NT) {
        const uint32_t lo_b = sb[i];
        const uint32_t slot = res[lo_b] + (i - off[lo_b]);
        if (slot < pcap) {
            const u64 o = (u64)(cb * fp + lo_b) * pcap + slot;
            if constexpr (SH) pe[o] = PEnt{sx[i], sc[i], slt[i]};
            else part_entries8(a.region)[o] = make_uint2(sx[i], sc[i]);
        }
    }
}

// Small networks (one coarse bucket, n <= kCoarseBins bins): the targets and
// one LDS counting sort of each chunk of sources straight into the regions of
// the 2^sub parts of every bin that inl_sort_dlv sorts (dl_coarse + dl_fine in
// one pass; the regions stay in cache at this size).
constexpr uint32_t kDirectParts = kInlThreads;  // nb << sub <= 1024 (one scan slot per part)
template <bool SH = false>
__global__ __launch_bounds__(kInlThreads) void dl_direct(InListArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t sh[];
    uint32_t *sx = sh, *sc = sh + kPartChunk;
    uint16_t *slt = reinterpret_cast<uint16_t *>(sh + 2 * kPartChunk);
    uint16_t *sb = slt + kPartChunk;
    __shared__ uint32_t cnt[kDirectParts], off[kDirectParts], res[kDirectParts + 1];
    __shared__ uint32_t lds_scan[kInlThreads / 64];
    const CsrPlan &p = a.p;
    const uint32_t np = p.nb << p.sub, plog = kBinLog - p.sub, pcap = kBinCap >> p.sub;
    uint32_t *fill = a.scratch + p.fill_off;
    for (uint32_t i = threadIdx.x; i < np; i += kInlThreads) cnt[i] = 0u;
    __syncthreads();
    const uint32_t lo = blockIdx.x * kPartChunk;
    uint32_t tv[kPartPer], cv[kPartPer], xs[kPartPer];
#pragma unroll
    for (uint32_t q = 0; q < kPartPer; ++q) {
        const uint32_t x = lo + threadIdx.x + q * kInlThreads;
        tv[q] = kTgDead;
        cv[q] = 0u;
        xs[q] = x;
        if (x < p.n) {
            dlv_source<SH>(a, x, tv[q], cv[q], xs[q]);
            if (!(tv[q] & kTgDead)) atomicAdd(&cnt[(tv[q] & kTgMask) >> plog], 1u);
        }
    }
    __syncthreads();
    {
        const uint32_t c = threadIdx.x < np ? cnt[threadIdx.x] : 0u;
        uint32_t total;
        const uint32_t ex = block_exclusive_scan_t<kInlThreads>(c, lds_scan, total);
        if (threadIdx.x < np) {
            off[threadIdx.x] = ex;
            uint32_t r0 = c ? atomicAdd(&fill[threadIdx.x], c) : 0u;
            if (r0 + c > pcap) {
                atomicOr(&a.flags[2], kFlagLimit);
                r0 = pcap;
            }
            res[threadIdx.x] = r0;
            cnt[threadIdx.x] = ex;  // cursor
        }
        if (threadIdx.x == 0) res[kDirectParts] = total;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < kPartPer; ++q) {
        if (tv[q] & kTgDead) continue;
        const uint32_t t = tv[q] & kTgMask, b = t >> plog;
        const uint32_t pos = atomicAdd(&cnt[b], 1u);
        sx[pos] = SH ? xs[q] : lo + threadIdx.x + q * kInlThreads;
        sc[pos] = cv[q];
        slt[pos] = (uint16_t)(t & (kBin - 1u));  // (relative to the bin)
        sb[pos] = (uint16_t)b;
    }
    __syncthreads();
    const uint32_t total = res[kDirectParts];
    for (uint32_t i = threadIdx.x; i < total; i += kInlThreads) {
        const uint32_t b = sb[i];
        const uint32_t slot = res[b] + (i - off[b]);
        if (slot < pcap) {
            // (small networks, eighth-bin parts: 12-byte entries with the
            // target, so their sort draws no targets; the regions stay in L2)
            if (SH || p.sub == kDlvSmallLog) part_entries(a.region)[(u64)b * pcap + slot] = PEnt{sx[i], sc[i], slt[i]};
            else part_entries8(a.region)[(u64)b * pcap + slot] = make_uint2(sx[i], sc[i]);
        }
    }
}

// DLV: the records of one HALF of a bin (kHalf targets; blockIdx.y picks the
// half) from the bin's region: an LDS counting sort of (id, push code) pairs
// by target, per target an insertion sort by id, the DlvRec and its tails;
// then, per pusher in order, the pull batch the target returns
// (Gossip::receive, src/gossip.rs:124-151: the target's live set plus what it
// created from the pushers ahead), partitioned by the pusher's coarse source
// bucket for the pull pass-back (pb_fine, pb_place).  Halving the bin keeps
// ids and codes in LDS.
// Small networks (few bins) sort with more blocks per bin, so the chip fills;
// their bin regions stay in L2 (config 2: 64 bins).
inline uint32_t dlv_split_log(uint32_t nb) { return nb >= 128u ? kSplitLog : kDlvSmallLog; }

template <uint32_t SL, bool OWN, bool SH = false>
// (own quarter-bin regions: two blocks per CU, 48 KiB of LDS and
// <= 64 VGPRs each; the second bound is waves per SIMD)
__global__ __launch_bounds__(kInlThreads, (SL == 2 && OWN) ? 8 : 1) void inl_sort_dlv(InListArgs a) {
    constexpr uint32_t kHalfLog = kBinLog - SL;  // (a "half": one of the 2^SL parts of a bin)
    constexpr uint32_t kHalf = 1u << kHalfLog;
    constexpr uint32_t kHalfCap = kBinCap >> SL;
    constexpr uint32_t kHalfPer = kHalf / kInlThreads;  // targets per thread
    static_assert(kHalfPer >= 2 && kHalfPer % 2 == 0, "the scan walks packed counter pairs: >= 2048 targets");
    // region entries per thread: the half's own region (OWN: p.sub == SL) or the whole bin's
    constexpr uint32_t kPer = ((OWN ? kHalfCap : kBinCap) + kInlThreads - 1) / kInlThreads;
    extern __shared__ __attribute__((aligned(16))) uint32_t sh[];
    const CsrPlan &p = a.p;
    uint32_t *h = sh;                   // [kHalf/2] packed per-target counters
    uint32_t *sid = sh + kHalf / 2;     // [kHalfCap] source ids by target
    uint32_t *scd = sid + kHalfCap;     // [kHalfCap] their push codes, then their pulls
    __shared__ uint32_t lds_scan[kInlThreads / 64];
    __shared__ uint32_t pcnt[kMaxCoarse], pres[kMaxCoarse];
    const uint32_t nc = n_coarse(p.nb);
    // tail slots each part owns (dlv_part_tails; DlvRec::mf holds the offset)
    constexpr uint32_t kPartTails = (kBin >> SL) / 4u + (kBin >> SL) / 16u;
    // p.sub == SL: dl_fine / dl_direct wrote this half's own region; small
    // networks (one coarse bucket) write every pull straight to PULL (no
    // pass-back partition)
    constexpr bool own = OWN;
    const bool direct = nc == 1u;
    uint32_t *pcfill = a.scratch + pcfill_off(p.nb);
    const PullArrays pa = pull_arrays(a.region, p.nb);
    // part w = (bin b, half hh) = w >> SL, w & (2^SL - 1)
    const uint32_t w = (blockIdx.x << SL) + blockIdx.y;
    uint32_t ex[kPer], ec[kPer], el[kPer];
    auto load_part = [&](uint32_t wp) {
        const uint32_t bp = wp >> SL, hp = wp & ((1u << SL) - 1u);
        const uint32_t cnt = own ? min(a.scratch[p.fill_off + wp], kHalfCap) : min(a.scratch[bp], kBinCap);
        const u64 rb = own ? (u64)wp * kHalfCap : (u64)bp * kBinCap;
#pragma unroll
        for (uint32_t q = 0; q < kPer; ++q) {
            const uint32_t i = threadIdx.x + q * kInlThreads;
            const bool ok = i < cnt;
            uint32_t lt;
            if constexpr (SH || SL == kDlvSmallLog) {  // (12-byte entries, dl_direct)
                const PEnt en = part_entries(a.region)[rb + (ok ? i : 0u)];
                lt = en.c;
                ex[q] = en.a;
                ec[q] = en.b;
            } else {  // (source, push code): the target is the source's Philox draw again
                const uint2 en = part_entries8(a.region)[rb + (ok ? i : 0u)];
                ex[q] = en.x;
                ec[q] = en.y;
                lt = peer_of(a.seed, a.epoch, a.round, en.x, p.n) & (kBin - 1u);
            }
            if (!ok) lt = kNone;
            el[q] = (ok && (lt >> kHalfLog) == hp) ? (lt & (kHalf - 1u)) : kNone;
        }
    };
    // the targets' own target words and what their planes say about the
    // pull batches they return: on the single engine the push code and the
    // known mask the round kernel wrote (PC, KN: 6 B per target), on a
    // code-row shard the class planes (R_pad <= 16: a node's segment lies in
    // one 32-bit half of its plane word; whole 128-B record lines)
    uint32_t tgv[kHalfPer];
    uint32_t w0[kHalfPer], w1[kHalfPer], w2[kHalfPer];  // SH: planes 0-2; else w0 = PC, w1 = KN
    const uint32_t *S32 = reinterpret_cast<const uint32_t *>(a.S);
    // (code-row shard: targets are the ntargets local nodes, p.n may be
    // larger -- the slot keys -- and t(y)'s pusher is flagged in its row)
    const uint32_t ny = SH ? a.ntargets : p.n;
    auto load_targets = [&](uint32_t wp) {
        const uint32_t t0p = wp << kHalfLog;
        const uint32_t np = t0p < ny ? min(kHalf, ny - t0p) : 0u;
#pragma unroll
        for (uint32_t q = 0; q < kHalfPer; ++q) {
            const uint32_t lt = threadIdx.x + q * kInlThreads;
            const uint32_t y = np ? t0p + (lt < np ? lt : 0u) : 0u;  // (a part past the last node: node 0)
            const uint32_t ysh = (y & ((1u << a.g.lognpu) - 1u)) << a.g.logr;
            const u64 rb = (u64)(y >> a.g.lognpu) * kPlanes * 2u + (ysh >> 5);
            if constexpr (SH) {
                tgv[q] = 0u;
                w0[q] = S32[rb];
                w1[q] = S32[rb + 2];
                w2[q] = S32[rb + 4];
            } else {
                tgv[q] = a.tg[y];
                w0[q] = a.PC[y];
                w1[q] = a.KN[y];
                w2[q] = 0u;
                (void)rb;
            }
        }
    };
    load_part(w);
    const uint32_t t0 = w << kHalfLog;
    const uint32_t nodes = t0 < p.n ? min(kHalf, p.n - t0) : 0u;
    if (nodes == 0) return;  // a half past the last node (uniform per block)
    for (uint32_t i = threadIdx.x; i < kHalf / 2; i += kInlThreads) h[i] = 0u;
    if (threadIdx.x < kMaxCoarse) pcnt[threadIdx.x] = 0u;
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q)
        if (el[q] != kNone) atomicAdd(&h[el[q] >> 1], 1u << ((el[q] & 1u) << 4));
    __syncthreads();
    const uint32_t i0 = threadIdx.x * kHalfPer;
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t q = 0; q < kHalfPer; ++q) sum += half_of(h, i0 + q);
    uint32_t total;
    uint32_t run = block_exclusive_scan_t<kInlThreads>(sum, lds_scan, total);
#pragma unroll
    for (uint32_t q = 0; q < kHalfPer; q += 2) {
        const uint32_t c0 = half_of(h, i0 + q), c1 = half_of(h, i0 + q + 1);
        h[(i0 + q) >> 1] = run | ((run + c0) << 16);
        run += c0 + c1;
    }
    __syncthreads();
    if (threadIdx.x == 0 && total > kHalfCap) atomicOr(&a.flags[2], kFlagLimit);
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q) {
        if (el[q] != kNone) {
            const uint32_t shf = (el[q] & 1u) << 4;
            const uint32_t pos = (atomicAdd(&h[el[q] >> 1], 1u << shf) >> shf) & 0xFFFFu;
            if (pos < kHalfCap) {
                sid[pos] = ex[q];
                scd[pos] = ec[q];
            }
        }
    }
    __syncthreads();
    load_targets(w);
    uint32_t mine = 0;
    for (uint32_t lt = threadIdx.x; lt < nodes; lt += kInlThreads)
        mine += tail_len<kDlvInline>(min(half_of(h, lt), kHalfCap) - (lt ? min(half_of(h, lt - 1), kHalfCap) : 0u));
    uint32_t cur;
    if (own && GS_DLV_OWN_TAILS) {  // the part's own tail region (dlv_part_tails): a block scan, no atomic
        uint32_t tot;
        const uint32_t offs = block_exclusive_scan_t<kInlThreads>(mine, lds_scan, tot);
        if (tot > kPartTails && threadIdx.x == 0) atomicOr(&a.flags[2], kFlagLimit);
        cur = tot > kPartTails ? kNone : w * kPartTails + offs;
    } else {
        cur = reserve_tails<kInlThreads>(a, mine, &a.scratch[p.nb], lds_scan);
    }
    const uint32_t m = (uint32_t)((1ull << a.g.rpad) - 1ull);
#pragma unroll
    for (uint32_t q = 0; q < kHalfPer; ++q) {
        const uint32_t lt = threadIdx.x + q * kInlThreads;
        if (lt >= nodes) break;
        const uint32_t e = min(half_of(h, lt), kHalfCap);
        const uint32_t s = lt ? min(half_of(h, lt - 1), kHalfCap) : 0u;
        uint32_t k = e - s;
        for (uint32_t j = s + 1; j < e; ++j) {  // insertion sort of (id, code) by id
            const uint32_t v = sid[j], vc = scd[j];
            uint32_t r = j;
            while (r > s && (SH ? (sid[r - 1] & kIdMask) > (v & kIdMask) : sid[r - 1] > v)) {  // (SH: bit 31 kRowMutual)
                sid[r] = sid[r - 1];
                scd[r] = scd[r - 1];
                --r;
            }
            sid[r] = v;
            scd[r] = vc;
        }
        if (k > kMaxIn) {
            atomicOr(&a.flags[2], kFlagLimit);
            k = kMaxIn;
        }
        const uint32_t tz = tgv[q] & kTgMask;  // t(y): did it push to y?
        const uint32_t mt = tail_len<kDlvInline>(k);
        const uint32_t first = (mt && cur != kNone) ? cur : 0u;
        uint32_t zi = kDlvNoZ;
        for (uint32_t j = 0; j < k; ++j) {
            if (SH ? (sid[s + j] & kRowMutual) != 0u : sid[s + j] == tz) zi = j;
            if (j >= kDlvInline && cur != kNone) a.dtail[first + j - kDlvInline] = scd[s + j];
        }
        if (mt && cur != kNone) cur += mt;
        DlvRec r;
        // (+ y's own delivery flags for the packed round kernel, which then
        // reads no target word: bit 10 no pull reaches y, bit 11 y offline;
        // and the tail offset within the part's own region, kDlvFirstShift)
        r.mf = k | (zi << 5) | (((tgv[q] >> 30) & 1u) << kDlvMetaNoPull) | (((tgv[q] >> 29) & 1u) << kDlvMetaOff) |
               ((first - (first ? w * kPartTails : 0u)) << kDlvFirstShift);
        r.c[0] = k > 0 ? scd[s] : 0u;
        r.c[1] = k > 1 ? scd[s + 1] : 0u;
        a.DR[t0 + lt] = r;
        // the pull batch of each pusher, in place of its push code: y's live
        // set (B with our_counter, C as 255) plus the entries y created from
        // the pushers ahead of it (first carrier B -> counter 1, C -> 255)
        // y's own pull base: the push code of its planes (B counter 1 -> 01,
        // counter 2 -> 10, C -> 11; the same as the round kernel's PC[y]) and
        // the rumors it does not know (state A)
        uint32_t y0, y1, pnot;
        if constexpr (SH) {
            const uint32_t ysh = (((t0 + lt) & ((1u << a.g.lognpu) - 1u)) << a.g.logr) & 31u;
            const uint32_t c = (w0[q] >> ysh) & m, a0 = (w1[q] >> ysh) & m, a1 = (w2[q] >> ysh) & m;
            const uint32_t zB = ~c & (a0 | a1), zC = c & ~(a0 & a1);
            y0 = (zB & a0 & ~a1) | zC;
            y1 = (zB & a1 & ~a0) | zC;
            pnot = ~c & ~a0 & ~a1 & m;
        } else {
            y0 = w0[q] & 0xFFFFu;
            y1 = w0[q] >> 16;
            pnot = ~w1[q] & m;
        }
        uint32_t pB = 0, pC = 0;
        for (uint32_t j = s; j < e; ++j) {  // (entries past kMaxIn keep the clamped pulls)
            const uint32_t code = scd[j];
            scd[j] = ((y0 | pB | pC) & 0xFFFFu) | ((y1 | pC) << 16);
            const uint32_t b0 = code & 0xFFFFu, b1 = code >> 16;
            const uint32_t vC = b0 & b1, sl = b0 | b1;  // the pusher's batch; C carries 255
            const uint32_t nw = pnot & sl;
            pB |= nw & ~vC;
            pC |= nw & vC;
            pnot &= ~sl;
            // an empty pull batch is not passed back: PULL[] reads 0 for it
            if (!direct && scd[j]) atomicAdd(&pcnt[(SH ? sid[j] & kIdMask : sid[j]) >> kCoarseLog], 1u);
        }
    }
    __syncthreads();
    if (direct) {  // one coarse bucket: every pull straight into PULL (cache-resident)
        const uint32_t placed = min(total, kHalfCap);
        if constexpr (SH) {  // a code-row shard: to the pusher's exchange-B slot
            for (uint32_t j = threadIdx.x; j < placed; j += kInlThreads) {
                shard_pull_store(a, sid[j] & kIdMask, scd[j]);
            }
        } else {
            for (uint32_t j = threadIdx.x; j < placed; j += kInlThreads) a.pull[sid[j]] = scd[j];
        }
        return;
    }
    // the (pusher, pull) pairs into the pushers' coarse source buckets
    if (threadIdx.x < nc) {
        const uint32_t c = pcnt[threadIdx.x];
        pres[threadIdx.x] = c ? atomicAdd(&pcfill[threadIdx.x], c) : 0u;
        pcnt[threadIdx.x] = 0u;  // cursor
    }
    __syncthreads();
    const uint32_t placed = min(total, kHalfCap);
    for (uint32_t j = threadIdx.x; j < placed; j += kInlThreads) {
        if (!scd[j]) continue;  // empty pull (pb_place zero-fills)
        const uint32_t x = SH ? sid[j] & kIdMask : sid[j], cb = x >> kCoarseLog;
        const uint32_t slot = pres[cb] + atomicAdd(&pcnt[cb], 1u);  // < 2^kCoarseLog: one per source
        const u64 o = ((u64)cb << kCoarseLog) + slot;
        pa.x[o] = x;
        pa.v[o] = scd[j];
    }
}

// Pull pass-back, level 2: per chunk of a coarse source bucket, an LDS
// counting sort of (pusher, pull) pairs into its kCoarseBins source bins.
__global__ __launch_bounds__(kInlThreads) void pb_fine(InListArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t sh[];
    uint32_t *sv = sh;
    uint16_t *sx = reinterpret_cast<uint16_t *>(sh + kPartChunk);
    uint8_t *sb = reinterpret_cast<uint8_t *>(sh + kPartChunk + kPartChunk / 2);
    __shared__ uint32_t cnt[kCoarseBins], off[kCoarseBins], res[kCoarseBins];
    __shared__ uint32_t lds_scan[kInlThreads / 64];
    const CsrPlan &p = a.p;
    const uint32_t cb = blockIdx.y;
    const uint32_t fill = min(a.scratch[pcfill_off(p.nb) + cb], 1u << kCoarseLog);
    const uint32_t lo = blockIdx.x * kPartChunk;
    if (lo >= fill) return;  // uniform per block
    const uint32_t hi = min(fill, lo + kPartChunk);
    const PullArrays pa = pull_arrays(a.region, p.nb);
    uint32_t *pffill = a.scratch + pffill_off(p.nb);
    if (threadIdx.x < kCoarseBins) cnt[threadIdx.x] = 0u;
    __syncthreads();
    uint32_t xv[kPartPer], vv[kPartPer];
#pragma unroll
    for (uint32_t q = 0; q < kPartPer; ++q) {
        const uint32_t i = lo + threadIdx.x + q * kInlThreads;
        const bool ok = i < hi;
        const u64 o = ((u64)cb << kCoarseLog) + (ok ? i : lo);
        xv[q] = ok ? pa.x[o] : kNone;
        vv[q] = pa.v[o];
        if (ok) atomicAdd(&cnt[(xv[q] >> kBinLog) & (kCoarseBins - 1u)], 1u);
    }
    __syncthreads();
    {
        const uint32_t c = threadIdx.x < kCoarseBins ? cnt[threadIdx.x] : 0u;
        uint32_t tot;
        const uint32_t ex = block_exclusive_scan_t<kInlThreads>(c, lds_scan, tot);
        if (threadIdx.x < kCoarseBins) {
            off[threadIdx.x] = ex;
            res[threadIdx.x] = c ? atomicAdd(&pffill[cb * kCoarseBins + threadIdx.x], c) : 0u;  // < kBin
            cnt[threadIdx.x] = ex;  // cursor
        }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < kPartPer; ++q) {
        if (xv[q] == kNone) continue;
        const uint32_t fb = (xv[q] >> kBinLog) & (kCoarseBins - 1u);
        const uint32_t pos = atomicAdd(&cnt[fb], 1u);
        sv[pos] = vv[q];
        sx[pos] = (uint16_t)(xv[q] & (kBin - 1u));
        sb[pos] = (uint8_t)fb;
    }
    __syncthreads();
    const uint32_t n_here = hi - lo;
    for (uint32_t i = threadIdx.x; i < n_here; i += kInlThreads) {
        const uint32_t fb = sb[i];
        const u64 o = (u64)(cb * kCoarseBins + fb) * kBin + res[fb] + (i - off[fb]);
        pa.fx[o] = sx[i];
        pa.fv[o] = sv[i];
    }
}

// Pull pass-back, level 3: per source bin, the pulls into an LDS image of
// PULL[bin], written out coalesced.  Only non-empty pull batches are passed
// back (while a dissemination is young most pulls are empty): a slot nobody
// wrote is an empty pull, or one not delivered this round, which the round
// kernel ignores.
template <bool SH = false>
__global__ __launch_bounds__(kInlThreads) void pb_place(InListArgs a) {
    __shared__ uint32_t img[kBin];
    const CsrPlan &p = a.p;
    const uint32_t b = blockIdx.x;
    const uint32_t cnt = min(a.scratch[pffill_off(p.nb) + b], kBin);
    const PullArrays pa = pull_arrays(a.region, p.nb);
    for (uint32_t i = threadIdx.x; i < kBin; i += kInlThreads) img[i] = 0u;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < cnt; i += kInlThreads) {
        const u64 o = (u64)b * kBin + i;
        img[pa.fx[o]] = pa.fv[o];
    }
    __syncthreads();
    const uint32_t x0 = b << kBinLog;
    if constexpr (SH) {  // a code-row shard: sources are slot keys, pulls go to their exchange-B slots
        const uint32_t keys = x0 < a.nkeys ? min(kBin, a.nkeys - x0) : 0u;
        for (uint32_t i = threadIdx.x; i < keys; i += kInlThreads)
            shard_pull_store(a, x0 + i, img[i]);
        return;
    }
    const uint32_t nodes = min(kBin, p.n - x0);
    for (uint32_t i = threadIdx.x; i < nodes; i += kInlThreads) a.pull[x0 + i] = img[i];
}

// ------------------------------------------------------------ generic path
// Two-stage counting sort of the n edges (x -> tg[x]) by target through an
// exact CSR (src[n]), for networks beyond the binned path's bin count:
//   bin_count   : per source chunk, an LDS histogram over target bins -> M
//   col_scan    : per bin, exclusive prefix over chunks; bin totals
//   scan_small  : exclusive prefix of the bin totals -> bin bases
//   bin_scatter : (local target, source) pairs into their bin's range
//   bin_sort    : per bin, LDS counting sort by local target -> src[] with each
//                 node's sources ascending, then the records
__global__ __launch_bounds__(256) void csr_bin_count(InListArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
    const CsrPlan &p = a.p;
    for (uint32_t i = threadIdx.x; i < p.nb; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    const u64 lo = (u64)blockIdx.x * p.chunk;
    const u64 hi = min((u64)p.n, lo + p.chunk);
    for (u64 x = lo + threadIdx.x; x < hi; x += blockDim.x) {
        const uint32_t t = target_of(a, (uint32_t)x);
        a.tg[x] = t;
        if (!(t & kTgDead)) atomicAdd(&hist[(t & kTgMask) >> p.logbin], 1u);
    }
    __syncthreads();
    uint32_t *M = a.scratch;
    for (uint32_t i = threadIdx.x; i < p.nb; i += blockDim.x) M[(u64)blockIdx.x * p.nb + i] = hist[i];
    if (blockIdx.x == 0 && threadIdx.x == 0) a.scratch[(size_t)p.ba * p.nb + 2 * (size_t)p.nb] = 0u;  // tails
}

__global__ __launch_bounds__(256) void csr_col_scan(InListArgs a) {
    const CsrPlan &p = a.p;
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.nb) return;
    uint32_t *M = a.scratch;
    uint32_t *tot = M + (size_t)p.ba * p.nb;
    uint32_t run = 0;
    for (uint32_t c = 0; c < p.ba; ++c) {
        const uint32_t v = M[(u64)c * p.nb + b];
        M[(u64)c * p.nb + b] = run;
        run += v;
    }
    tot[b] = run;
}

// Exclusive scan of the bin totals (one block).
__global__ __launch_bounds__(kScanBlock) void csr_scan_small(InListArgs a) {
    __shared__ uint32_t lds[kScanBlock / 64];
    const CsrPlan &p = a.p;
    const uint32_t *in = a.scratch + (size_t)p.ba * p.nb;
    uint32_t *out = a.scratch + (size_t)p.ba * p.nb + p.nb;
    uint32_t carry = 0;
    for (uint32_t base = 0; base < p.nb; base += kScanBlock) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < p.nb ? in[i] : 0u;
        uint32_t tot;
        const uint32_t ex = block_exclusive_scan(v, lds, tot);
        if (i < p.nb) out[i] = carry + ex;
        carry += tot;
    }
}

__global__ __launch_bounds__(256) void csr_bin_scatter(InListArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t cur[];
    const CsrPlan &p = a.p;
    const uint32_t *M = a.scratch;
    const uint32_t *base = a.scratch + (size_t)p.ba * p.nb + p.nb;
    u64 *pairs = reinterpret_cast<u64 *>(a.region);
    for (uint32_t i = threadIdx.x; i < p.nb; i += blockDim.x) cur[i] = base[i] + M[(u64)blockIdx.x * p.nb + i];
    __syncthreads();
    const u64 lo = (u64)blockIdx.x * p.chunk;
    const u64 hi = min((u64)p.n, lo + p.chunk);
    const uint32_t lm = p.bin - 1u;
    for (u64 x = lo + threadIdx.x; x < hi; x += blockDim.x) {
        const uint32_t t = a.tg[x];
        if (t & kTgDead) continue;
        const uint32_t pos = atomicAdd(&cur[(t & kTgMask) >> p.logbin], 1u);
        pairs[pos] = ((u64)(t & lm) << 32) | (uint32_t)x;
    }
}

__global__ __launch_bounds__(256) void csr_bin_sort(InListArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t h[];  // [bin] + 16 scan words
    const CsrPlan &p = a.p;
    const u64 *pairs = reinterpret_cast<const u64 *>(a.region);
    uint32_t *csr = a.region + 2 * (size_t)p.n;  // exact CSR of the round's edges
    const uint32_t *tot = a.scratch + (size_t)p.ba * p.nb;
    const uint32_t *base = tot + p.nb;
    uint32_t *tailcnt = a.scratch + (size_t)p.ba * p.nb + 2 * (size_t)p.nb;
    uint32_t *lds_scan = h + p.bin;
    const uint32_t b = blockIdx.x;
    const uint32_t start = base[b], cnt = tot[b];
    const uint32_t nb0 = b << p.logbin;
    const uint32_t nodes = min(p.bin, p.n - nb0);
    for (uint32_t i = threadIdx.x; i < p.bin; i += blockDim.x) h[i] = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) atomicAdd(&h[pairs[start + i] >> 32], 1u);
    __syncthreads();
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
        csr[start + pos] = (uint32_t)pr;
    }
    __syncthreads();
    uint32_t mine = 0;
    for (uint32_t i = threadIdx.x; i < nodes; i += blockDim.x) mine += tail_len<>(h[i] - (i ? h[i - 1] : 0u));
    uint32_t cur = reserve_tails<256>(a, mine, tailcnt, lds_scan);
    for (uint32_t i = threadIdx.x; i < nodes; i += blockDim.x) {
        const uint32_t s = start + (i ? h[i - 1] : 0u), e = start + h[i];
        uint32_t *lst = csr + s;
        const uint32_t k = e - s;
        for (uint32_t q = 1; q < k; ++q) {
            const uint32_t v = lst[q];
            uint32_t r = q;
            while (r > 0 && lst[r - 1] > v) {
                lst[r] = lst[r - 1];
                --r;
            }
            lst[r] = v;
        }
        emit_target(a, nb0 + i, lst, k, emit_tail(a, lst, k, cur));
    }
}

// Test hook: SAFE_GOSSIP_AMD_GENERIC_INLISTS=1 forces the generic path.
bool getenv_generic_inlists() {
    const char *v = std::getenv("SAFE_GOSSIP_AMD_GENERIC_INLISTS");
    return v && *v && *v != '0';
}

}  // namespace

// Tail slots of one own sort part (kBin >> sub targets): pushers beyond
// kDlvInline average 3/e - 1 = 0.104 per target with a variance of ~0.15, so
// kHalf * 5/16 is 25-35 standard deviations above the mean (2048-4096
// targets); the sort blocks then need no shared tail counter (one returning
// atomic per block on one word queued ~6 us behind 512 small-network blocks).
inline uint32_t dlv_part_tails(uint32_t sub) {
    const uint32_t half = kBin >> sub;
    return half / 4u + half / 16u;
}

void dlv_tail_parts(const CsrPlan &p, uint32_t *log, uint32_t *per) {
    *log = kBinLog - p.sub;
    *per = dlv_part_tails(p.sub);
}

CsrPlan dlv_plan(uint32_t n) {
    CsrPlan p{};
    p.n = n;
    const uint32_t nb_binned = (uint32_t)(((u64)n + kBin - 1) / kBin);
    if (nb_binned > kBinnedMaxBins || getenv_generic_inlists()) return p;  // binned == 0: no DLV path
    p.binned = 1;
    p.dlv = 1;
    p.bin = kBin;
    p.logbin = kBinLog;
    p.nb = nb_binned;
    p.ba = (uint32_t)(((u64)n + kPartChunk - 1) / kPartChunk);  // dl_coarse blocks
    p.chunk = kPartChunk;
    // pushers beyond kDlvInline: E[max(k - 2, 0)] = 3/e - 1 = 10.4 % of n
    p.tailcap = n / 8u + 4096u;  // (the tails hold push codes only: src_words = tailcap)
    // the partition writes the sort blocks' parts (one coarse bucket:
    // dl_direct; dl_fine: at most two parts per bin)
    const uint32_t nc = n_coarse(p.nb);
    p.sub = dlv_split_log(p.nb);
    if (nc > 1u && p.sub > kMaxFineSub) p.sub = 0u;  // (kFineParts)
    p.fill_off = p.sub ? dlv_head_words(p.nb) : 0u;  // after fill[nb], tailcnt, pull fills
    // own parts: a fixed tail region per part (dlv_part_tails), no shared counter
    if (p.sub && GS_DLV_OWN_TAILS) p.tailcap = (uint32_t)std::min<u64>((u64)(p.nb << p.sub) * dlv_part_tails(p.sub), 0xFFFFFFFFu);
    return p;
}

CsrPlan csr_plan(uint32_t n) {
    CsrPlan p{};
    p.n = n;
    const uint32_t nb_binned = (uint32_t)(((u64)n + kBin - 1) / kBin);
    if (nb_binned <= kBinnedMaxBins && !getenv_generic_inlists()) {
        p.binned = 1;
        p.bin = kBin;
        p.logbin = kBinLog;
        p.nb = nb_binned;
        // small networks: shorter chunks, so the partition fills the chip
        // (2^20 nodes: 512 blocks instead of 128)
        p.chunk = n >= (1u << 22) ? kChunk : kChunkSmall;
        p.ba = (uint32_t)(((u64)n + p.chunk - 1) / p.chunk);
        // GS_SORT_OWN_TAILS: kBin / 8 tail slots per bin, split over its parts
        p.tailcap = GS_SORT_OWN_TAILS ? nb_binned * (kBin / 8u) : n / 32u + 1024u;
        // several sort blocks per bin: inl_bin partitions into their parts
        p.sub = sort_split_log(p.nb);
        p.fill_off = p.sub ? p.nb + 1 : 0u;  // after fill[nb], tailcnt
        return p;
    }
    uint32_t bin = 4096;
    while ((u64)bin * 16384u < n) bin <<= 1;  // <= 16384 bins: bin_count LDS <= 64 KiB
    p.bin = bin;
    p.logbin = 0;
    while ((1u << p.logbin) < bin) ++p.logbin;
    p.nb = (uint32_t)(((u64)n + bin - 1) / bin);
    uint32_t ba = (uint32_t)(((u64)n + 4095) / 4096);
    p.ba = ba < 256u ? (ba ? ba : 1u) : 256u;
    p.chunk = (uint32_t)(((u64)n + p.ba - 1) / p.ba);
    p.tailcap = n / 32u + 1024u;
    return p;
}

// The counters a binned build needs cleared before it runs, as one range of
// scratch (words == 0: none; the whole-bin sort clears its own).
void inlist_zero_range(const CsrPlan &p, size_t *first, size_t *words) {
    *first = 0;
    *words = 0;
    if (!p.binned) return;
    if (p.dlv) {
        *words = cfill_off(p);  // the coarse fills are cleared a round later (inlist_cfill_range)
    } else if (p.sub) {
        *first = p.fill_off;
        *words = (size_t)p.nb << p.sub;
    }
}

void inlist_cfill_range(const CsrPlan &p, size_t *first, size_t *words) {
    *first = p.dlv && p.binned ? cfill_off(p) : 0u;
    *words = p.dlv && p.binned ? (size_t)n_coarse(p.nb) * kCoarseShards : 0u;
}


InListSizes inlist_sizes(const CsrPlan &p) {
    InListSizes z{};
    if (p.binned) {
        z.src_words = p.tailcap;  // ids (or DLV: push codes) of the in-list tails
        // sources (u32) + local targets (u16) [+ push codes (u32) + the coarse buckets]
        // (gather path: 8-byte (source, target within the bin) records)
        z.region_words = p.dlv ? (size_t)p.nb * kBinCap * kDlvRegionWords : (size_t)p.nb * kBinCap * 2;
        const size_t nc = (p.nb + kCoarseBins - 1) / kCoarseBins;
        if (p.dlv) z.region_words += 3 * nc * kCoarseCap + pull_words(p.nb);
        // fill[nb], tailcnt[, coarse fill[nc], pull coarse fill[nc], pull bin fill[nb]]
        if (p.dlv) {
            z.scratch_words = dlv_scratch_words(p);
        } else {
            z.scratch_words = (size_t)p.nb + 1;
            if (p.sub) z.scratch_words = (size_t)p.fill_off + ((size_t)p.nb << p.sub);  // part fills
        }
    } else {
        z.src_words = p.tailcap;
        z.region_words = 3 * (size_t)p.n;  // u64 pairs + the CSR
        z.scratch_words = (size_t)p.ba * p.nb + 2 * (size_t)p.nb + 1;  // M, tot, base, tail count
    }
    return z;
}

// The DLV build (binned plan, p.dlv): partitions, the part sorts with the
// records and pulls, the pull pass-back.  SH: a code-row shard's build.
template <bool SH>
hipError_t launch_dlv_build(const InListArgs &a, hipStream_t s) {
    const CsrPlan &p = a.p;
    const uint32_t dsl = dlv_split_log(p.nb);
    const size_t lds_dlv = ((size_t)(kBin >> dsl) / 2 + 2 * (size_t)(kBinCap >> dsl)) * sizeof(uint32_t);
    const bool own = p.sub != 0u;
    // the records index their tails within their part's own region
    // (DlvRec::mf): whole-bin regions and a shared tail counter (A/B
    // variants) would need global tail indices
    if (!own || !GS_DLV_OWN_TAILS) return hipErrorInvalidValue;
    const void *kd = dsl == kSplitLog ? (const void *)inl_sort_dlv<kSplitLog, true, SH>
                                      : (const void *)inl_sort_dlv<kDlvSmallLog, true, SH>;
    hipError_t e = hipFuncSetAttribute(kd, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_dlv);
    if (e != hipSuccess) return e;
    if (a.lvm || a.zl) return hipErrorInvalidValue;  // DLV records gather nothing
    if (SH && (!a.rowsA || !a.pullB || !a.pullB_self || !a.self_cnt || a.nkeys > p.n || a.ntargets > p.n))
        return hipErrorInvalidValue;
    InListArgs ab = a;
    // fill counts (both half-bin blocks of a bin read them, so they are
    // cleared here rather than by the sort), tail count, coarse fills
    const uint32_t nc = (p.nb + kCoarseBins - 1) / kCoarseBins;
    if (!a.prezeroed) e = hipMemsetAsync(a.scratch, 0, inlist_sizes(p).scratch_words * sizeof(uint32_t), s);
    const size_t lds_c = 3 * (size_t)kPartChunk * sizeof(uint32_t);
    const size_t lds_f = 3 * (size_t)kFineChunk * sizeof(uint32_t);
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void *)dl_coarse<kCoarseThreads, SH>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds_c);
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void *)dl_fine<kFineThreads, SH>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds_f);
    if (e != hipSuccess) return e;
    const bool direct = nc == 1u;  // small n: one pass into the parts, pulls written directly
    if ((p.sub && p.sub != dsl) || (direct && (!p.sub || (p.nb << p.sub) > kDirectParts)) ||
        (!direct && p.sub > kMaxFineSub))
        return hipErrorInvalidValue;
    if (direct) {
        const size_t lds_d = (2 * (size_t)kPartChunk + kPartChunk) * sizeof(uint32_t);
        e = hipFuncSetAttribute((const void *)dl_direct<SH>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_d);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(dl_direct<SH>, dim3(p.ba), dim3(kInlThreads), lds_d, s, ab);
    } else {
        hipLaunchKernelGGL((dl_coarse<kCoarseThreads, SH>), dim3(p.ba), dim3(kCoarseThreads), lds_c, s, ab);
        hipLaunchKernelGGL((dl_fine<kFineThreads, SH>), dim3((kShardCap + kFineChunk - 1) / kFineChunk, nc * kCoarseShards),
                           dim3(kFineThreads), lds_f, s, ab);
    }
    void *kargs[] = {&ab};
    e = hipLaunchKernel(kd, dim3(p.nb, 1u << dsl), dim3(kInlThreads), kargs, lds_dlv, s);
    if (e != hipSuccess) return e;
    const size_t lds_pb = ((size_t)kPartChunk + kPartChunk / 2 + kPartChunk / 4) * sizeof(uint32_t);
    e = hipFuncSetAttribute((const void *)pb_fine, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_pb);
    if (e != hipSuccess) return e;
    if (!direct) {
        hipLaunchKernelGGL(pb_fine, dim3((1u << kCoarseLog) / kPartChunk, nc), dim3(kInlThreads), lds_pb, s, ab);
        hipLaunchKernelGGL(pb_place<SH>, dim3(p.nb), dim3(kInlThreads), 0, s, ab);
    }
    return hipGetLastError();
}

hipError_t launch_build_inlists(const InListArgs &a, hipStream_t s) {
    const CsrPlan &p = a.p;
    if (p.n == 0) return hipSuccess;
    if (p.binned && p.dlv) return a.rowsA ? launch_dlv_build<true>(a, s) : launch_dlv_build<false>(a, s);
    if (a.rowsA) return hipErrorInvalidValue;  // code-row shards build delivery records only
    if (p.binned) {
        const uint32_t np = p.nb << p.sub;
        const size_t lds_bin = ((size_t)p.chunk + p.chunk / 2 + (np + 1) / 2) * sizeof(uint32_t) +
                               ((size_t)2 * np + p.chunk) * sizeof(uint16_t);
        const void *kb = p.chunk == kChunk ? (const void *)inl_bin<kChunk> : (const void *)inl_bin<kChunkSmall>;
        const uint32_t sl = sort_split_log(p.nb);
        const size_t lds_sort = ((size_t)(kBin >> sl) / 2 + (kBinCap >> sl)) * sizeof(uint32_t);
        const void *ks = sl == 0   ? (const void *)inl_sort<0, kSortThreads>
                         : sl == 1 ? (const void *)inl_sort<1, kSortThreads>
                         : sl == 2 ? (const void *)inl_sort<2, kSortThreads>
                                   : (const void *)inl_sort<3, kSortThreads>;
        hipError_t e = hipFuncSetAttribute(kb, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bin);
        if (e == hipSuccess) e = hipFuncSetAttribute(ks, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_sort);
        if (e != hipSuccess) return e;
        if ((a.lvm == nullptr) != (a.zl == nullptr) || (a.lvm && !a.cpm)) return hipErrorInvalidValue;
        InListArgs ab = a;
        if (sl > 0) {  // the split sort cannot clear the fill counts itself
            if (p.sub != sl) return hipErrorInvalidValue;
            if (!a.prezeroed)
                e = hipMemsetAsync(a.scratch + p.fill_off, 0, ((size_t)p.nb << p.sub) * sizeof(uint32_t), s);
            if (e != hipSuccess) return e;
        }
        if (p.chunk == kChunk) hipLaunchKernelGGL(inl_bin<kChunk>, dim3(p.ba), dim3(kInlThreads), lds_bin, s, ab);
        else hipLaunchKernelGGL(inl_bin<kChunkSmall>, dim3(p.ba), dim3(kInlThreads), lds_bin, s, ab);
        const dim3 gs(p.nb, 1u << sl);
        if (sl == 0) hipLaunchKernelGGL((inl_sort<0, kSortThreads>), gs, dim3(kSortThreads), lds_sort, s, ab);
        else if (sl == 1) hipLaunchKernelGGL((inl_sort<1, kSortThreads>), gs, dim3(kSortThreads), lds_sort, s, ab);
        else if (sl == 2) hipLaunchKernelGGL((inl_sort<2, kSortThreads>), gs, dim3(kSortThreads), lds_sort, s, ab);
        else hipLaunchKernelGGL((inl_sort<3, kSortThreads>), gs, dim3(kSortThreads), lds_sort, s, ab);
        return hipGetLastError();
    }
    // the generic path writes no skip flags (live-filtered gathers are binned only)
    if (a.lvm || a.zl) return hipErrorInvalidValue;
    const size_t lds_nb = (size_t)p.nb * sizeof(uint32_t);
    hipLaunchKernelGGL(csr_bin_count, dim3(p.ba), dim3(256), lds_nb, s, a);
    hipLaunchKernelGGL(csr_col_scan, dim3((p.nb + 255) / 256), dim3(256), 0, s, a);
    hipLaunchKernelGGL(csr_scan_small, dim3(1), dim3(kScanBlock), 0, s, a);
    hipLaunchKernelGGL(csr_bin_scatter, dim3(p.ba), dim3(256), lds_nb, s, a);
    const size_t lds_sort = ((size_t)p.bin + 16) * sizeof(uint32_t);
    if (lds_sort > 65536) {  // n > 2^28: bins of 32768 nodes need 128 KiB of the 160 KiB LDS
        hipError_t e = hipFuncSetAttribute((const void *)csr_bin_sort,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_sort);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(csr_bin_sort, dim3(p.nb), dim3(256), lds_sort, s, a);
    return hipGetLastError();
}

}  // namespace gs
