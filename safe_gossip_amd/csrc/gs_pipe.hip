// gs_pipe.hip -- the pipelined round kernel of the wide 2P gather path
// (R_pad = 128 / 256 / 512: W = 2 / 4 / 8 words of 64 rumors per node), the
// bench path of config 4.
//
// Same per-lane work as round_kernel<false, MODE 0/1> (gs_kernels.hip): one
// lane per (node x, 64-rumor word j) receives round t at x (Gossip::receive
// of every push batch and of the pull batch, src/gossip.rs:118-163), then
// runs phase 0 of round t+1 (src/gossip.rs:71-113,
// src/message_state.rs:86-171).  What differs is the latency structure.
// round_kernel makes each wave wait for two dependent memory levels per tile
// of 64 nodes: the coalesced per-node records (own planes, IN/SIB/tg/zl,
// Statistics), then the random class-row gathers they address.  Here a
// persistent block walks tiles bid, bid + grid, ... and the whole first level
// of tile i+1 is copied into LDS by LDS-DMA (global_load_lds_dwordx4: no
// registers) while tile i's gathers are in flight, so a tile costs ONE memory
// latency (gathers and the next tile's records together) plus its compute:
//
//   B1 barrier  | tile i's records (DMA'd during tile i-1) -> registers
//               | issue tile i's gathers; issue the DMA of tile i+1
//               | absorb, transition (waits for the gathers and the DMA)
//   B2 barrier  | round-(t+1) planes -> LDS (swizzled)
//   B3 barrier  | 16-B nontemporal stores of the tile, Statistics
//
// LDS: two buffers of {planes 4W KiB, IN 1 KiB, SIB 1 KiB, Statistics 1 KiB,
// tg 256 B, zl, eadd}; 39.5 KiB per block at W = 4 (four blocks per CU).  The
// plane image is plane-major (plane p = the tile's words in lane order), built
// through the DMA's per-lane SOURCE addresses (the LDS side of an LDS-DMA is
// lane-linear): a lane reads and writes its eight plane words at one base
// address plus immediate offsets, conflict-free (round_kernel's node-major
// image is an 8-way conflict, 208 LDS conflict cycles per wave at config 4).
#include <algorithm>

#include "gs_kernels.h"
#include "gs_device.h"
#include "gs_recv.h"

namespace gs {

template <uint32_t W>
struct PipeTile {
    static constexpr uint32_t kNodes = kPipeTileNodes;     // nodes per tile (a zl word)
    static constexpr uint32_t kThreads = kNodes * W;       // one lane per (node, word)
    static constexpr uint32_t kLogW = W == 2 ? 1u : (W == 4 ? 2u : 3u);
    static constexpr uint32_t kNodeSlots = 4u * W;         // 16-B plane slots of a node record
    static constexpr uint32_t kSlots = kNodes * kNodeSlots;
    // plane-major image: plane p = the tile's kThreads words in lane order,
    // planes kPlaneStride bytes apart (the pad staggers the banks of the
    // store pass's 16-B reads, which walk one node's record across planes)
    static constexpr uint32_t kPlaneBytes = kThreads * 8u;
    static constexpr uint32_t kPlaneStride = kPlaneBytes + (W == 8 ? 64u : 32u);
    static constexpr uint32_t oIN = kPlanes * kPlaneStride;  // InRec [64]
    static constexpr uint32_t oSIB = oIN + kNodes * 16u;   // SibRec [64]
    static constexpr uint32_t oST = oSIB + kNodes * 16u;   // u32 Statistics deltas [64][4]
    static constexpr uint32_t oTG = oST + kNodes * 16u;    // target words [64]
    static constexpr uint32_t oZL = oTG + kNodes * 4u;     // the tile's zl word (64 lanes x 4 B copies)
    static constexpr uint32_t oEA = oZL + 256u;            // rumor slices: eadd [64] (2 B)
    static constexpr uint32_t kBuf = oEA + kNodes * 2u;
    static constexpr uint32_t oAny = 2u * kBuf;            // block any-live flag
    static constexpr uint32_t kLds = oAny + 16u;
    static_assert(W == 2 || W == 4 || W == 8, "wide path: W = 2, 4 or 8");
    static_assert(kPlaneBytes % 1024u == 0u, "plane DMA in whole wave-instructions");
    // LDS byte offset of global 16-B slot s of tile node xl (the store pass)
    static GS_DEV uint32_t slot_lds(uint32_t xl, uint32_t s) {
#ifdef GS_PIPE_NODEMAJOR
        return (xl * kNodeSlots + (s ^ swz(xl))) * 16u;
#else
        const uint32_t p = s >> (kLogW - 1u), h = s & (W / 2u - 1u);
        return p * kPlaneStride + (xl * W + 2u * h) * 8u;
#endif
    }
    // LDS byte offset of plane word p of lane (xl, j)
    static GS_DEV uint32_t word_lds(uint32_t tid, uint32_t p) {
#ifdef GS_PIPE_NODEMAJOR
        const uint32_t xl = tid >> kLogW, q = p * W + (tid & (W - 1u));
        return (xl * kNodeSlots + ((q >> 1) ^ swz(xl))) * 16u + (q & 1u) * 8u;
#else
        return p * kPlaneStride + tid * 8u;
#endif
    }
    // node-major image (GS_PIPE_NODEMAJOR): slot s of node xl at s ^ swz(xl)
    static GS_DEV uint32_t swz(uint32_t xl) {
        if constexpr (W == 2) return (xl >> 1) & 7u;
        else if constexpr (W == 4) return (xl << 1) & 14u;
        else return (xl << 2) & 12u;
    }
};

// One LDS-DMA wave-instruction: lane l copies SZ bytes from its own global
// address to lds + l * SZ (lds wave-uniform).
template <uint32_t SZ>
GS_DEV void lds_dma(const void *src, uint8_t *lds) {
    auto *l = (__attribute__((address_space(3))) void *)lds;
    static_assert(SZ == 2 || SZ == 4 || SZ == 16, "LDS-DMA widths used here");
    if constexpr (SZ == 16) __builtin_amdgcn_global_load_lds(src, l, 16, 0, 0);
    else if constexpr (SZ == 4) __builtin_amdgcn_global_load_lds(src, l, 4, 0, 0);
    else __builtin_amdgcn_global_load_lds(src, l, 2, 0, 0);
}

// Class planes (isC, a0, a1) of node s, word j (records [node][plane][W]).
template <uint32_t W>
GS_DEV Cls load_cls_w(const u64 *__restrict__ S, uint32_t s, uint32_t j) {
    const u64 b = (u64)s * (kPlanes * W) + j;
    return Cls{S[b], S[b + W], S[b + 2 * W]};
}

// First-level records of tile t into LDS buffer buf, by LDS-DMA: the waves of
// the block share the wave-instructions (plane slots first, then one per
// record array).  Every array is padded to whole tiles (gs_engine.cpp), so
// the last tile reads past n without clamping; only the caller-owned eadd
// (rumor slices) is clamped.
template <uint32_t W, bool DELIVER, bool FILT>
GS_DEV void pipe_issue(const RoundArgs &a, uint32_t t, uint8_t *buf, uint32_t wv, uint32_t lane) {
    using T = PipeTile<W>;
    constexpr uint32_t lw = T::kLogW, perp = T::kPlaneBytes / 1024u;  // wave-instructions per plane
    const uint32_t node0 = t * T::kNodes;
    const uint4 *S4 = reinterpret_cast<const uint4 *>(a.Scur) + (u64)node0 * T::kNodeSlots;
#pragma unroll
    for (uint32_t i = 0; i < kPlanes * perp / W; ++i) {
        const uint32_t ins = wv + i * W;
#ifdef GS_PIPE_NODEMAJOR
        const uint32_t L = ins * 64u + lane;  // LDS slot: node xl, slot s ^ swz(xl)
        const uint32_t xl = L >> (lw + 2u), s = L & (T::kNodeSlots - 1u);
        lds_dma<16>(S4 + xl * T::kNodeSlots + (s ^ T::swz(xl)), buf + ins * 1024u);
#else
        const uint32_t p = ins / perp, h = ins % perp;  // plane p, 1-KiB piece h of it
        const uint32_t r = h * 64u + lane;  // 16-B slot of the plane image: words 2r, 2r + 1
        const uint32_t node = r >> (lw - 1u), slot = p * (W / 2u) + (r & (W / 2u - 1u));
        lds_dma<16>(S4 + node * T::kNodeSlots + slot, buf + p * T::kPlaneStride + h * 1024u);
#endif
    }
    const uint32_t node = node0 + lane;
    if (DELIVER) {
        if (wv == 0u % W) lds_dma<16>(a.IN8 + node, buf + T::oIN);
        if (wv == 1u % W) lds_dma<16>(a.SIB8 + node, buf + T::oSIB);
        if (wv == 3u % W) lds_dma<4>(a.tg + node, buf + T::oTG);
        if (FILT && wv == 4u % W)
            lds_dma<4>(reinterpret_cast<const uint32_t *>(a.zlm) + 2u * t + (lane & 1u), buf + T::oZL);
    }
    if (wv == 2u % W) lds_dma<16>(reinterpret_cast<const uint4 *>(a.st32) + node, buf + T::oST);
    if (a.eadd && wv == 5u % W)
        lds_dma<2>(reinterpret_cast<const uint16_t *>(a.eadd) + min(node, a.g.n - 1u), buf + T::oEA);
}

template <uint32_t W, int MODE, bool FILT>
__global__ __launch_bounds__(PipeTile<W>::kThreads) void round_pipe(RoundArgs a, uint32_t ntiles) {
    using T = PipeTile<W>;
    constexpr bool DELIVER = MODE == 1;
    constexpr uint32_t lw = T::kLogW;
    __shared__ __attribute__((aligned(16))) uint8_t lds[T::kLds];
    const Geometry &g = a.g;
    const uint32_t tid0 = threadIdx.x;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid0 >> 6);
    const u64 *__restrict__ S = a.Scur;
    uint32_t *blk_any = reinterpret_cast<uint32_t *>(lds + T::oAny);
    if (a.zero_buf || a.zero_rows) zero_for_build(a.zero_buf, a.zero_words, a.zero_rows);
    if (a.zero_buf2) zero_for_build(a.zero_buf2, a.zero_words2, nullptr);
    if (tid0 == 0) *blk_any = 0u;
    if (blockIdx.x == 0 && tid0 == 0) {
        // slot of round t, read by the host already
        __hip_atomic_store(&a.flags[(a.round_new + 1u) & 1u], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // traffic accounting of timed launches: the class rows this round's
        // build left to gather (counted there, off the kernel's path)
        if (MODE == 1 && a.acct && a.rows_cnt) atomicAdd(a.acct, *a.rows_cnt);
    }
    uint32_t t = blockIdx.x;
    uint32_t b = 0;
    pipe_issue<W, DELIVER, FILT>(a, t, lds, wv, tid0 & 63u);
    for (; t < ntiles; t += gridDim.x, b ^= 1u) {
        // lane coordinates, opaque to the compiler so that it recomputes the
        // addresses derived from them per tile instead of holding them in
        // registers across the loop
        uint32_t tid = tid0;
        asm volatile("" : "+v"(tid));
        const uint32_t lane = tid & 63u, xl = tid >> lw, j = tid & (W - 1u);
        uint8_t *buf = lds + b * T::kBuf;
        // B1: every wave's DMA of tile t has landed (__syncthreads waits its
        // own), and no wave still reads buffer b ^ 1 (tile t - grid's stores)
        __syncthreads();
        const uint32_t x = t * T::kNodes + xl;
        const bool valid = x < g.n;
        const u64 seg = (u64)x * W + j;
        u64 P[kPlanes];
#pragma unroll
        for (uint32_t p = 0; p < (uint32_t)kPlanes; ++p)
            P[p] = *reinterpret_cast<const u64 *>(buf + T::word_lds(tid, p));

        // ---- first level (from LDS) and the gathers it addresses
        InRec in8 = {};
        SibRec sb8 = {};
        uint32_t tgw = 0, z = x, k = 0, r = 0, qskip = 0, eskip = 0;
        bool zneed = false, zlive = false;
        if (DELIVER) {
            in8 = *reinterpret_cast<const InRec *>(buf + T::oIN + xl * 16u);
            sb8 = *reinterpret_cast<const SibRec *>(buf + T::oSIB + xl * 16u);
            tgw = *reinterpret_cast<const uint32_t *>(buf + T::oTG + xl * 4u);
            z = tgw & kTgMask;
            k = valid ? in8.k() : 0u;
            const bool sib_ok = valid && (sb8.tag >> 8) == (a.serial & kSerialMask);
            r = sib_ok ? (sb8.tag & kSibRankMask) : 0u;
            if (FILT) {
                // live-filtered gathers: the skip flags (gs_common.h)
                const u64 zlw = *reinterpret_cast<const u64 *>(buf + T::oZL);
                zlive = ((zlw >> xl) & 1ull) != 0;
                qskip = in8.kf >> kInSkipShift;
                in8.kf &= kInFlagMask;
                eskip = ((sb8.tag >> kSibSkipShift) & 3u) | ((sb8.e[2] >> 31) << 2);
                sb8.e[2] &= kIdMask;
                zneed = sib_ok && (sb8.tag & kSibZNeed) != 0;
            }
        }
        const uint32_t xs = valid ? x : 0u;  // a harmless valid node for unconditional loads
        Cls q[kBatchK], e[kBatchE], qz = {0, 0, 0};
        bool gq[kBatchK], ge[kBatchE];
#pragma unroll
        for (uint32_t i = 0; i < kBatchK; ++i) q[i] = {0, 0, 0};
#pragma unroll
        for (uint32_t i = 0; i < kBatchE; ++i) e[i] = {0, 0, 0};
        if (DELIVER) {
            if (FILT) {
                // rows that cannot change any result are not gathered
                // (round_kernel, "live-filtered gathers")
#pragma unroll
                for (uint32_t i = 0; i < kBatchK; ++i) {
                    gq[i] = i < k && !((qskip >> i) & 1u);
                    if (gq[i]) q[i] = load_cls_w<W>(S, in8.s[i], j);
                }
                if (valid && !(tgw & kTgNoPull) && (zlive || zneed)) qz = load_cls_w<W>(S, z, j);
#pragma unroll
                for (uint32_t i = 0; i < kBatchE; ++i) {
                    ge[i] = i < r && !((eskip >> i) & 1u);
                    if (ge[i]) e[i] = load_cls_w<W>(S, sb8.e[i], j);
                }
            } else {
#pragma unroll
                for (uint32_t i = 0; i < kBatchK; ++i) {
                    gq[i] = true;
                    q[i] = load_cls_w<W>(S, i < k ? in8.s[i] : xs, j);
                }
                qz = load_cls_w<W>(S, valid ? z : 0u, j);
#pragma unroll
                for (uint32_t i = 0; i < kBatchE; ++i) {
                    ge[i] = true;
                    e[i] = load_cls_w<W>(S, i < r ? sb8.e[i] : xs, j);
                }
            }
        }
        // ---- the next tile's first level, in flight beside the gathers
        if (t + gridDim.x < ntiles) pipe_issue<W, DELIVER, FILT>(a, t + gridDim.x, lds + (b ^ 1u) * T::kBuf, wv, lane);

        const u64 isC = P[0], a0 = P[1], a1 = P[2];
        const u64 A = ~isC & ~a0 & ~a1;
        const u64 B = ~isC & (a0 | a1);
        const u64 C = isC & ~(a0 & a1);
        const u64 liveX = B | C;

        // ---- phases 1 and 2 of round t at x (Gossip::receive)
        const bool off_t = DELIVER && (tgw & kTgOff);
        const bool pulled = !(tgw & kTgNoPull);
        Recv<false> rv;
        rv.init(A, B, B & a0 & ~a1);
        uint32_t psize = 0, ext_new = 0, ext_full = 0, ext_empty = 0, ext_recv = 0;
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
                rv.push(load_cls_w<W>(S, s, j), i, k, !(pulled && s == z));
            }
            // Pull batch from z: z's live set plus what z created from pushers
            // ahead of x.
            const u64 zB = ~qz.c & (qz.a0 | qz.a1);
            const u64 zC = qz.c & ~(qz.a0 & qz.a1);
            u64 pnot = ~qz.c & ~qz.a0 & ~qz.a1, pB = 0, pC = 0;
#pragma unroll
            for (uint32_t i = 0; i < kBatchE; ++i)
                if (i < r && ge[i]) sibling(e[i], pnot, pB, pC);
            if (r > kBatchE && pnot && pulled && (!FILT || zneed)) {  // rank > kBatchE (rare)
                for (uint32_t i = kBatchE; i < min(r, kSibInline); ++i)
                    if (!((eskip >> i) & 1u)) sibling(load_cls_w<W>(S, pick_sib(sb8.e, i), j), pnot, pB, pC);
                if (r > kSibInline && pnot) {  // rank > 3: 0.2% of nodes
                    InRec zin8 = a.IN8[z];
                    if (FILT) zin8.kf &= kInFlagMask;  // (skip flags above the tail start)
                    for (uint32_t i = kSibInline; i < r && pnot; ++i) {
                        const uint32_t s = i < kInline ? pick_inline(zin8.s, i) : a.src[zin8.first() + (i - kInline)];
                        sibling(load_cls_w<W>(S, s, j), pnot, pB, pC);
                    }
                }
            }
            u64 pv2 = zB & qz.a1 & ~qz.a0;
            u64 pvB = zB | pB;  // counter 1 (created entries: 1) or 2
            u64 pCl = zC | pC;
            if (!pulled) pv2 = pvB = pCl = 0;
            const u64 pl = pvB | pCl;
            {
                const u64 newc = rv.notyet & pl;
                rv.record(rv.recB & pl, pvB, pv2, pCl);
                rv.create(newc, pCl);
            }
            rv.recv += popc(pl);
            if (a.n_ext) {
                // External RPCs to x (gs_handle_received), after every internal
                // delivery of the round, in call order (round_kernel).
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
                        const uint32_t cnt = group_sum(popc(B | C | rv.crB | rv.crC), W);
                        if (cnt) ext_full += cnt; else ++ext_empty;
                    }
                    if (info & kExtEmpty) continue;
                    ++ext_recv;
                    const uint32_t rr = info & 0xFFFu, c = (info >> 12) & 0xFFu;
                    if ((rr >> 6) != j) continue;
                    const u64 bit = 1ull << (rr & 63u);
                    const u64 vC = c >= a.cmax ? bit : 0ull;
                    const u64 vB = (c >= 1u && c < a.cmax) ? bit : 0ull;
                    const u64 v2 = (c == 2u && c < a.cmax) ? bit : 0ull;
                    const u64 newc = rv.notyet & bit;
                    rv.record(rv.recB & bit & ((info & kExtRec) ? ~0ull : 0ull), vB, v2, vC);
                    rv.create(newc, vC);
                }
            }
            psize = k + ((pulled && !zin) ? 1u : 0u) + ext_new;  // |peers_in_this_round|
        }

        // ---- node-level statistics of the deliveries
        uint32_t lc = popc(liveX), part_cw = rv.part_cw, recv = rv.recv, first_create = rv.first_create;
        uint32_t d_full_sent = 0, d_empty_pull = 0, d_recv = 0;
        if (DELIVER) {
            lc = group_sum(lc, W);
            part_cw = group_sum(part_cw, W);
            recv = group_sum(recv, W);
            first_create = group_min(first_create, W);
            d_full_sent = k * lc + part_cw;  // pull rows sent by x
            if (k > 0 && lc == 0) d_empty_pull = (first_create == kNone) ? k : first_create + 1u;
            d_recv = recv;
        }
        d_full_sent += ext_full;
        d_empty_pull += ext_empty;
        d_recv += ext_recv;

        // ---- phase 0 of round t+1 at x
        u64 inj = 0;
        if (a.n_inj && valid) inj = find_injection(a, seg);
        const bool on_next =
            !(a.f.churn && valid && offline_of(a.seed, a.epoch, a.round_new, a.node_lo + x, a.f.churn));
        const u64 pidx = ((u64)x * 2u) * W + j;
        const bool pending = off_t && valid;
        const u64 pb = pending ? a.pend[pidx] : 0ull, pa = pending ? a.pend[pidx + W] : 0ull;
        NextOut o;
        next_round_seg(P, rv, inj, psize, pending, pb, pa, on_next, a.cmax, a.maxc, a.maxr, o);
        if (!on_next && valid) {
            a.pend[pidx] = o.bump;
            a.pend[pidx + W] = o.anyC;
        }

        // ---- node maps of the round-(t+1) planes for the next in-list build
        // (live-filtered gathers): "live" and "complete", a ballot per wave
        if (a.lvm) {
            u64 lvw, aw;
            if (a.f.churn == 0u) {
                lvw = o.Bn | o.Cn;
                aw = ~(o.N[0] | o.Bn);
            } else {
                lvw = (o.N[0] & ~(o.N[1] & o.N[2])) | (~o.N[0] & (o.N[1] | o.N[2]));
                aw = ~o.N[0] & ~o.N[1] & ~o.N[2];
            }
            const u64 bl = __ballot(valid && lvw != 0);
            const u64 bc = __ballot(valid && aw == 0);
            const u64 seg0 = seg - lane;
            if (lane == 0 && seg0 < g.nseg) {
                const u64 cl = compress_stride(group_or_bits(bl, lw), lw);
                const u64 cc = compress_stride(group_and_bits(bc, lw), lw);
                uint8_t *ml = reinterpret_cast<uint8_t *>(a.lvm), *mc = reinterpret_cast<uint8_t *>(a.cpm);
                const u64 byte0 = (seg0 >> lw) >> 3;  // first node of the wave / 8
                if constexpr (W == 2) {
                    *reinterpret_cast<uint32_t *>(ml + byte0) = (uint32_t)cl;
                    *reinterpret_cast<uint32_t *>(mc + byte0) = (uint32_t)cc;
                } else if constexpr (W == 4) {
                    *reinterpret_cast<uint16_t *>(ml + byte0) = (uint16_t)cl;
                    *reinterpret_cast<uint16_t *>(mc + byte0) = (uint16_t)cc;
                } else {
                    ml[byte0] = (uint8_t)cl;
                    mc[byte0] = (uint8_t)cc;
                }
            }
        }

        // ---- round-(t+1) planes through LDS (B2: every wave read its P)
        uint32_t live_new = (valid && on_next) ? popc(o.Bn | o.Cn) : 0u;
        live_new = group_sum(live_new, W);
        if (__ballot(live_new != 0u) != 0ull && lane == 0u) *blk_any = 1u;
        __syncthreads();
#pragma unroll
        for (uint32_t p = 0; p < (uint32_t)kPlanes; ++p) *reinterpret_cast<u64 *>(buf + T::word_lds(tid, p)) = o.N[p];
        __syncthreads();  // B3
        {
            // streaming (nontemporal) 16-B stores: the tile's records are one
            // contiguous range, written in order (the image is read across planes)
            uint4 *dst4 = reinterpret_cast<uint4 *>(a.Snext) + (u64)t * T::kSlots;
#pragma unroll
            for (uint32_t i = 0; i < T::kSlots / T::kThreads; ++i) {
                const uint32_t G = tid + i * T::kThreads;
                const uint32_t xo = G >> (lw + 2u), s = G & (T::kNodeSlots - 1u);
                if (t * T::kNodes + xo < g.n)
                    nt_store4(*reinterpret_cast<const uint4 *>(buf + T::slot_lds(xo, s)), dst4 + G);
            }
        }

        // ---- push list + Statistics (src/gossip.rs:80,103-111)
        if (valid && j == 0u) {
            // rounds is the engine's round count; the other four are u32
            // deltas folded into u64 before they can wrap
            uint4 v = *reinterpret_cast<const uint4 *>(buf + T::oST + xl * 16u);
            const uint32_t d_empty_push = (on_next && live_new == 0u) ? 1u : 0u;
            if (a.emin) {  // rumor slice: empty only if empty in every slice (MIN per byte, caller)
                reinterpret_cast<uint16_t *>(a.emin)[x] = (uint16_t)(min(d_empty_pull, 255u) | (d_empty_push << 8));
                const uint32_t ea = a.eadd ? *reinterpret_cast<const uint16_t *>(buf + T::oEA + xl * 2u) : 0u;
                v.x += ea & 0xFFu;  // an earlier round's network counts (reduced by the caller)
                v.y += ea >> 8;
            } else {
                v.x += d_empty_pull;  // empty_pull_sent
                v.y += d_empty_push;  // empty_push_sent
            }
            v.z += live_new + d_full_sent;  // full_message_sent
            v.w += d_recv;                  // full_message_received
            reinterpret_cast<uint4 *>(a.st32)[x] = v;
            if (!on_next) atomicAdd(&a.offc[x], 1u);  // (no return: nothing waits for it)
        }
    }
    __syncthreads();
    if (tid0 == 0 && *blk_any) {
        uint32_t *f = &a.flags[a.round_new & 1u];
        if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) atomicOr(f, 1u);
    }
}

namespace {

template <uint32_t W, int MODE, bool FILT>
hipError_t launch_pipe_t(const RoundArgs &a, hipStream_t s) {
    using T = PipeTile<W>;
    const uint32_t ntiles = (a.g.n + T::kNodes - 1u) / T::kNodes;
    if (ntiles == 0) return hipSuccess;
    // persistent grid: every resident block of the device, at most one per tile
    static uint32_t resident = 0;
    if (resident == 0) {
        int dev = 0, cus = 0, per = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, round_pipe<W, MODE, FILT>, T::kThreads, 0) !=
                hipSuccess)
            return hipErrorUnknown;
        resident = (uint32_t)std::max(1, cus * per);
    }
    const uint32_t grid = std::min(ntiles, a.pipe_grid ? a.pipe_grid : resident);
    hipLaunchKernelGGL((round_pipe<W, MODE, FILT>), dim3(grid), dim3(T::kThreads), 0, s, a, ntiles);
    return hipGetLastError();
}

template <uint32_t W>
hipError_t launch_pipe_w(const RoundArgs &a, int mode, hipStream_t s) {
    const bool filt = a.zlm != nullptr;
    if (mode == 0) return filt ? launch_pipe_t<W, 0, true>(a, s) : launch_pipe_t<W, 0, false>(a, s);
    return filt ? launch_pipe_t<W, 1, true>(a, s) : launch_pipe_t<W, 1, false>(a, s);
}

}  // namespace

bool pipe_eligible(const RoundArgs &a, int mode) {
    return (mode == 0 || mode == 1) && !a.g.small && a.g.W >= 2 && a.g.W <= 8 && !a.recvA && !a.Wb && !a.DR &&
           !a.zb_nxt && a.blk_count == 0 && a.blk_off == 0;
}

hipError_t launch_round_pipe(const RoundArgs &a, int mode, hipStream_t s) {
    switch (a.g.W) {
    case 2: return launch_pipe_w<2>(a, mode, s);
    case 4: return launch_pipe_w<4>(a, mode, s);
    case 8: return launch_pipe_w<8>(a, mode, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace gs
