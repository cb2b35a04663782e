// gs_device.h -- device helpers shared by the round, CSR and shard kernels.
#pragma once
#include "gs_common.h"

namespace gs {

#define GS_DEV __device__ __forceinline__

GS_DEV uint32_t popc(u64 v) { return (uint32_t)__popcll(v); }

// Round kernels clear the next in-list build's counters (RoundArgs::zero_*)
// instead of a memset launch: grid-stride vector stores of buf[0, words), and
// *one = 0 from the first thread.
GS_DEV void zero_for_build(uint32_t *buf, uint32_t words, u64 *one) {
    const uint32_t gt = blockIdx.x * blockDim.x + threadIdx.x;
    for (uint32_t i = gt; i < words; i += gridDim.x * blockDim.x) buf[i] = 0u;
    if (one && gt == 0u) *one = 0ull;
}

// c += in (bit-sliced 5-bit counters, one per rumor).
GS_DEV void add5(u64 (&c)[5], u64 in) {
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        u64 t = c[i] & in;
        c[i] ^= in;
        in = t;
    }
}

// Bit-sliced "x >= K" for an NB-bit number per rumor, K a per-lane constant:
// the borrow of x - K, LSB first (borrow' = k ? ~x | b : ~x & b, one 3-input
// op per 32-bit half and bit), x >= K iff no final borrow.
template <int NB>
GS_DEV u64 ge_k(const u64 (&x)[NB], uint32_t K) {
    u64 b = 0ull;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const uint32_t m = 0u - ((K >> i) & 1u);
        const u64 k = ((u64)m << 32) | m;
        b = (~x[i] & b) | (k & (~x[i] | b));
    }
    return K >= (1u << NB) ? 0ull : ~b;
}

// Same with K wave-uniform (max_rounds, max_c_rounds): the masks are scalar.
template <int NB>
GS_DEV u64 ge_u(const u64 (&x)[NB], uint32_t K) {
    if (K >= (1u << NB)) return 0ull;
    u64 b = 0ull;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const u64 k = ((K >> i) & 1u) ? ~0ull : 0ull;
        b = (~x[i] & b) | (k & (~x[i] | b));
    }
    return ~b;
}

// The bit-sliced helpers for a lane word of either width (u64, or u32 for
// the 32-bit lane kernels: gs_dlv4.hip, gs_w32.hip).
template <typename T>
GS_DEV uint32_t popcT(T v) {
    if constexpr (sizeof(T) == 8) return (uint32_t)__popcll(v);
    else return (uint32_t)__popc(v);
}
template <typename T>
GS_DEV void add5T(T (&c)[5], T in) {
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const T t = c[i] & in;
        c[i] ^= in;
        in = t;
    }
}
// "x >= K" for a wave-uniform K (the borrow chain of x - K)
template <int NB, typename T>
GS_DEV T ge_uT(const T (&x)[NB], uint32_t K) {
    if (K >= (1u << NB)) return (T)0;
    T b = 0;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const T k = ((K >> i) & 1u) ? (T)~(T)0 : (T)0;
        b = (~x[i] & b) | (k & (~x[i] | b));
    }
    return ~b;
}
// "x >= K" for a per-lane K
template <int NB, typename T>
GS_DEV T ge_kT(const T (&x)[NB], uint32_t K) {
    T b = 0;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const T k = (T)0 - (T)((K >> i) & 1u);
        b = (~x[i] & b) | (k & (~x[i] | b));
    }
    return K >= (1u << NB) ? (T)0 : ~b;
}

template <typename T>
struct ClsT {
    T c, a0, a1;
};
using Cls = ClsT<u64>;

#ifndef GS_CLS_VEC
#define GS_CLS_VEC 0  // A/B: 1 = 16-byte loads for a gathered row's planes 0-1 (no gain / slower)
#endif
template <bool SMALL>
struct Lane {
    // segment geometry
    uint32_t x, j;
    u64 base;       // index of plane 0 of this lane's word
    uint32_t sh;    // bit offset of the segment in its word (small)
    u64 m;          // segment mask (after shifting down)
    uint32_t W, lognpu, logr;

    GS_DEV void init(const Geometry &g, u64 seg) {
        W = g.W;
        lognpu = g.lognpu;
        logr = g.logr;
        if (SMALL) {
            x = (uint32_t)seg;
            j = 0;
            base = (u64)(x >> lognpu) * kPlanes;
            sh = (x & ((1u << lognpu) - 1u)) << logr;
            m = (1ull << g.rpad) - 1ull;  // rpad < 64 here
        } else {
            // W = 2^(logr - 6): shifts, not a 64-bit division by a runtime W
            const uint32_t lw = logr - 6u;
            x = (uint32_t)(seg >> lw);
            j = (uint32_t)seg & (W - 1u);
            base = ((u64)x << (lw + 3u)) + j;
            sh = 0;
            m = ~0ull;
        }
    }
    GS_DEV u64 plane_index(uint32_t p) const {
        return SMALL ? base + p : base + ((u64)p << (logr - 6u));
    }
    // Exchange rows (SHARD): row e holds `np` planes of W words, [e][np][W]; a
    // node with R < 64 keeps its segment in the low bits of one word per plane.
    GS_DEV u64 row_index(uint32_t e, uint32_t np, uint32_t p) const {
        return ((u64)e * np + p) * W + j;
    }
    // A push row: the 2-plane class code of the pusher's live entries (b0, b1):
    // 01 counter 1, 10 counter 2, 11 counter 255 (C), 00 none.  Decoded into
    // class planes that push()/sibling() read the same way (a C entry as
    // C{round 0}, "none" as A: a pusher's A and D push nothing alike).
    GS_DEV Cls load_push_row(const u64 *__restrict__ rows, uint32_t e) const {
        const u64 b0 = rows[row_index(e, 2, 0)], b1 = rows[row_index(e, 2, 1)];
        return Cls{b0 & b1, b0 & ~b1, b1 & ~b0};
    }
    // Class planes (isC, a0, a1) of node s for this lane's word.
    GS_DEV Cls load_cls(const u64 *__restrict__ S, uint32_t s) const {
        Cls r;
        if (SMALL) {
            u64 b = (u64)(s >> lognpu) * kPlanes;
            uint32_t ss = (s & ((1u << lognpu) - 1u)) << logr;
            if (GS_CLS_VEC) {  // planes 0-1 in one 16-byte load (a unit's planes are 64-B aligned)
                const ulonglong2 v = *reinterpret_cast<const ulonglong2 *>(S + b);
                r.c = (v.x >> ss) & m;
                r.a0 = (v.y >> ss) & m;
            } else {
                r.c = (S[b] >> ss) & m;
                r.a0 = (S[b + 1] >> ss) & m;
            }
            r.a1 = (S[b + 2] >> ss) & m;
        } else {
            const uint32_t lw = logr - 6u;
            u64 b = ((u64)s << (lw + 3u)) + j;
            if (GS_CLS_VEC && lw == 0u) {
                // one word per plane (64 rumors): planes 0-1 in one 16-byte
                // load, two load requests per row instead of three
                const ulonglong2 v = *reinterpret_cast<const ulonglong2 *>(S + b);
                r.c = v.x;
                r.a0 = v.y;
                r.a1 = S[b + 2];
                return r;
            }
            r.c = S[b];
            r.a0 = S[b + W];
            r.a1 = S[b + 2 * (u64)W];
        }
        return r;
    }
};

// Sum / min over the W lanes of one node (W a power of two <= 64, lanes of a
// node are consecutive and W-aligned inside the wave).
GS_DEV uint32_t group_sum(uint32_t v, uint32_t W) {
    for (uint32_t o = 1; o < W; o <<= 1) v += __shfl_xor(v, (int)o, 64);
    return v;
}
GS_DEV uint32_t group_min(uint32_t v, uint32_t W) {
    for (uint32_t o = 1; o < W; o <<= 1) v = min(v, (uint32_t)__shfl_xor(v, (int)o, 64));
    return v;
}

constexpr uint32_t kNone = 0xffffffffu;

// Statistics deltas of node x between folds (RoundArgs::st32): [n][4] u32,
// or with st16 [n][4] u16 -- the delivery-record engines (R_pad <= 16), whose
// per-round deltas of internal deliveries are below 32 R_pad + 32 and fold
// into the u64 totals well before 16 bits wrap (8 B read + 8 written per node
// and round instead of 16 + 16).  Order: empty_pull, empty_push, full_sent,
// full_received.
GS_DEV uint4 load_stats(const uint32_t *st, uint32_t st16, u64 x) {
    if (st16) {
        const uint2 h = reinterpret_cast<const uint2 *>(st)[x];
        return make_uint4(h.x & 0xFFFFu, h.x >> 16, h.y & 0xFFFFu, h.y >> 16);
    }
    return reinterpret_cast<const uint4 *>(st)[x];
}
GS_DEV void store_stats(uint32_t *st, uint32_t st16, u64 x, uint4 v) {
    if (st16) reinterpret_cast<uint2 *>(st)[x] = make_uint2((v.x & 0xFFFFu) | (v.y << 16), (v.z & 0xFFFFu) | (v.w << 16));
    else reinterpret_cast<uint4 *>(st)[x] = v;
}

// First-carrier class of the entries z created from its pushers ahead of x
// (the pull row is built before x's push is absorbed, src/gossip.rs:124-151).
GS_DEV void sibling(const Cls &q, u64 &pnot, u64 &pB, u64 &pC) {
    const u64 vC = q.c & ~(q.a0 & q.a1);
    const u64 sl = (~q.c & (q.a0 | q.a1)) | vC;
    const u64 nc = pnot & sl;
    pB |= nc & ~vC;
    pC |= nc & vC;
    pnot &= ~sl;
}

// v[i] for a runtime i < kInline without dynamic register indexing.
GS_DEV uint32_t pick_inline(const uint32_t (&v)[kInline], uint32_t i) {
    uint32_t r = v[0];
#pragma unroll
    for (uint32_t q = 1; q < kInline; ++q) r = (i == q) ? v[q] : r;
    return r;
}

GS_DEV uint32_t pick_sib(const uint32_t (&v)[kSibInline], uint32_t i) {
    uint32_t r = v[0];
#pragma unroll
    for (uint32_t q = 1; q < kSibInline; ++q) r = (i == q) ? v[q] : r;
    return r;
}

// 16-byte streaming (nontemporal) store, for outputs nobody reads again
// while they could still be cached (the next round's planes, 4.3 GB at config 4).
typedef unsigned int gs_u32x4 __attribute__((ext_vector_type(4)));
GS_DEV void nt_store4(const uint4 &v, uint4 *p) {
    const gs_u32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<gs_u32x4 *>(p));
}

constexpr uint32_t kScanBlock = 256;

// Block-wide exclusive scan of one value per thread; returns the block total.
GS_DEV uint32_t block_exclusive_scan(uint32_t v, uint32_t *lds, uint32_t &total) {
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t t = __shfl_up(inc, (unsigned)o, 64);
        if (lane >= (uint32_t)o) inc += t;
    }
    if (lane == 63) lds[wid] = inc;
    __syncthreads();
    uint32_t wbase = 0, tot = 0;
    for (uint32_t w = 0; w < kScanBlock / 64; ++w) {
        if (w < wid) wbase += lds[w];
        tot += lds[w];
    }
    __syncthreads();
    total = tot;
    return wbase + inc - v;
}

// Exclusive scan over a block of NT threads (NT a multiple of 64, <= 1024);
// `lds` holds NT/64 words.
template <uint32_t NT>
GS_DEV uint32_t block_exclusive_scan_t(uint32_t v, uint32_t *lds, uint32_t &total) {
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t t = __shfl_up(inc, (unsigned)o, 64);
        if (lane >= (uint32_t)o) inc += t;
    }
    if (lane == 63) lds[wid] = inc;
    __syncthreads();
    uint32_t wbase = 0, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < NT / 64; ++w) {
        const uint32_t c = lds[w];
        wbase += (w < wid) ? c : 0u;
        tot += c;
    }
    __syncthreads();
    total = tot;
    return wbase + inc - v;
}

// Keep the bits of m at multiples of W = 2^logw (W <= 8), packed to the bottom.
GS_DEV u64 compress_stride(u64 m, uint32_t logw) {
    if (logw == 1u) {
        m &= 0x5555555555555555ull;
        m = (m | (m >> 1)) & 0x3333333333333333ull;
        m = (m | (m >> 2)) & 0x0F0F0F0F0F0F0F0Full;
        m = (m | (m >> 4)) & 0x00FF00FF00FF00FFull;
        m = (m | (m >> 8)) & 0x0000FFFF0000FFFFull;
        m = (m | (m >> 16)) & 0x00000000FFFFFFFFull;
    } else if (logw == 2u) {
        m &= 0x1111111111111111ull;
        m = (m | (m >> 3)) & 0x0303030303030303ull;
        m = (m | (m >> 6)) & 0x000F000F000F000Full;
        m = (m | (m >> 12)) & 0x000000FF000000FFull;
        m = (m | (m >> 24)) & 0x000000000000FFFFull;
    } else if (logw == 3u) {
        m &= 0x0101010101010101ull;
        m = (m | (m >> 7)) & 0x0003000300030003ull;
        m = (m | (m >> 14)) & 0x0000000F0000000Full;
        m = (m | (m >> 28)) & 0x00000000000000FFull;
    }
    return m;
}
// OR / AND of each aligned group of W bits, into the group's lowest bit.
GS_DEV u64 group_or_bits(u64 m, uint32_t logw) {
    for (uint32_t o = 1; o < (1u << logw); o <<= 1) m |= m >> o;
    return m;
}
GS_DEV u64 group_and_bits(u64 m, uint32_t logw) {
    for (uint32_t o = 1; o < (1u << logw); o <<= 1) m &= m >> o;
    return m;
}

}  // namespace gs
