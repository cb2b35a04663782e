/*
 * gs_dense.c -- "best CPU" baseline: the 2P round as a dense, bit-sliced,
 * OpenMP-parallel CPU program (the secondary CPU line
 * beside the reference-faithful oracle).
 *
 * TEST / MEASUREMENT INFRASTRUCTURE ONLY, like gs_oracle.c: loaded by tests/
 * (checked round by round against the oracle) and by bench.py's cpu_baseline
 * leg; the product never links it.
 *
 * It is the same algebra as the GPU round kernel (2P
 * semantics derived from src/gossip.rs:118-163 and src/message_state.rs:62-171)
 * written for a CPU core: per (node, rumor) 8 bit-planes, 64 rumors per u64,
 * peer_counters never materialised (a 5-bit bit-sliced counter of recorded
 * counters >= own, plus anyC), in-edge lists by a counting sort of the Philox
 * targets (pushers ascending, as the harness delivers them,
 * src/gossiper.rs:217-231).  One thread owns a node across all its words.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "gs_oracle.h"

#ifdef _OPENMP
#include <omp.h>
#endif

typedef uint64_t u64;

/* Threads the parallel loops use (the bench reports it as `cores`). */
int dn_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

enum { PLANES = 8 };

typedef struct {
    uint32_t n, R, W;
    uint64_t seed;
    uint32_t epoch, round;
    uint8_t cmax, maxc, maxr;
    int pending;        /* deliveries of `round` not yet absorbed */
    u64 *S[2];          /* [n][8][W] */
    int cur;
    u64 *st;            /* [n][4]: empty_pull, empty_push, full_sent, full_received */
    uint32_t *tg, *off, *src, *rank;  /* targets, CSR of in-edges, rank of x at t(x) */
    u64 *inj;           /* [n][W] rumors injected before the next round */
} dn_net;

static u64 wmask(const dn_net *d, uint32_t j)
{
    const uint32_t bits = d->R - 64u * j;
    return bits >= 64 ? ~0ull : ((1ull << bits) - 1ull);
}

static int popc(u64 v) { return __builtin_popcountll(v); }

static void add5(u64 c[5], u64 in)
{
    for (int i = 0; i < 5; ++i) {
        u64 t = c[i] & in;
        c[i] ^= in;
        in = t;
    }
}

static u64 ge_k(const u64 *x, int nb, uint32_t K)
{
    if (K >= (1u << nb)) return 0;
    u64 gt = 0, eq = ~0ull;
    for (int i = nb - 1; i >= 0; --i) {
        u64 ki = ((K >> i) & 1u) ? ~0ull : 0ull;
        gt |= eq & x[i] & ~ki;
        eq &= ~(x[i] ^ ki);
    }
    return gt | eq;
}

void *dn_create(uint32_t n, uint32_t R, uint64_t seed, uint32_t epoch)
{
    dn_net *d = (dn_net *)calloc(1, sizeof(dn_net));
    if (!d || n < 2 || R == 0) { free(d); return NULL; }
    d->n = n; d->R = R; d->W = (R + 63) / 64; d->seed = seed; d->epoch = epoch;
    uint8_t p[3];
    or_derive_params(n, p);
    d->cmax = p[0]; d->maxc = p[1]; d->maxr = p[2];
    const size_t sw = (size_t)n * PLANES * d->W;
    d->S[0] = (u64 *)calloc(sw, 8);
    d->S[1] = (u64 *)calloc(sw, 8);
    d->st = (u64 *)calloc((size_t)n * 4, 8);
    d->tg = (uint32_t *)calloc(n, 4);
    d->off = (uint32_t *)calloc((size_t)n + 1, 4);
    d->src = (uint32_t *)calloc(n, 4);
    d->rank = (uint32_t *)calloc(n, 4);
    d->inj = (u64 *)calloc((size_t)n * d->W, 8);
    if (!d->S[0] || !d->S[1] || !d->st || !d->tg || !d->off || !d->src || !d->rank || !d->inj) abort();
    return d;
}

void dn_destroy(void *h)
{
    dn_net *d = (dn_net *)h;
    if (!d) return;
    free(d->S[0]); free(d->S[1]); free(d->st); free(d->tg); free(d->off);
    free(d->src); free(d->rank); free(d->inj);
    free(d);
}

void dn_send_new(void *h, uint32_t node, uint32_t rumor)
{
    dn_net *d = (dn_net *)h;
    d->inj[(size_t)node * d->W + rumor / 64] |= 1ull << (rumor % 64);
}

/* Targets of `round` and their in-lists (stable counting sort: pushers of a
 * node in ascending order), with every source's rank at its target. */
static void build_lists(dn_net *d)
{
    const uint32_t n = d->n;
    #pragma omp parallel for schedule(static)
    for (uint32_t x = 0; x < n; ++x) d->tg[x] = or_peer(d->seed, d->epoch, d->round, x, n);
    memset(d->off, 0, ((size_t)n + 1) * 4);
    memset(d->rank, 0, (size_t)n * 4);
    for (uint32_t x = 0; x < n; ++x) d->off[d->tg[x] + 1]++;
    for (uint32_t y = 0; y < n; ++y) d->off[y + 1] += d->off[y];
    for (uint32_t x = 0; x < n; ++x) {
        const uint32_t y = d->tg[x];
        const uint32_t pos = d->off[y] + d->rank[y];  /* rank[] doubles as a cursor */
        d->src[pos] = x;
        d->rank[y]++;
    }
    #pragma omp parallel for schedule(static)
    for (uint32_t y = 0; y < n; ++y)
        for (uint32_t i = d->off[y]; i < d->off[y + 1]; ++i) d->rank[d->src[i]] = i - d->off[y];
}

/* Deliveries of the pending round at x and (transition) phase 0 of the next
 * round, or (observe) the u16 state codes after the deliveries. */
static int process_node(dn_net *d, uint32_t x, int transition, uint16_t *codes, u64 *stout)
{
    const uint32_t W = d->W;
    const u64 *S = d->S[d->cur];
    u64 *N = d->S[d->cur ^ 1];
    const u64 *Px = S + (size_t)x * PLANES * W;
    const int deliver = d->pending;
    const uint32_t k = deliver ? d->off[x + 1] - d->off[x] : 0;
    const uint32_t *ins = d->src + (deliver ? d->off[x] : 0);
    const uint32_t z = d->tg[x];
    const uint32_t r = deliver ? d->rank[x] : 0;
    const uint32_t *ahead = d->src + (deliver ? d->off[z] : 0);
    int zin = 0;
    for (uint32_t i = 0; i < k; ++i) zin |= ins[i] == z;
    const uint32_t psize = deliver ? k + (zin ? 0u : 1u) : 0u;
    uint32_t lc = 0, part_cw = 0, recv = 0, first_create = 0xffffffffu, live_new = 0;
    for (uint32_t j = 0; j < W; ++j) {
        const u64 m = wmask(d, j);
        u64 P[PLANES];
        for (int p = 0; p < PLANES; ++p) P[p] = Px[(size_t)p * W + j];
        const u64 isC = P[0], a0 = P[1], a1 = P[2];
        const u64 A = ~isC & ~a0 & ~a1 & m, B = ~isC & (a0 | a1), C = isC & ~(a0 & a1), D = isC & a0 & a1;
        lc += (uint32_t)popc(B | C);
        u64 notyet = A, recB = B, oc1r = B & a0 & ~a1, crB = 0, crC = 0, anyC = 0, cv[5] = {0};
        u64 c1[5] = {0}, c2[5] = {0};
#define RECORD(rec, vB, v2, vC)                      \
        do {                                         \
            anyC |= (rec) & (vC);                    \
            add5(cv, (rec) & (vB) & ((v2) | oc1r));  \
            add5(c1, (rec) & (vB));                  \
            add5(c2, (rec) & (v2));                  \
        } while (0)
        for (uint32_t i = 0; i < k; ++i) {  /* push batches, ascending pushers */
            const u64 *Q = S + (size_t)ins[i] * PLANES * W + j;
            const u64 qc = Q[0], q0 = Q[W], q1 = Q[2 * W];
            const u64 vC = qc & ~(q0 & q1), vB = ~qc & (q0 | q1), v2 = vB & q1 & ~q0, sl = vB | vC;
            const u64 newc = notyet & sl;
            if (ins[i] != z) RECORD(recB & sl, vB, v2, vC);
            crB |= newc & ~vC; crC |= newc & vC; recB |= newc & ~vC; oc1r |= newc & ~vC; notyet &= ~newc;
            const uint32_t pc = (uint32_t)popc(newc);
            part_cw += (k - 1 - i) * pc;
            if (pc && first_create > i) first_create = i;
            recv += (uint32_t)popc(sl);
        }
        if (deliver) {  /* the pull batch from z: its live set + what it created ahead of x */
            const u64 *Z = S + (size_t)z * PLANES * W + j;
            const u64 zc = Z[0], z0 = Z[W], z1 = Z[2 * W];
            const u64 zB = ~zc & (z0 | z1), zC = zc & ~(z0 & z1);
            u64 pnot = ~zc & ~z0 & ~z1 & m, pB = 0, pC = 0;
            for (uint32_t i = 0; i < r && pnot; ++i) {
                const u64 *Q = S + (size_t)ahead[i] * PLANES * W + j;
                const u64 qc = Q[0], q0 = Q[W], q1 = Q[2 * W];
                const u64 vC = qc & ~(q0 & q1), sl = (~qc & (q0 | q1)) | vC, nc = pnot & sl;
                pB |= nc & ~vC; pC |= nc & vC; pnot &= ~sl;
            }
            const u64 pv2 = zB & z1 & ~z0, pvB = zB | pB, pCl = zC | pC, pl = pvB | pCl;
            const u64 newc = notyet & pl;
            RECORD(recB & pl, pvB, pv2, pCl);
            crB |= newc & ~pCl; crC |= newc & pCl; recB |= newc & ~pCl; oc1r |= newc & ~pCl; notyet &= ~newc;
            recv += (uint32_t)popc(pl);
        }
#undef RECORD
        if (!transition) {  /* observation: codes after the deliveries */
            for (uint32_t b = 0; b < 64 && 64 * j + b < d->R; ++b) {
                const u64 bit = 1ull << b;
                uint32_t bf = 0, af = (uint32_t)((a0 >> b) & 1u) | ((uint32_t)((a1 >> b) & 1u) << 1);
                for (int i = 0; i < 5; ++i) bf |= (uint32_t)((P[3 + i] >> b) & 1u) << i;
                uint16_t code = 0;
                if (crB & bit) code = (uint16_t)((1u << 14) | (1u << 7));
                else if (crC & bit) code = (uint16_t)(2u << 14);
                else if (B & bit) code = (uint16_t)((1u << 14) | (af << 7) | bf);
                else if (C & bit) code = (uint16_t)((2u << 14) | (af << 7) | bf);
                else if (D & bit) code = (uint16_t)(3u << 14);
                codes[(size_t)x * d->R + 64 * j + b] = code;
            }
            continue;
        }
        /* phase 0 of the next round: injections (replace), then next_round */
        const u64 inj = d->inj[(size_t)x * W + j] & m, ninj = ~inj;
        const u64 Bold = B & ninj, Cold = C & ninj, Dold = D & ninj, cB = crB & ninj, cC = crC & ninj;
        const u64 Bf = Bold | cB | inj, Cf = Cold | cC;
        const u64 oc1 = (Bold & a0 & ~a1) | cB | inj, oc2 = Bold & a1 & ~a0;
        const u64 bump = ge_k(cv, 5, psize / 2 + 1) & (Bold | cB);
        const u64 anyCe = anyC & ninj;
        u64 nr[6], carry = ~0ull;
        for (int i = 0; i < 5; ++i) {
            const u64 rb = P[3 + i] & Bold;
            nr[i] = rb ^ carry;
            carry &= rb;
        }
        nr[5] = carry;
        const u64 toD = ge_k(nr, 6, d->maxr);
        const u64 oc1n = oc1 & ~bump, oc2n = (oc1 & bump) | (oc2 & ~bump), oc3n = oc2 & bump;
        const u64 ocge = d->cmax <= 1 ? ~0ull : (d->cmax == 2 ? (oc2n | oc3n) : oc3n);
        const u64 toC = anyCe | ocge;
        const u64 BD = Bf & toD, BC = Bf & ~toD & toC, BB = Bf & ~toD & ~toC;
        const u64 cr0 = a0 & Cold, cr1 = a1 & Cold;
        const u64 dd[3] = {~cr0, cr1 ^ cr0, cr1 & cr0};
        u64 rib[5], sum[6], c = 0;
        for (int i = 0; i < 5; ++i) rib[i] = P[3 + i] & Cold;
        for (int i = 0; i < 5; ++i) {
            const u64 di = i < 3 ? dd[i] : 0;
            sum[i] = rib[i] ^ di ^ c;
            c = (rib[i] & di) | (c & (rib[i] ^ di));
        }
        sum[5] = c;
        const u64 CtoD = ge_k(sum, 6, d->maxr) | ge_k(dd, 3, d->maxc);
        const u64 CD = Cf & CtoD, CC = Cf & ~CtoD;
        const u64 Dn = BD | CD | Dold, Cn = BC | CC, Bn = BB;
        u64 *Nx = N + (size_t)x * PLANES * W + j;
        Nx[0] = (Cn | Dn) & m;
        Nx[W] = ((Bn & oc1n) | (CC & dd[0]) | Dn) & m;
        Nx[2 * W] = ((Bn & oc2n) | (CC & dd[1]) | Dn) & m;
        for (int i = 0; i < 5; ++i) Nx[(size_t)(3 + i) * W] = (((Bn | BC) & nr[i]) | (CC & rib[i])) & m;
        live_new += (uint32_t)popc((Bn | Cn) & m);
    }
    uint32_t d_full = 0, d_empty = 0;
    if (deliver) {
        d_full = k * lc + part_cw;
        if (k > 0 && lc == 0) d_empty = first_create == 0xffffffffu ? k : first_create + 1;
    }
    u64 *st = d->st + (size_t)x * 4;
    if (!transition) {
        stout[0] = d->round;
        stout[1] = st[0] + d_empty;
        stout[2] = st[1];
        stout[3] = st[2] + d_full;
        stout[4] = st[3] + recv;
        return 0;
    }
    st[0] += d_empty;
    st[1] += live_new == 0;
    st[2] += live_new + d_full;
    st[3] += recv;
    return live_new > 0;
}

/* One harness round for every node (2P); returns NoPeers as the oracle does. */
int dn_next_round(void *h, uint32_t *any_live)
{
    dn_net *d = (dn_net *)h;
    int live = 0;
    #pragma omp parallel for schedule(static, 256) reduction(| : live)
    for (uint32_t x = 0; x < d->n; ++x) live |= process_node(d, x, 1, NULL, NULL);
    memset(d->inj, 0, (size_t)d->n * d->W * 8);
    d->cur ^= 1;
    d->round += 1;
    build_lists(d);
    d->pending = 1;
    if (any_live) *any_live = (uint32_t)live;
    return 0;
}

/* Observers after the last round's deliveries (oracle formats). */
void dn_dump_state(void *h, uint16_t *codes, uint64_t *stats /* n*5 */)
{
    dn_net *d = (dn_net *)h;
    #pragma omp parallel for schedule(static, 256)
    for (uint32_t x = 0; x < d->n; ++x) process_node(d, x, 0, codes, stats + (size_t)x * 5);
}
