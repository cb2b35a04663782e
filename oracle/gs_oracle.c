/*
 * gs_oracle.c -- CPU ORACLE (test infrastructure only; see gs_oracle.h header
 * for the pinning statement: parity is unpinned w.r.t. reference outputs and
 * pinned by hand-derived KATs, Philox KATs and the README convergence table).
 *
 * Data structures deliberately mirror the reference: every node owns an
 * ordered map rumor -> MessageState (BTreeMap<Vec<u8>,MessageState>,
 * src/gossip.rs:27), every B state owns an ordered map peer -> counter
 * (BTreeMap<Id,u8>, src/message_state.rs:35) and every node an ordered set
 * peers_in_this_round (BTreeSet<Id>, src/gossip.rs:41).  Ordered maps are kept
 * as sorted arrays with binary search.
 */
#include "gs_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- Philox */
#define PH_M0 0xD2511F53u
#define PH_M1 0xCD9E8D57u
#define PH_W0 0x9E3779B9u
#define PH_W1 0xBB67AE85u

void or_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4])
{
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)PH_M0 * c0;
        uint64_t p1 = (uint64_t)PH_M1 * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += PH_W0; k1 += PH_W1;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static uint64_t ph_u64(uint64_t seed, uint32_t a, uint32_t b, uint32_t stream,
                       uint32_t epoch)
{
    uint32_t ctr[4] = {a, b, stream, epoch};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t o[4];
    or_philox(ctr, key, o);
    return ((uint64_t)o[1] << 32) | o[0];
}

static uint32_t mulhi64(uint64_t v, uint32_t m)
{
    return (uint32_t)(((unsigned __int128)v * m) >> 64);
}

/* rand::thread_rng().choose(&self.peers) (src/gossiper.rs:71) with the peer
 * list order of create_network (src/gossiper.rs:157-171): node k's peers are
 * [0..k-1, k+1..n-1], so index u maps to u + (u >= k). */
uint32_t or_peer(uint64_t seed, uint32_t epoch, uint32_t round, uint32_t node,
                 uint32_t n)
{
    uint32_t u = mulhi64(ph_u64(seed, round, node, 0u, epoch), n - 1u);
    return u + (u >= node);
}

/* rand::thread_rng().choose_mut(gossipers) for the first origin
 * (src/gossiper.rs:192); also used for the per-rumor origins of the bench
 * configurations. */
uint32_t or_origin(uint64_t seed, uint32_t epoch, uint32_t rumor, uint32_t n)
{
    return mulhi64(ph_u64(seed, rumor, 0u, 1u, epoch), n);
}

/* rng.gen::<bool>() per node per round (src/gossiper.rs:204). */
uint32_t or_coin(uint64_t seed, uint32_t epoch, uint32_t round, uint32_t node)
{
    return (uint32_t)(ph_u64(seed, round, node, 2u, epoch) & 1u);
}

/* Harness-injected faults of round `round` at `node` (SURVEY.md section 8d,
 * config 5): Philox stream 3, word 0 churn, word 1 push-batch drop, word 2
 * pull-batch drop, each against its threshold (probability = thr / 2^32). */
uint32_t or_fault(uint64_t seed, uint32_t epoch, uint32_t round, uint32_t node,
                  uint32_t churn, uint32_t drop_push, uint32_t drop_pull)
{
    uint32_t ctr[4] = {round, node, 3u, epoch};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t o[4];
    or_philox(ctr, key, o);
    return (o[0] < churn ? OR_FAULT_OFFLINE : 0u) | (o[1] < drop_push ? OR_FAULT_PUSH : 0u) |
           (o[2] < drop_pull ? OR_FAULT_PULL : 0u);
}

/* ------------------------------------------------------------ parameters */
/* Gossip::add_peer, src/gossip.rs:59-64: after (n-1) add_peer calls
 * network_size == n.  f64 ln -> ln -> ceil -> `as u8` (saturating) -> max 1. */
static uint8_t as_u8(double v)
{
    if (!(v > 0.0)) return 0;          /* NaN, -0.0 and negatives -> 0 */
    if (v >= 255.0) return 255;
    return (uint8_t)v;
}

void or_derive_params(uint32_t network_size, uint8_t out[3])
{
    if (network_size <= 1) { out[0] = out[1] = out[2] = 0; return; } /* Gossip::new */
    double ns = (double)network_size;
    uint8_t lnln = as_u8(ceil(log(log(ns))));
    uint8_t ln = as_u8(ceil(log(ns)));
    out[0] = lnln < 1 ? 1 : lnln;   /* counter_max  */
    out[1] = lnln < 1 ? 1 : lnln;   /* max_c_rounds */
    out[2] = ln < 1 ? 1 : ln;       /* max_rounds   */
}

/* ----------------------------------------------------------- state types */
enum { TAG_A = 0, TAG_B = 1, TAG_C = 2, TAG_D = 3 };

typedef struct { uint32_t peer; uint8_t val; } pc_entry;

typedef struct {
    uint8_t tag;          /* B, C or D (A = absent from the node's map)       */
    uint8_t round;        /* B.round / C.round                                */
    uint8_t our_counter;  /* B.our_counter                                    */
    uint8_t rib;          /* C.rounds_in_state_b                              */
    uint32_t npc, cap;    /* B.peer_counters: sorted by peer                  */
    pc_entry *pc;
} or_state;

typedef struct { uint32_t rumor; or_state st; } or_msg;

typedef struct { uint8_t push; int32_t msg; uint8_t counter; } or_rpc; /* msg -1 = empty */

typedef struct { or_rpc *v; uint32_t n, cap; } rpc_vec;

typedef struct {
    or_msg *msgs; uint32_t nmsgs, cap;      /* BTreeMap<msg, MessageState> */
    uint8_t counter_max, max_c_rounds, max_rounds;
    uint32_t *pir; uint32_t npir, cap_pir;  /* BTreeSet<Id> peers_in_this_round */
    or_stats stats;
} or_gossip;

typedef struct { uint32_t node, rumor; } inj;

struct or_net {
    uint32_t n, R;
    uint64_t seed;
    uint32_t epoch;
    uint32_t round;
    or_gossip *g;
    inj *pend; uint32_t npend, cap_pend;
    /* harness-injected faults (thresholds over 2^32, 0 = none) */
    uint32_t f_churn, f_push, f_pull;
    /* per-round scratch */
    uint32_t *target;
    uint8_t *fault;       /* or_fault bits of the round, per node */
    rpc_vec *push, *pull;
};

static void *xrealloc(void *p, size_t sz)
{
    void *q = realloc(p, sz ? sz : 1);
    if (!q) abort();
    return q;
}

static void rpc_push(rpc_vec *v, uint8_t push, int32_t msg, uint8_t counter)
{
    if (v->n == v->cap) {
        v->cap = v->cap ? 2 * v->cap : 4;
        v->v = (or_rpc *)xrealloc(v->v, v->cap * sizeof(or_rpc));
    }
    v->v[v->n].push = push; v->v[v->n].msg = msg; v->v[v->n].counter = counter;
    v->n++;
}

/* ------------------------------------------------------ MessageState impl */
/* MessageState::new, message_state.rs:51-57 */
static void ms_new(or_state *s)
{
    s->tag = TAG_B; s->round = 0; s->our_counter = 1; s->rib = 0; s->npc = 0;
}

/* MessageState::new_from_peer, message_state.rs:62-74 */
static void ms_new_from_peer(or_state *s, uint8_t counter, uint8_t counter_max)
{
    s->npc = 0; s->cap = 0; s->pc = NULL;
    if (counter < counter_max) {
        s->tag = TAG_B; s->round = 0; s->our_counter = 1; s->rib = 0;
        return;
    }
    s->tag = TAG_C; s->rib = 0; s->round = 0; s->our_counter = 0;
}

static int pc_find(const or_state *s, uint32_t peer, uint32_t *pos)
{
    uint32_t lo = 0, hi = s->npc;
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (s->pc[mid].peer < peer) lo = mid + 1; else hi = mid;
    }
    *pos = lo;
    return lo < s->npc && s->pc[lo].peer == peer;
}

/* peer_counters.insert(peer, v) (overwrite) -- BTreeMap::insert */
static void pc_insert(or_state *s, uint32_t peer, uint8_t v, int overwrite)
{
    uint32_t pos;
    if (pc_find(s, peer, &pos)) {
        if (overwrite) s->pc[pos].val = v;
        return;
    }
    if (s->npc == s->cap) {
        s->cap = s->cap ? 2 * s->cap : 4;
        s->pc = (pc_entry *)xrealloc(s->pc, s->cap * sizeof(pc_entry));
    }
    memmove(s->pc + pos + 1, s->pc + pos, (s->npc - pos) * sizeof(pc_entry));
    s->pc[pos].peer = peer; s->pc[pos].val = v;
    s->npc++;
}

/* MessageState::receive, message_state.rs:77-83: only B records. */
static void ms_receive(or_state *s, uint32_t peer, uint8_t counter)
{
    if (s->tag == TAG_B) pc_insert(s, peer, counter, 1);
}

static void ms_free(or_state *s)
{
    free(s->pc); s->pc = NULL; s->npc = 0; s->cap = 0;
}

/* MessageState::next_round, message_state.rs:86-171 */
static void ms_next_round(or_state *s, uint8_t counter_max, uint8_t max_c_rounds,
                          uint8_t max_rounds, const uint32_t *pir, uint32_t npir)
{
    if (s->tag == TAG_B) {
        uint8_t round = (uint8_t)(s->round + 1);
        uint8_t our_counter = s->our_counter;
        if (round >= max_rounds) {                       /* :101-103 */
            s->tag = TAG_D; s->npc = 0;
            return;
        }
        for (uint32_t i = 0; i < npir; ++i)              /* :108-112, Vacant -> 0 */
            pc_insert(s, pir[i], 0, 0);
        uint32_t less = 0, ge = 0;
        for (uint32_t i = 0; i < s->npc; ++i) {          /* :116-129, key order */
            uint8_t v = s->pc[i].val;
            if (v < our_counter) {
                less++;
            } else if (v >= counter_max) {
                s->tag = TAG_C; s->rib = round; s->round = 0; s->npc = 0;
                return;
            } else {
                ge++;
            }
        }
        if (ge > less) our_counter++;                    /* :130-132 */
        if (our_counter >= counter_max) {                /* :136-141 */
            s->tag = TAG_C; s->rib = round; s->round = 0; s->npc = 0;
            return;
        }
        s->round = round; s->our_counter = our_counter;  /* :142-146 */
        s->npc = 0;                                      /* peer_counters: BTreeMap::new() */
        return;
    }
    if (s->tag == TAG_C) {
        uint8_t round = (uint8_t)(s->round + 1);
        if ((uint8_t)(round + s->rib) >= max_rounds) {   /* :154-156 */
            s->tag = TAG_D; return;
        }
        if (round >= max_c_rounds) {                     /* :159-161 */
            s->tag = TAG_D; return;
        }
        s->round = round;
        return;
    }
    /* D stays D (:169) */
}

/* MessageState::our_counter, message_state.rs:175-181; -1 = None */
static int ms_our_counter(const or_state *s)
{
    if (s->tag == TAG_B) return s->our_counter;
    if (s->tag == TAG_C) return 255;
    return -1;
}

/* ------------------------------------------------------------ Gossip impl */
static int msg_find(const or_gossip *g, uint32_t rumor, uint32_t *pos)
{
    uint32_t lo = 0, hi = g->nmsgs;
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (g->msgs[mid].rumor < rumor) lo = mid + 1; else hi = mid;
    }
    *pos = lo;
    return lo < g->nmsgs && g->msgs[lo].rumor == rumor;
}

static or_state *msg_insert_slot(or_gossip *g, uint32_t pos, uint32_t rumor)
{
    if (g->nmsgs == g->cap) {
        g->cap = g->cap ? 2 * g->cap : 4;
        g->msgs = (or_msg *)xrealloc(g->msgs, g->cap * sizeof(or_msg));
    }
    memmove(g->msgs + pos + 1, g->msgs + pos, (g->nmsgs - pos) * sizeof(or_msg));
    g->msgs[pos].rumor = rumor;
    memset(&g->msgs[pos].st, 0, sizeof(or_state));
    g->nmsgs++;
    return &g->msgs[pos].st;
}

/* BTreeSet::insert -> is_new */
static int pir_insert(or_gossip *g, uint32_t peer)
{
    uint32_t lo = 0, hi = g->npir;
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (g->pir[mid] < peer) lo = mid + 1; else hi = mid;
    }
    if (lo < g->npir && g->pir[lo] == peer) return 0;
    if (g->npir == g->cap_pir) {
        g->cap_pir = g->cap_pir ? 2 * g->cap_pir : 4;
        g->pir = (uint32_t *)xrealloc(g->pir, g->cap_pir * sizeof(uint32_t));
    }
    memmove(g->pir + lo + 1, g->pir + lo, (g->npir - lo) * sizeof(uint32_t));
    g->pir[lo] = peer;
    g->npir++;
    return 1;
}

/* Gossip::new_message, gossip.rs:71-75: insert (replace) a fresh MessageState::new */
static void gossip_new_message(or_gossip *g, uint32_t rumor)
{
    uint32_t pos;
    or_state *s;
    if (msg_find(g, rumor, &pos)) {
        s = &g->msgs[pos].st;
        /* replaced value drops its peer_counters */
        s->npc = 0;
    } else {
        s = msg_insert_slot(g, pos, rumor);
    }
    ms_new(s);
}

/* Gossip::next_round, gossip.rs:79-113 */
static void gossip_next_round(or_gossip *g, rpc_vec *push_list)
{
    g->stats.rounds += 1;
    push_list->n = 0;
    for (uint32_t i = 0; i < g->nmsgs; ++i) {
        or_state *s = &g->msgs[i].st;
        ms_next_round(s, g->counter_max, g->max_c_rounds, g->max_rounds, g->pir,
                      g->npir);
        int c = ms_our_counter(s);
        if (c >= 0) rpc_push(push_list, 1, (int32_t)g->msgs[i].rumor, (uint8_t)c);
    }
    g->npir = 0;                                         /* :102 */
    g->stats.full_message_sent += push_list->n;          /* :103 */
    if (push_list->n == 0) {                             /* :105-111 */
        g->stats.empty_push_sent += 1;
        rpc_push(push_list, 1, -1, 0);
    }
}

/* Gossip::receive, gossip.rs:118-166 */
static void gossip_receive(or_gossip *g, uint32_t peer, const or_rpc *rpc,
                           rpc_vec *responses)
{
    if (responses) responses->n = 0;
    int is_new = pir_insert(g, peer);                    /* :125 */
    if (is_new && rpc->push) {                           /* :126-148 */
        uint32_t before = responses->n;
        for (uint32_t i = 0; i < g->nmsgs; ++i) {
            int c = ms_our_counter(&g->msgs[i].st);
            if (c >= 0) rpc_push(responses, 0, (int32_t)g->msgs[i].rumor, (uint8_t)c);
        }
        uint32_t k = responses->n - before;
        g->stats.full_message_sent += k;
        if (k == 0) {
            g->stats.empty_pull_sent += 1;
            rpc_push(responses, 0, -1, 0);
        }
    }
    if (!(rpc->msg < 0 && rpc->counter == 0)) {          /* :153-163 */
        g->stats.full_message_received += 1;
        uint32_t pos;
        if (msg_find(g, (uint32_t)rpc->msg, &pos)) {
            ms_receive(&g->msgs[pos].st, peer, rpc->counter);
        } else {
            or_state *s = msg_insert_slot(g, pos, (uint32_t)rpc->msg);
            ms_new_from_peer(s, rpc->counter, g->counter_max);
        }
    }
}

static void gossip_clear(or_gossip *g)                 /* gossip.rs:168-174 */
{
    for (uint32_t i = 0; i < g->nmsgs; ++i) ms_free(&g->msgs[i].st);
    g->nmsgs = 0;
    g->npir = 0;
    memset(&g->stats, 0, sizeof(g->stats));
}

/* --------------------------------------------------------------- network */
or_net *or_create(uint32_t n, uint32_t R, uint64_t seed, uint32_t epoch)
{
    or_net *net = (or_net *)calloc(1, sizeof(or_net));
    if (!net) abort();
    net->n = n; net->R = R; net->seed = seed; net->epoch = epoch;
    net->g = (or_gossip *)calloc(n ? n : 1, sizeof(or_gossip));
    net->target = (uint32_t *)calloc(n ? n : 1, sizeof(uint32_t));
    net->fault = (uint8_t *)calloc(n ? n : 1, 1);
    net->push = (rpc_vec *)calloc(n ? n : 1, sizeof(rpc_vec));
    net->pull = (rpc_vec *)calloc(n ? n : 1, sizeof(rpc_vec));
    if (!net->g || !net->target || !net->fault || !net->push || !net->pull) abort();
    /* create_network: every node add_peer's the n-1 others; the parameters
     * after the last add_peer are those of network_size == n. */
    uint8_t p[3];
    or_derive_params(n, p);
    for (uint32_t i = 0; i < n; ++i) {
        net->g[i].counter_max = p[0];
        net->g[i].max_c_rounds = p[1];
        net->g[i].max_rounds = p[2];
    }
    return net;
}

void or_destroy(or_net *net)
{
    if (!net) return;
    for (uint32_t i = 0; i < net->n; ++i) {
        gossip_clear(&net->g[i]);
        free(net->g[i].msgs);
        free(net->g[i].pir);
        free(net->push[i].v);
        free(net->pull[i].v);
    }
    free(net->g); free(net->target); free(net->fault); free(net->push); free(net->pull);
    free(net->pend);
    free(net);
}

void or_set_params(or_net *net, uint8_t cmax, uint8_t maxc, uint8_t maxr)
{
    for (uint32_t i = 0; i < net->n; ++i) {
        net->g[i].counter_max = cmax;
        net->g[i].max_c_rounds = maxc;
        net->g[i].max_rounds = maxr;
    }
}

void or_set_faults(or_net *net, uint32_t churn, uint32_t drop_push, uint32_t drop_pull)
{
    net->f_churn = churn;
    net->f_push = drop_push;
    net->f_pull = drop_pull;
}

void or_get_params(const or_net *net, uint8_t out[3])
{
    if (net->n == 0) { out[0] = out[1] = out[2] = 0; return; }
    out[0] = net->g[0].counter_max;
    out[1] = net->g[0].max_c_rounds;
    out[2] = net->g[0].max_rounds;
}

int or_send_new(or_net *net, uint32_t node, uint32_t rumor)
{
    if (net->n < 2) return 1;                            /* Error::NoPeers */
    if (net->npend == net->cap_pend) {
        net->cap_pend = net->cap_pend ? 2 * net->cap_pend : 16;
        net->pend = (inj *)xrealloc(net->pend, net->cap_pend * sizeof(inj));
    }
    net->pend[net->npend].node = node;
    net->pend[net->npend].rumor = rumor;
    net->npend++;
    return 0;
}

static int inj_cmp(const void *a, const void *b)
{
    const inj *x = (const inj *)a, *y = (const inj *)b;
    if (x->node != y->node) return x->node < y->node ? -1 : 1;
    return 0;  /* stable w.r.t. rumor order not needed: distinct rumors */
}

/* The push batch of x reaches d: x and d online and the batch not dropped.
 * A dropped push is never answered (the harness only calls
 * handle_received_message on what it delivers, src/gossiper.rs:217-231). */
static int edge_alive(const or_net *net, uint32_t x, uint32_t d)
{
    return net->push[x].n > 0 && !(net->fault[d] & OR_FAULT_OFFLINE) &&
           !(net->fault[x] & OR_FAULT_PUSH);
}

int or_next_round(or_net *net, int schedule, uint32_t *any_live)
{
    const uint32_t n = net->n;
    if (n < 2) return 1;                                 /* Error::NoPeers */
    net->round += 1;
    uint32_t live = 0;
    /* phase 0: every node (Vec order) -- pending send_new first, then
     * Gossiper::next_round (peer choice + Gossip::next_round). */
    qsort(net->pend, net->npend, sizeof(inj), inj_cmp);
    uint32_t pi = 0;
    const int faults = net->f_churn | net->f_push | net->f_pull;
    for (uint32_t x = 0; x < n; ++x)
        net->fault[x] = faults ? (uint8_t)or_fault(net->seed, net->epoch, net->round, x, net->f_churn,
                                                   net->f_push, net->f_pull) : 0u;
    for (uint32_t x = 0; x < n; ++x) {
        while (pi < net->npend && net->pend[pi].node == x) {
            gossip_new_message(&net->g[x], net->pend[pi].rumor);
            pi++;
        }
        net->pull[x].n = 0;
        if (net->fault[x] & OR_FAULT_OFFLINE) {
            /* churn: the harness skips this node's next_round (no peer
             * choice, no transition, no push); its state is kept */
            net->push[x].n = 0;
            continue;
        }
        net->target[x] = or_peer(net->seed, net->epoch, net->round, x, n);
        gossip_next_round(&net->g[x], &net->push[x]);
        if (!(net->push[x].n == 1 && net->push[x].v[0].msg < 0)) live = 1;
    }
    net->npend = 0;
    if (schedule == OR_SCHED_SEQ) {
        /* src/gossiper.rs:217-234: pairs in (src,dst) order; pulls delivered
         * immediately after the pushes of the same pair. */
        for (uint32_t x = 0; x < n; ++x) {
            uint32_t d = net->target[x];
            rpc_vec *pv = &net->push[x];
            rpc_vec *pl = &net->pull[x];
            if (!edge_alive(net, x, d)) continue;
            for (uint32_t i = 0; i < pv->n; ++i) {
                if (i == 0) {
                    gossip_receive(&net->g[d], x, &pv->v[i], pl);
                } else {
                    rpc_vec tmp = {0, 0, 0};
                    gossip_receive(&net->g[d], x, &pv->v[i], &tmp);
                    if (tmp.n) abort();                  /* :226 assert */
                    free(tmp.v);
                }
            }
            if (net->fault[x] & OR_FAULT_PULL) continue;   /* pull batch dropped */
            for (uint32_t i = 0; i < pl->n; ++i) {
                rpc_vec tmp = {0, 0, 0};
                gossip_receive(&net->g[x], d, &pl->v[i], &tmp);
                if (tmp.n) abort();                      /* :232 assert */
                free(tmp.v);
            }
        }
    } else {
        /* 2P: phase 1 = all pushes in src order (pull batches buffered),
         * phase 2 = every buffered pull batch to its src. */
        for (uint32_t x = 0; x < n; ++x) {
            uint32_t d = net->target[x];
            rpc_vec *pv = &net->push[x];
            rpc_vec *pl = &net->pull[x];
            if (!edge_alive(net, x, d)) continue;
            for (uint32_t i = 0; i < pv->n; ++i) {
                if (i == 0) {
                    gossip_receive(&net->g[d], x, &pv->v[i], pl);
                } else {
                    rpc_vec tmp = {0, 0, 0};
                    gossip_receive(&net->g[d], x, &pv->v[i], &tmp);
                    if (tmp.n) abort();
                    free(tmp.v);
                }
            }
        }
        for (uint32_t x = 0; x < n; ++x) {
            uint32_t d = net->target[x];
            rpc_vec *pl = &net->pull[x];
            if (net->fault[x] & OR_FAULT_PULL) continue;   /* pull batch dropped */
            for (uint32_t i = 0; i < pl->n; ++i) {
                rpc_vec tmp = {0, 0, 0};
                gossip_receive(&net->g[x], d, &pl->v[i], &tmp);
                if (tmp.n) abort();
                free(tmp.v);
            }
        }
    }
    if (any_live) *any_live = live;
    return 0;
}

void or_clear(or_net *net, uint32_t epoch)
{
    for (uint32_t i = 0; i < net->n; ++i) gossip_clear(&net->g[i]);
    net->npend = 0;
    net->round = 0;
    net->epoch = epoch;
}

uint32_t or_round(const or_net *net) { return net->round; }

/* --------------------------------------------------------------- observe */
/* u16 state code: tag<<14 | f2<<7 | f1, with
 *   B: f1 = round, f2 = our_counter;  C: f1 = rounds_in_state_b, f2 = round;
 *   A (absent) and D: 0. */
void or_dump_state(const or_net *net, uint16_t *out)
{
    const uint32_t R = net->R;
    memset(out, 0, (size_t)net->n * R * sizeof(uint16_t));
    for (uint32_t x = 0; x < net->n; ++x) {
        const or_gossip *g = &net->g[x];
        for (uint32_t i = 0; i < g->nmsgs; ++i) {
            uint32_t r = g->msgs[i].rumor;
            if (r >= R) continue;
            const or_state *s = &g->msgs[i].st;
            uint16_t c = (uint16_t)((uint16_t)s->tag << 14);
            if (s->tag == TAG_B) c |= (uint16_t)((s->our_counter & 0x7f) << 7) | (s->round & 0x7f);
            if (s->tag == TAG_C) c |= (uint16_t)((s->round & 0x7f) << 7) | (s->rib & 0x7f);
            out[(size_t)x * R + r] = c;
        }
    }
}

/* Summary of B.peer_counters (what MessageState::next_round consumes):
 *   rec = anyC<<15 | cnt2<<7 | cnt1, where over the recorded values v
 *   cnt1 = #{1 <= v < cmax}, cnt2 = #{v == 2 and 2 < cmax}, anyC = any v >= cmax;
 * psize[x] = |peers_in_this_round|. */
void or_dump_records(const or_net *net, uint16_t *rec, uint32_t *psize)
{
    const uint32_t R = net->R;
    memset(rec, 0, (size_t)net->n * R * sizeof(uint16_t));
    for (uint32_t x = 0; x < net->n; ++x) {
        const or_gossip *g = &net->g[x];
        if (psize) psize[x] = g->npir;
        for (uint32_t i = 0; i < g->nmsgs; ++i) {
            uint32_t r = g->msgs[i].rumor;
            const or_state *s = &g->msgs[i].st;
            if (r >= R || s->tag != TAG_B) continue;
            uint32_t c1 = 0, c2 = 0, anyc = 0;
            for (uint32_t k = 0; k < s->npc; ++k) {
                uint8_t v = s->pc[k].val;
                if (v >= g->counter_max) anyc = 1;
                else if (v >= 1) { c1++; if (v == 2) c2++; }
            }
            rec[(size_t)x * R + r] = (uint16_t)((anyc << 15) | ((c2 & 0x7f) << 7) | (c1 & 0x7f));
        }
    }
}

void or_statistics(const or_net *net, uint64_t *out)
{
    for (uint32_t x = 0; x < net->n; ++x) {
        const or_stats *s = &net->g[x].stats;
        out[5 * (size_t)x + 0] = s->rounds;
        out[5 * (size_t)x + 1] = s->empty_pull_sent;
        out[5 * (size_t)x + 2] = s->empty_push_sent;
        out[5 * (size_t)x + 3] = s->full_message_sent;
        out[5 * (size_t)x + 4] = s->full_message_received;
    }
}

/* Gossip::messages (gossip.rs:66-68): the map's keys (B, C or D). */
void or_messages(const or_net *net, uint32_t node, uint64_t *words)
{
    uint32_t nw = (net->R + 63) / 64;
    memset(words, 0, nw * sizeof(uint64_t));
    const or_gossip *g = &net->g[node];
    for (uint32_t i = 0; i < g->nmsgs; ++i) {
        uint32_t r = g->msgs[i].rumor;
        if (r < net->R) words[r >> 6] |= 1ull << (r & 63);
    }
}

void or_known_all(const or_net *net, uint64_t *words)
{
    const uint32_t nw = (net->R + 63) / 64;
    for (uint32_t x = 0; x < net->n; ++x) or_messages(net, x, words + (size_t)x * nw);
}

uint64_t or_known_total(const or_net *net)
{
    uint64_t t = 0;
    for (uint32_t x = 0; x < net->n; ++x) t += net->g[x].nmsgs;
    return t;
}

/* ------------------------------------------------------- byte-level RPCs */
/* Gossiper::next_round's push list of `node` in the current round
 * (src/gossip.rs:93-111): rumors (-1 = the empty Push) and counters in map
 * order; *n = 0 for a node the harness skipped (churn). */
void or_push_list(const or_net *net, uint32_t node, int32_t *rumors, uint8_t *counters, uint32_t *n)
{
    const rpc_vec *pv = &net->push[node];
    *n = net->round ? pv->n : 0u;
    for (uint32_t i = 0; i < *n; ++i) {
        rumors[i] = pv->v[i].msg;
        counters[i] = pv->v[i].counter;
    }
}

/* Gossiper::handle_received_message from `peer` on `node`, now (after the
 * round's deliveries): Gossip::receive (src/gossip.rs:118-166) with the RPC
 * {push, rumor (-1 = empty message), counter}; the responses (Pull RPCs) into
 * rumors/counters (rumor -1 = the empty Pull), *n of them. */
void or_receive(or_net *net, uint32_t node, uint32_t peer, int push, int32_t rumor, uint8_t counter,
                int32_t *rumors, uint8_t *counters, uint32_t *n)
{
    or_rpc rpc;
    rpc.push = (uint8_t)(push != 0);
    rpc.msg = rumor;
    rpc.counter = counter;
    rpc_vec resp = {0, 0, 0};
    gossip_receive(&net->g[node], peer, &rpc, &resp);
    *n = resp.n;
    for (uint32_t i = 0; i < resp.n; ++i) {
        rumors[i] = resp.v[i].msg;
        counters[i] = resp.v[i].counter;
    }
    free(resp.v);
}

/* --------------------------------------------------------------- harness */
/* send_messages, src/gossiper.rs:173-259. */
int or_send_messages(or_net *net, uint32_t num_msgs, int schedule, or_metrics *out)
{
    const uint32_t n = net->n;
    if (n < 2 || num_msgs < 1) return 1;                 /* :191 assert */
    memset(out, 0, sizeof(*out));
    uint32_t next_rumor = 0;
    /* Inform the initial message (:190-195). */
    or_send_new(net, or_origin(net->seed, net->epoch, 0u, n), next_rumor++);
    int processed = 1;
    while (processed) {                                  /* :199 */
        processed = 0;
        /* Phase 0 injection coin per node in Vec order (:204-207): the
         * send_new is applied right before that node's next_round, which is
         * exactly how or_next_round applies queued injections. */
        uint32_t rnd = net->round + 1;
        for (uint32_t x = 0; x < n && next_rumor < num_msgs; ++x) {
            if (or_coin(net->seed, net->epoch, rnd, x)) or_send_new(net, x, next_rumor++);
        }
        uint32_t live = 0;
        or_next_round(net, schedule, &live);
        processed = (int)live;
        out->rounds_run++;
        if (!out->round_full) {
            int full = 1;
            for (uint32_t x = 0; x < n && full; ++x)
                if (net->g[x].nmsgs != num_msgs) full = 0;
            if (full) out->round_full = net->round;
        }
    }
    or_stats st;
    memset(&st, 0, sizeof(st));
    for (uint32_t x = 0; x < n; ++x) {                   /* :241-251 */
        const or_stats *s = &net->g[x].stats;
        st.rounds += s->rounds;
        st.empty_pull_sent += s->empty_pull_sent;
        st.empty_push_sent += s->empty_push_sent;
        st.full_message_sent += s->full_message_sent;
        st.full_message_received += s->full_message_received;
        st.rounds = s->rounds;
        if (net->g[x].nmsgs != num_msgs) {
            out->nodes_missed += 1;
            out->msgs_missed += (uint64_t)(num_msgs - net->g[x].nmsgs);
        }
    }
    st.empty_pull_sent -= n;                             /* :255-256 */
    st.empty_push_sent -= n;
    out->stats = st;
    or_clear(net, net->epoch + 1);
    return 0;
}

/* ------------------------------------------------------------ KAT hooks */
/* Drive one MessageState through MessageState::receive for each recorded
 * (peer, counter) and then MessageState::next_round with the given
 * peers_in_this_round; io = {tag, round, our_counter, rib} in and out.
 * With io[0] == TAG_A the first receive creates the state via new_from_peer
 * (as Gossip::receive does for a Vacant entry) and is not recorded. */
void or_ms_step(uint8_t io[4], const uint32_t *peers, const uint8_t *vals, uint32_t nrec,
                const uint32_t *pir, uint32_t npir, uint8_t cmax, uint8_t maxc,
                uint8_t maxr, int do_next_round)
{
    or_state s;
    memset(&s, 0, sizeof(s));
    s.tag = io[0]; s.round = io[1]; s.our_counter = io[2]; s.rib = io[3];
    uint32_t i = 0;
    if (s.tag == TAG_A && nrec > 0) { ms_new_from_peer(&s, vals[0], cmax); i = 1; }
    for (; i < nrec; ++i) ms_receive(&s, peers[i], vals[i]);
    if (do_next_round && s.tag != TAG_A) ms_next_round(&s, cmax, maxc, maxr, pir, npir);
    io[0] = s.tag; io[1] = s.round; io[2] = s.our_counter; io[3] = s.rib;
    if (s.tag == TAG_D) { io[1] = io[2] = io[3] = 0; }
    if (s.tag == TAG_C) io[2] = 0;
    if (s.tag == TAG_B) io[3] = 0;
    ms_free(&s);
}

/* MessageState::new (message_state.rs:51-57) -> io */
void or_ms_new(uint8_t io[4])
{
    or_state s;
    memset(&s, 0, sizeof(s));
    ms_new(&s);
    io[0] = s.tag; io[1] = s.round; io[2] = s.our_counter; io[3] = s.rib;
}

/* MessageState::our_counter (message_state.rs:175-181), -1 = None */
int or_ms_our_counter(const uint8_t io[4])
{
    or_state s;
    memset(&s, 0, sizeof(s));
    s.tag = io[0]; s.round = io[1]; s.our_counter = io[2]; s.rib = io[3];
    if (s.tag == TAG_A) return -1;
    return ms_our_counter(&s);
}
