/*
 * gs_oracle.h -- CPU ORACLE for the safe_gossip push-pull round.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (safe_gossip_amd/, include/)
 * includes, links or calls this.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py load it (as liboracle.so via ctypes), and only as
 * the checker / the timed CPU port -- never as the thing measured on the GPU.
 *
 * PARITY PINNING.  The reference (Rust, /root/reference) cannot be compiled
 * here (no rustc/cargo, unvendored crates) and its tests hold no golden vectors
 * (they print, never assert values: src/gossiper.rs:299-322).  This oracle is
 * therefore "parity unpinned" with respect to reference OUTPUTS.  It is pinned by
 *   (1) hand-derived known-answer tests taken from the reference code paths
 *       (tests/golden/kat_*.json, generator tests/golden/make_golden.py),
 *   (2) Philox4x32-10 Random123 KATs, cross-checked against rocrand's header,
 *   (3) a statistical check of the SEQ schedule against the published
 *       convergence table (README.md:5 / img/evaluate_result.png).
 *
 * It restates, with the reference's own data structures (ordered maps), the
 * algorithm of:
 *   src/message_state.rs:48-181  (MessageState: new, new_from_peer, receive,
 *                                 next_round, our_counter)
 *   src/gossip.rs:46-180         (Gossip: add_peer, new_message, next_round,
 *                                 receive, clear) and :209-264 (Statistics)
 *   src/gossiper.rs:45-79        (Gossiper: add_peer, send_new, next_round)
 *   src/gossiper.rs:157-259      (test harness: create_network, send_messages)
 * Node Ids are u32 indices (Id order == index order); rumor byte strings are
 * dense indices 0..R-1 (map order == index order).
 */
#ifndef GS_ORACLE_H
#define GS_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_SCHED_2P = 0, OR_SCHED_SEQ = 1 };

/* or_fault bits (harness-injected faults). */
enum { OR_FAULT_OFFLINE = 1, OR_FAULT_PUSH = 2, OR_FAULT_PULL = 4 };

/* Statistics, src/gossip.rs:209-221 (field order kept). */
typedef struct {
    uint64_t rounds;
    uint64_t empty_pull_sent;
    uint64_t empty_push_sent;
    uint64_t full_message_sent;
    uint64_t full_message_received;
} or_stats;

/* Result of one send_messages() iteration, src/gossiper.rs:173-259. */
typedef struct {
    uint64_t nodes_missed;
    uint64_t msgs_missed;
    or_stats stats;         /* summed, rounds = last node's, empties minus n */
    uint32_t rounds_run;    /* harness loop iterations (== stats.rounds)     */
    uint32_t round_full;    /* first round after which all nodes know all
                               injected rumors (0 = never)                   */
} or_metrics;

typedef struct or_net or_net;

or_net  *or_create(uint32_t n, uint32_t R, uint64_t seed, uint32_t epoch);
void     or_destroy(or_net *net);
/* Override the derived parameters (counter_max, max_c_rounds, max_rounds). */
void     or_set_params(or_net *net, uint8_t cmax, uint8_t maxc, uint8_t maxr);
void     or_get_params(const or_net *net, uint8_t out[3]);
/* Harness-injected faults, as thresholds over 2^32 (probability = thr/2^32):
 * churn = a node is offline for a round (the harness skips its next_round
 * and every RPC to or from it; its state is kept), drop_push = a
 * push batch is not delivered (and so never answered), drop_pull = a pull
 * batch is not delivered.  Drawn per (round, node) from or_fault. */
void     or_set_faults(or_net *net, uint32_t churn, uint32_t drop_push, uint32_t drop_pull);
/* Gossiper::send_new: queued, applied in the next round's phase 0 right before
 * that node's next_round (src/gossiper.rs:203-208).  1 = NoPeers. */
int      or_send_new(or_net *net, uint32_t node, uint32_t rumor);
/* One harness round: phase 0 (next_round for every node) then delivery in the
 * chosen schedule.  *any_live = some node pushed a live rumor
 * (src/gossiper.rs:209-212).  Returns 1 = NoPeers. */
int      or_next_round(or_net *net, int schedule, uint32_t *any_live);
/* Gossiper::clear (src/gossiper.rs:111-115), plus a new Philox epoch. */
void     or_clear(or_net *net, uint32_t epoch);
uint32_t or_round(const or_net *net);

/* Observers (state after the last delivery). */
void     or_dump_state(const or_net *net, uint16_t *out);          /* n*R  */
void     or_dump_records(const or_net *net, uint16_t *rec, uint32_t *psize);
void     or_statistics(const or_net *net, uint64_t *out);         /* n*5  */
void     or_messages(const or_net *net, uint32_t node, uint64_t *words);
uint64_t or_known_total(const or_net *net);
void     or_known_all(const or_net *net, uint64_t *words);   /* n*ceil(R/64) */

/* Byte-level RPC hooks (the wire-format tests): the push list of `node` this
 * round, and Gossip::receive of one RPC from `peer` on `node` now, after the
 * round's deliveries (rumor -1 = the empty message). */
void     or_push_list(const or_net *net, uint32_t node, int32_t *rumors, uint8_t *counters,
                      uint32_t *n);
void     or_receive(or_net *net, uint32_t node, uint32_t peer, int push, int32_t rumor,
                    uint8_t counter, int32_t *rumors, uint8_t *counters, uint32_t *n);

/* send_messages(gossipers, num_of_msgs) restated (src/gossiper.rs:173-259):
 * Philox-chosen first origin, then 50% per node per round while rumors remain,
 * termination after a round with no live push; clears the network at the end. */
int      or_send_messages(or_net *net, uint32_t num_msgs, int schedule,
                          or_metrics *out);

/* Philox4x32-10 (Random123) and the injected peer schedule. */
void     or_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
uint32_t or_peer(uint64_t seed, uint32_t epoch, uint32_t round, uint32_t node,
                 uint32_t n);
uint32_t or_origin(uint64_t seed, uint32_t epoch, uint32_t rumor, uint32_t n);
uint32_t or_coin(uint64_t seed, uint32_t epoch, uint32_t round, uint32_t node);
uint32_t or_fault(uint64_t seed, uint32_t epoch, uint32_t round, uint32_t node,
                  uint32_t churn, uint32_t drop_push, uint32_t drop_pull);
/* Parameter derivation, src/gossip.rs:59-64 (f64 ln, ceil, as u8, max 1). */
void     or_derive_params(uint32_t network_size, uint8_t out[3]);

/* Known-answer-test hooks on a single MessageState (io = {tag, round,
 * our_counter, rounds_in_state_b}; tag 0=A 1=B 2=C 3=D). */
void     or_ms_step(uint8_t io[4], const uint32_t *peers, const uint8_t *vals,
                    uint32_t nrec, const uint32_t *pir, uint32_t npir, uint8_t cmax,
                    uint8_t maxc, uint8_t maxr, int do_next_round);
void     or_ms_new(uint8_t io[4]);
int      or_ms_our_counter(const uint8_t io[4]);

/* gs_dense.c: the 2P round as a dense bit-sliced OpenMP CPU program (the
 * secondary "best CPU" baseline); checked against the oracle in tests/. */
void    *dn_create(uint32_t n, uint32_t R, uint64_t seed, uint32_t epoch);
void     dn_destroy(void *d);
void     dn_send_new(void *d, uint32_t node, uint32_t rumor);
int      dn_next_round(void *d, uint32_t *any_live);
void     dn_dump_state(void *d, uint16_t *codes /* n*R */, uint64_t *stats /* n*5 */);
void     dn_dump_records(void *d, uint16_t *recs /* n*R */, uint32_t *psize /* n */);
void     dn_set_faults(void *d, uint32_t churn, uint32_t drop_push, uint32_t drop_pull);
void     dn_digest(void *d, uint64_t *out /* n */);
/* dn_next_round, also writing the dn_digest of the state before it (NULL: none). */
int      dn_next_round_digest(void *d, uint32_t *any_live, uint64_t *digest /* n */);
int      dn_threads(void);

#ifdef __cplusplus
}
#endif
#endif
