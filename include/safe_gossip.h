/*
 * safe_gossip.h -- C ABI of the MI355X-native safe_gossip push-pull engine.
 *
 * One handle (gs_engine) is one simulated full-mesh network of n Gossipers,
 * each gossiping up to R rumors, resident in HBM on one MI355X.  Every entry
 * point is population-level: a call replaces the per-node Rust call it cites
 * for ALL nodes at once.  Plain C types only; caller owns every host buffer,
 * the engine owns every device buffer.  Not thread-safe per handle.
 *
 * Reference interface replaced (paths relative to the reference crate):
 *   gs_create          <- Gossiper::default + create_network's add_peer mesh
 *                         (src/gossiper.rs:130-140, :45-52, :157-171) and the
 *                         parameter derivation of Gossip::add_peer
 *                         (src/gossip.rs:59-64)
 *   gs_send_new        <- Gossiper::send_new      (src/gossiper.rs:55-61)
 *   gs_next_round      <- Gossiper::next_round for every node + delivery of
 *                         every Push/Pull through handle_received_message
 *                         (src/gossiper.rs:70-99; harness loop :198-235)
 *   gs_messages        <- Gossiper::messages      (src/gossiper.rs:102-104)
 *   gs_statistics      <- Gossiper::statistics    (src/gossiper.rs:107-109)
 *   gs_statistics_reduce <- Statistics::add/min/max (src/gossip.rs:225-263)
 *   gs_push_batch      <- Gossiper::next_round's serialised Push RPCs
 *                         (src/gossiper.rs:70-79, src/messages.rs:57-64)
 *   gs_handle_received <- Gossiper::handle_received_message (src/gossiper.rs:82-99)
 *                         for peers outside the simulated network
 *   gs_rpc_encode/decode <- Message::serialise/deserialise (src/messages.rs:46-55)
 *   gs_set_params      <- Gossiper::add_peer's AlreadyStarted rule and
 *                         Gossip::add_peer's parameters (src/gossiper.rs:45-52,
 *                         src/gossip.rs:59-64)
 *   gs_clear           <- Gossiper::clear (cfg(test), src/gossiper.rs:111-115)
 *   status codes       <- enum Error               (src/error.rs:23-51)
 *
 * Round schedule: "2P" -- SURVEY.md section 8, i.e. the reference harness with
 * pull batches delivered after all push batches of the round.  Peer choice is
 * the injected Philox4x32-10 stream (gs_peer).
 */
#ifndef SAFE_GOSSIP_H
#define SAFE_GOSSIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Mirrors src/error.rs:23-51 (positive) + engine errors (negative). */
typedef enum {
    GS_OK = 0,
    GS_ERR_NO_PEERS = 1,          /* Error::NoPeers         */
    GS_ERR_ALREADY_STARTED = 2,   /* Error::AlreadyStarted  */
    GS_ERR_SIG_FAILURE = 3,       /* Error::SigFailure: a signed frame failed verification */
    GS_ERR_IO = 4,                /* Error::Io (reserved)   */
    GS_ERR_SERIALISATION = 5,     /* Error::Serialisation: undecodable RPC bytes, buffer too small */
    GS_ERR_INVALID_ARGUMENT = -1,
    GS_ERR_UNSUPPORTED = -2,      /* parameters outside the packed state layout,
                                     or a shard layout the engine cannot hold */
    GS_ERR_HIP = -3,
    GS_ERR_OUT_OF_MEMORY = -4,
    GS_ERR_DEVICE_LIMIT = -5      /* a node's in-degree exceeded the packed
                                     counter range (probability ~1e-34/node) */
} gs_status;

/* Delivery order of a round.  2P: the reference harness
 * with each pull batch delivered after all push batches of the round.  SEQ:
 * the harness's literal order (src/gossiper.rs:217-234), each pull answered
 * from the responder's current state and delivered at once.  SEQ runs on one
 * engine and on rumor slices (cfg.rumor_slice); node
 * shards refuse it (GS_ERR_UNSUPPORTED: its pull chains cross node ranges). */
typedef enum { GS_SCHED_2P = 0, GS_SCHED_SEQ = 1 } gs_schedule;

typedef struct {
    uint32_t n_nodes;        /* network size n (full mesh)                   */
    uint32_t n_rumors;       /* R: rumor slots per node (1..4096)            */
    uint64_t seed;           /* Philox key                                   */
    uint32_t epoch;          /* Philox counter word 3 (iteration index)      */
    uint8_t counter_max;     /* 0 = derive from n (src/gossip.rs:61)         */
    uint8_t max_c_rounds;    /* 0 = derive from n (src/gossip.rs:62)         */
    uint8_t max_rounds;      /* 0 = derive from n (src/gossip.rs:63)         */
    uint8_t schedule;        /* gs_schedule: delivery order of a round       */
    int32_t device;          /* HIP device ordinal, -1 = current             */
    /* Harness-injected faults (BASELINE config 5), thresholds over 2^32
     * (probability = value / 2^32), drawn per (round, node) from the Philox
     * stream 3 (gs_fault): the calls the reference harness would skip.      */
    uint32_t churn;          /* node offline for the round: no next_round,
                                every RPC to or from it dropped, state kept  */
    uint32_t drop_push;      /* push batch not delivered (so never answered) */
    uint32_t drop_pull;      /* pull batch not delivered                     */
    /* Nonzero: this engine holds one rumor slice of a rumor-sliced network
     * (gs_slice_*; 2P or SEQ; external RPCs: see gs_handle_received).       */
    uint32_t rumor_slice;
    uint32_t reserved1[3];
} gs_config;

/* src/gossip.rs:209-221, same field order. */
typedef struct {
    uint64_t rounds;
    uint64_t empty_pull_sent;
    uint64_t empty_push_sent;
    uint64_t full_message_sent;
    uint64_t full_message_received;
} gs_statistics_t;

typedef enum { GS_REDUCE_SUM = 0, GS_REDUCE_MIN = 1, GS_REDUCE_MAX = 2 } gs_reduce_op;

typedef struct {
    uint32_t round;          /* 1-based index of the round just run          */
    uint32_t any_live;       /* some node pushed a live rumor this round
                                (the harness's `processed`, src/gossiper.rs:209-212) */
} gs_round_report;

typedef struct gs_engine gs_engine;

/* Version of this C ABI (struct layouts and array lengths of the entry points
 * below); a binding checks it before calling anything else.  2: gs_shard_info
 * writes 14 entries, info[4] in u32 words. */
#define GS_ABI_VERSION 2u
uint32_t    gs_abi_version(void);
/* Provenance of the loaded library: the first 16 hex digits of the SHA-256
 * of its sources and headers (safe_gossip_amd/build.py source_hash computes
 * the same over a tree), fixed at build time. */
const char *gs_build_id(void);

gs_status   gs_create(const gs_config *cfg, gs_engine **out);
void        gs_destroy(gs_engine *e);
gs_status   gs_get_params(const gs_engine *e, uint8_t out[3]);

/* Queue Gossiper::send_new(rumor) on `node`; applied in the next round's phase
 * 0 right before that node's next_round (src/gossiper.rs:203-208).  Observers
 * see it at once, as Gossip::new_message inserts it (src/gossip.rs:71-75). */
gs_status   gs_send_new(gs_engine *e, uint32_t node, uint32_t rumor);

/* Gossiper::add_peer's parameter update (src/gossiper.rs:45-52 ->
 * src/gossip.rs:59-64): params[i] = 0 derives from the network size.  Fails
 * with GS_ERR_ALREADY_STARTED once any send_new happened since the last
 * clear, like add_peer once a gossiper holds a message. */
gs_status   gs_set_params(gs_engine *e, const uint8_t params[3]);

/* One round for the whole population.  `report` may be NULL (no host sync). */
gs_status   gs_next_round(gs_engine *e, gs_round_report *report);

/* Observers: state after the last round's deliveries. */
gs_status   gs_statistics(gs_engine *e, uint32_t node, gs_statistics_t *out);
gs_status   gs_statistics_all(gs_engine *e, uint64_t *out /* n*5 */);
gs_status   gs_statistics_reduce(gs_engine *e, gs_reduce_op op, gs_statistics_t *out);
gs_status   gs_messages(gs_engine *e, uint32_t node, uint64_t *words /* ceil(R/64) */);
gs_status   gs_known_all(gs_engine *e, uint64_t *words /* n*ceil(R/64) */);
gs_status   gs_known_counts(gs_engine *e, uint64_t *known_total, uint64_t *nodes_complete);
/* As gs_known_counts, with "complete" = knows at least `min_known` rumors
 * (the harness's messages().len() == num_of_msgs, src/gossiper.rs:246). */
gs_status   gs_known_counts_min(gs_engine *e, uint32_t min_known, uint64_t *known_total,
                                uint64_t *nodes_complete);
/* |Gossiper::messages()| of every node (n u32). */
gs_status   gs_known_popcounts(gs_engine *e, uint32_t *counts);

/* Parity dumps (u16 codes identical to the oracle's):
 *   state: tag<<14 | f2<<7 | f1  (B: f1 round, f2 our_counter; C: f1
 *          rounds_in_state_b, f2 round; A/D: 0), n*R entries.
 *   rec:   anyC<<15 | cnt2<<7 | cnt1 over B.peer_counters; psize: n. */
gs_status   gs_dump_state(gs_engine *e, uint16_t *out);
gs_status   gs_dump_records(gs_engine *e, uint16_t *rec, uint32_t *psize);
/* A 64-bit digest per node of everything the parity dumps and gs_statistics_all
 * report (n u64, 8 B per node instead of 4R + 44): the sum mod 2^64 of one
 * SplitMix64-finaliser term per 64-rumor word over the 20 bit-planes of its
 * state codes and record summaries, one for psize and one per Statistics
 * counter (exact definition: safe_gossip_amd/csrc/gs_common.h digest_*).  For checking large networks against a CPU program that computes
 * the same function (oracle/gs_dense.c dn_digest).  GS_ERR_INVALID_ARGUMENT
 * while send_new calls are queued (call it before injecting). */
gs_status   gs_state_digest(gs_engine *e, uint64_t *out);
/* The same digest for a network whose rumors are sliced over several engines
 * (gs_config.rumor_slice; this engine holds the network's rumors [rumor_lo,
 * rumor_lo + R)): adds this engine's per-word sums (before the final mix,
 * gs_common.h digest_sum) with device atomics into the caller's device buffer
 * dpart[n][words] (words = ceil(R_network / 64); zeroed by the caller), then
 * gs_digest_finish mixes the summed parts of every slice and adds each
 * node's term of |peers_in_this_round| (equal on every slice) and its network
 * Statistics (host, n*5: gs_statistics_all's rows after the slices' MIN /
 * SUM combine) into out (host, n).  The result is what gs_state_digest of one
 * engine holding all rumors would give. */
gs_status   gs_state_digest_part(gs_engine *e, uint32_t rumor_lo, uint32_t words, uint64_t *dpart);
gs_status   gs_digest_finish(gs_engine *e, const uint64_t *dpart, uint32_t words, const uint64_t *stats,
                             uint64_t *out);

/* Gossiper::clear for every node.  Returns GS_ERR_DEVICE_LIMIT (after
 * clearing) when a device limit was hit since the previous clear. */
gs_status   gs_clear(gs_engine *e, uint32_t epoch);
/* Wait for every queued round; GS_ERR_DEVICE_LIMIT when a device limit was hit
 * since the last clear (gs_next_round with report == NULL does not check). */
gs_status   gs_sync(gs_engine *e);
uint32_t    gs_round(const gs_engine *e);

/* Device-time of the last `gs_next_round`'s round kernel (HIP events on the
 * engine stream), ms; for bench.py's roofline.  Returns <0 if unavailable. */
float       gs_last_round_kernel_ms(gs_engine *e);
/* Enable/disable HIP-event timing of the round kernel (default off); enabling
 * (re)starts a ring of up to 4096 per-round timings. */
void        gs_set_timing(gs_engine *e, int enable);
/* Copy the recorded per-round kernel times (ms, oldest first) into out_ms,
 * return how many were copied (or <0) and restart the ring.  Synchronises. */
int32_t     gs_round_kernel_times(gs_engine *e, float *out_ms, uint32_t max);
/* Algorithmic HBM bytes of one round kernel (DESIGN.md, section Roofline). */
double      gs_round_kernel_bytes(const gs_engine *e);
/* Name of the deliver+transition kernel this engine launches (the one
 * gs_round_kernel_bytes describes), e.g. "round_kernel_dlv4<1,u32,2>". */
const char *gs_round_kernel_name(const gs_engine *e);
/* Algorithmic HBM bytes per deliver+transition round kernel launched since
 * gs_set_timing(e, 1), as counted by the kernels: with live-filtered gathers
 * (the 2P gather path) only the class rows the in-list build leaves to
 * gather count, so the bytes depend on the state; otherwise
 * gs_round_kernel_bytes (and *launches = 0).  Synchronises. */
gs_status   gs_round_traffic(gs_engine *e, double *bytes_per_launch, uint32_t *launches);

/* ---- Sharded network (multi-GPU): one engine per rank owns the node range
 * [lo, lo+m), cut into P pipeline parts of mP nodes.  Per round t the caller
 * moves two sets of rows between ranks with FIXED-SIZE
 * all-to-all exchanges (equal splits: no row count ever reaches the host, a
 * round needs no host synchronisation).  Both buffers are part-major: part h's
 * region starts at row h*world*capP and holds one sub-block per rank, so the
 * exchange of one part is ONE equal-split all-to-all over a contiguous region:
 *   A_h(t): exchange-A buffer set t % 2, part h: world sub-blocks of capP rows
 *           (the last part: capP + idrows rows, the idrows carrying the source
 *           ids of round t+1 for the in-lists, built one round ahead) -- push
 *           rows of round t of the sources in part h;
 *   B_h(t): part h of sendB -> part h of recvB, world sub-blocks of capP rows.
 * A row holds `row words` u32 (info[4] for A, info[12] for B): the 2-plane
 * class code of the rows' rumors (2W u64 both ways), or at R_pad <= 16 in
 * the 2P schedule "code rows" (info[13] = 1): an A row is the push code (b0 |
 * b1 << 16: 01 counter 1, 10 counter 2, 11 counter 255) and the pusher's
 * target local to the receiving rank, bit 31 set when the pusher is that
 * target's own target; a B row is the pull code.  Code rows carry no id rows
 * (idrows = 0): the receiver sorts the arrived rows into delivery records
 * and runs the packed kernels.  Sequence per round t >= 1, after round t exists:
 *   [t == 1, class rows: A_{P-1}(0) on set 0] -> all A_h(t) -> gs_shard_pull -> B_h(t) ->
 *   for h < P-1: gs_shard_round_part(h) (needs B_h(t); its rows are A_h(t+1))
 *   -> gs_next_round (the remaining parts: round t+1 exists) -> A_{P-1}(t+1).
 * So A_h(t+1) and B_{h+1}(t) run while the round kernel of another part does.
 * Exchanges must be ordered against the engine stream (gs_stream).
 * gs_send_new takes global node ids owned by this rank; observers report the
 * owned nodes only.  A capacity overflow (probability < 1e-50 per round) is
 * reported as GS_ERR_DEVICE_LIMIT by gs_sync / gs_clear / the observers. */
gs_status   gs_shard_create(const gs_config *cfg, uint32_t rank, uint32_t world, gs_engine **out);
/* The same with `parts` (1..4) pipeline parts (gs_shard_create: 1). */
gs_status   gs_shard_create_parts(const gs_config *cfg, uint32_t rank, uint32_t world, uint32_t parts,
                                  gs_engine **out);
/* info = {lo, m, capP (row slots per rank sub-block of a part), idrows (id
 *         rows per sub-block of A's last part), A row words (u32 words per
 *         row: 4W for the class-code rows, 2 for code rows), world, rank,
 *         nodes per rank, parts P, nodes per part mP, rows of an A buffer
 *         (world * (P*capP + idrows)), rows of a B buffer (world * P * capP),
 *         B row words (4W, or 1 for code rows), 1 for code rows}: 14 entries
 *         since ABI version 2 (gs_abi_version; version 1 wrote 12 and counted
 *         info[4] in u64 words).  Every rank must see the same
 *         SAFE_GOSSIP_AMD_NO_DLV. */
gs_status   gs_shard_info(const gs_engine *e, uint32_t info[14]);
/* The same layout without creating an engine (host only, no device needed):
 * what gs_shard_create_parts(cfg, rank, world, parts) would report, so a
 * caller can size its exchange buffers and collectives beforehand. */
gs_status   gs_shard_plan_info(const gs_config *cfg, uint32_t rank, uint32_t world, uint32_t parts,
                               uint32_t info[14]);
/* Device buffers: sendA[2], recvA[2] (info[10] rows of info[4] u32 each),
 * sendB, recvB (info[11] rows of info[12] u32 each). */
gs_status   gs_shard_bind(gs_engine *e, void *sendA0, void *sendA1, void *recvA0, void *recvA1,
                          void *sendB, void *recvB);
/* Round kernel of pipeline part `part` of the pending round (parts in order,
 * part < P-1; gs_next_round launches the rest and completes the round). */
gs_status   gs_shard_round_part(gs_engine *e, uint32_t part);
/* After exchange A of the current round: the pull rows (into sendB), and the
 * next round's in-lists on the side stream. */
gs_status   gs_shard_pull(gs_engine *e);
/* The engine's HIP stream (hipStream_t), to order collectives on it. */
uint64_t    gs_stream(const gs_engine *e);
/* The HIP device the engine runs on (gs_config.device). */
int         gs_device(const gs_engine *e);

/* ---- Rumor-sliced network (multi-GPU): rank g holds
 * ALL n nodes and the rumors [lo_g, lo_g + R_g) as a plain engine of R_g
 * rumor slots created with cfg.rumor_slice = 1 (same seed, epoch and
 * parameters on every rank).  Rumors evolve independently: a MessageState
 * sees only copies of its own rumor (src/message_state.rs:73-84), and
 * peers_in_this_round counts RPCs (src/gossip.rs:125), which every node sends
 * whether its batch is empty or not (src/gossip.rs:105-111) -- so the slices
 * exchange no state.  Only the EMPTY-RPC Statistics depend on every slice: a
 * push is empty iff it is empty in every slice, and x's empty pulls are its
 * answered pushers up to its first creating one, a count that is monotone in
 * the slice's first creation, so the network's count is the MIN over the
 * slices of each slice's count.  The round kernel of round t writes them
 * (per node x: byte 2x empty pulls, byte 2x+1 empty push; 2n bytes) into buffer
 * t % 3 instead of its Statistics; the caller all-reduces the buffer with MIN
 * over the slices and hands it back, before the buffer is written again
 * (round t+3), with gs_slice_apply (added at once) or gs_slice_defer (added by
 * the next round kernel, no extra pass; an observer adds it first).
 * Observers report the slice's rumors, and Statistics with this slice's
 * full_message_sent / full_message_received (the network's are the SUM over
 * slices) and empty_pull_sent WITHOUT the pending round's empty pulls, which
 * the observer call leaves in `obs` (n bytes; the caller adds their MIN
 * over the slices). */
/* Device buffers (caller-owned, bound before the first round / observer):
 * buf0..buf2 for rounds t with t % 3 == 0 / 1 / 2 (2n bytes each), obs for the
 * observers (n bytes). */
gs_status   gs_slice_bind(gs_engine *e, void *buf0, void *buf1, void *buf2, void *obs);
/* Add round buffer `which` (0..2, already reduced with MIN over the slices)
 * to the Statistics, on the engine stream (gs_stream). */
gs_status   gs_slice_apply(gs_engine *e, uint32_t which);
/* The same, folded into the next round kernel's Statistics update (one
 * buffer at a time; a second call adds the first at once).  The buffer must
 * stay unchanged until that kernel ran. */
gs_status   gs_slice_defer(gs_engine *e, uint32_t which);
/* External first Pushes a slice answers per node and round (its one-byte
 * empty count and u16 deltas must not wrap; GS_ERR_DEVICE_LIMIT past it):
 * by default min(200, 32 R_pad) of the slice's own R_pad, which differs
 * between slices of uneven size.  Set every slice of a network to the same
 * bound, min(200, 32 * next_pow2(floor(R / world))) = the smallest slice's,
 * so a batch is refused by all of them or by none (1..the slice's own). */
gs_status   gs_slice_set_ext_limit(gs_engine *e, uint32_t limit);

/* ---- A whole multi-GPU network through this ABI alone (DESIGN.md section
 * 7d): the per-round loop of the two sections above -- exchanges, pipeline
 * parts, the slices' MIN reductions -- run by the library, so a host without
 * Python drives node shards or rumor slices over several GPUs with gs_net_*
 * calls only (safe_gossip_amd/sharded.py and sliced.py are the Python
 * drivers of the same engines).
 *
 * gs_net_create: one rank per process (one GPU each: cfg->device), joined
 * through RCCL (loaded at run time; GS_ERR_UNSUPPORTED without it): rank 0
 * makes an id with gs_net_unique_id and hands it to every rank out of band.
 * The collectives run on a stream of the rank's, ordered against the engine
 * stream with events, so gs_net_next_round(net, NULL) enqueues a round without
 * a host synchronisation.  Every rank makes the same calls in the same order
 * (gs_net_send_new is ignored by ranks that do not hold the node / rumor;
 * the observers are collective and return the WHOLE network on every rank).
 * gs_net_create_local: all `world` ranks in this process on cfg->device,
 * exchanged by device copies with host synchronisation (a test transport for
 * the same loop on one GPU).  `parts`: node shards' pipeline parts (1..4;
 * ignored by slices).  SEQ runs on slices only (node shards:
 * GS_ERR_UNSUPPORTED).  The wire calls (gs_push_batch, gs_handle_received*)
 * go to the engines themselves (gs_net_engine), as the sections above say. */
#define GS_NET_ID_BYTES 128
typedef struct gs_net gs_net;
typedef enum { GS_NET_SLICES = 0, GS_NET_SHARDS = 1 } gs_net_mode;
gs_status   gs_net_unique_id(uint8_t id[GS_NET_ID_BYTES]);
gs_status   gs_net_create(const gs_config *cfg, gs_net_mode mode, uint32_t rank, uint32_t world, uint32_t parts,
                          const uint8_t id[GS_NET_ID_BYTES], gs_net **out);
gs_status   gs_net_create_local(const gs_config *cfg, gs_net_mode mode, uint32_t world, uint32_t parts,
                                gs_net **out);
void        gs_net_destroy(gs_net *net);
/* Collectives a host brings instead of RCCL (gs_net_create_with): the
 * library calls them on HOST buffers it staged -- after synchronising the
 * rank's device work, copying the results back after they return -- in the
 * same order on every rank; 0 = success (else GS_ERR_IO).  alltoall: block i
 * of `send` (bytes_per_rank each) to rank i, block j of `recv` from rank j;
 * allgather: `send` of every rank into `recv` in rank order; allreduce: in
 * place over `count` elements of `dtype` with `op`.  Any transport (MPI,
 * sockets, gloo) serves; several ranks may share a GPU. */
enum { GS_NET_U8 = 0, GS_NET_U32 = 1, GS_NET_U64 = 2 };
enum { GS_NET_SUM = 0, GS_NET_MIN = 1, GS_NET_MAX = 2 };
typedef struct {
    void *ctx;
    int (*alltoall)(void *ctx, const void *send, void *recv, uint64_t bytes_per_rank);
    int (*allreduce)(void *ctx, void *buf, uint64_t count, int dtype, int op);
    int (*allgather)(void *ctx, const void *send, void *recv, uint64_t bytes_per_rank);
} gs_net_collectives;
gs_status   gs_net_create_with(const gs_config *cfg, gs_net_mode mode, uint32_t rank, uint32_t world, uint32_t parts,
                               const gs_net_collectives *coll, gs_net **out);
/* Gossiper::send_new on a node of the network (global ids). */
gs_status   gs_net_send_new(gs_net *net, uint32_t node, uint32_t rumor);
/* One round of the whole network; with a report, any_live is the network's
 * (a host synchronisation, as gs_next_round's report). */
gs_status   gs_net_next_round(gs_net *net, gs_round_report *report);
gs_status   gs_net_sync(gs_net *net);
gs_status   gs_net_clear(gs_net *net, uint32_t epoch);
/* Observers of the whole network (collective with RCCL). */
gs_status   gs_net_known_counts(gs_net *net, uint64_t *known_total, uint64_t *nodes_complete);
gs_status   gs_net_statistics_all(gs_net *net, uint64_t *out /* n*5 */);
gs_status   gs_net_dump_state(gs_net *net, uint16_t *out /* n*R, gs_dump_state's codes */);
/* The engines this process holds (1 with RCCL, `world` local ones). */
uint32_t    gs_net_local_engines(const gs_net *net);
gs_engine  *gs_net_engine(gs_net *net, uint32_t i);

/* ---- Wire format (src/messages.rs) ----------------------------------------
 * GossipRpc as maidsafe_utilities::serialisation (bincode, fixed-width little
 * endian) writes it: u32 variant (0 Push, 1 Pull) | u64 msg length | msg |
 * u8 counter.  The signed Message(Vec<u8>, Signature) wrapper used outside
 * cfg(test) (src/messages.rs:26-44) = u64 payload length | payload | u64 64 |
 * 64 signature bytes; gs_message_wrap / _unwrap only frame it, the signed
 * entry points below (gs_handle_received_signed, gs_push_batch_signed) also
 * verify / sign it on the GPU.  Size errors return GS_ERR_SERIALISATION with
 * *out_len = the size needed. */
gs_status   gs_rpc_encode(int pull, const uint8_t *msg, uint32_t msg_len, uint8_t counter, uint8_t *out,
                          uint32_t cap, uint32_t *out_len);
gs_status   gs_rpc_decode(const uint8_t *buf, uint32_t len, int *pull, uint32_t *msg_off, uint32_t *msg_len,
                          uint8_t *counter);
gs_status   gs_message_wrap(const uint8_t *payload, uint32_t len, const uint8_t signature[64], uint8_t *out,
                            uint32_t cap, uint32_t *out_len);
gs_status   gs_message_unwrap(const uint8_t *buf, uint32_t len, uint32_t *payload_off, uint32_t *payload_len,
                              uint32_t *signature_off);
/* The message bytes (Gossip's BTreeMap<Vec<u8>, _> key) of rumor slot `rumor`;
 * default: bincode of the 4-byte big-endian slot number (u64 length 4 + bytes).
 * Keys must be distinct; a push list is in key (byte) order. */
gs_status   gs_set_rumor_key(gs_engine *e, uint32_t rumor, const uint8_t *key, uint32_t len);
gs_status   gs_rumor_key(const gs_engine *e, uint32_t rumor, uint8_t *out, uint32_t cap, uint32_t *len);
/* Gossiper::next_round's return value for `node` in the current round
 * (src/gossiper.rs:70-79, src/gossip.rs:79-113): the Push RPCs as frames
 * (u32 LE length + bincode GossipRpc), key order; one empty Push if none;
 * no frame for a node the harness skipped (churn).  A shard engine takes a
 * global node id it owns. */
gs_status   gs_push_batch(gs_engine *e, uint32_t node, uint8_t *out, uint32_t cap, uint32_t *len,
                          uint32_t *count);
/* Gossiper::handle_received_message(peer, bytes) on `node` for a peer
 * OUTSIDE the simulated network (peer >= n_nodes), after the current round's
 * internal deliveries (src/gossiper.rs:82-99 -> src/gossip.rs:118-166): a
 * first Push from the peer this round is answered with the node's live
 * entries as Pull frames (or one empty Pull); the copy is absorbed (a new
 * entry is created, or recorded on a B entry); peers_in_this_round and the
 * Statistics count it.  2P or SEQ schedule; after a gs_next_round.
 * Shard engine: `node` a global id this rank owns, peer >= the network's
 * n_nodes, after gs_shard_pull and exchange B of the round.
 * Rumor slice: the caller hands EVERY slice the RPC -- the slice holding its
 * message as sent, the others the empty RPC of the same kind -- and merges
 * the slices' answers in key order, one empty Pull only if every slice's is
 * empty (safe_gossip_amd/sliced.py); a slice answers at most
 * min(200, 32 * R_pad) first Pushes per node and round
 * (GS_ERR_DEVICE_LIMIT past that: its empty answers ride the one-byte
 * per-round empty count the slices reduce with MIN).
 * Messages whose bytes are no rumor slot's key: GS_ERR_INVALID_ARGUMENT.
 * A node offline this round (churn) drops the RPC: GS_OK, no frames, no
 * effect.  Undecodable bytes: GS_ERR_SERIALISATION, nothing applied; so is a
 * response list larger than `cap` (*out_len = the size needed; call again). */
gs_status   gs_handle_received(gs_engine *e, uint32_t node, uint32_t peer, const uint8_t *msg,
                               uint32_t msg_len, uint8_t *out, uint32_t cap, uint32_t *out_len,
                               uint32_t *out_count);
/* A batch of external RPCs in one call, exactly as `count` gs_handle_received
 * calls in this order (message i = msgs[off[i] .. off[i] + len[i]) from
 * peers[i] >= n to nodes[i]), with ONE observation launch for every node a
 * first Push makes answer (instead of one per call): the responses of RPC i
 * are out[resp_off[i] .. resp_off[i+1]) (frames "u32 LE length + RPC";
 * resp_off holds count+1 offsets).  All or nothing: a malformed message, an unknown rumor or an
 * `out` smaller than the responses (GS_ERR_SERIALISATION, *out_len = bytes
 * needed) applies none of them. */
gs_status   gs_handle_received_batch(gs_engine *e, uint32_t count, const uint32_t *nodes, const uint32_t *peers,
                                     const uint8_t *msgs, const uint32_t *off, const uint32_t *len, uint8_t *out,
                                     uint32_t cap, uint32_t *out_len, uint32_t *resp_off);

/* ---- Signatures (src/messages.rs:28-44): ed25519 over SHA3-512 ----------
 * As ed25519-dalek ~0.6.1 with sha3 ~0.7.2 (not vendored in the reference;
 * restated from their published algorithms, gs_verify.hip): Keypair::sign::
 * <Sha3_512> and PublicKey::verify::<Sha3_512> for batches, one signature per
 * GPU lane.  Messages are packed in one buffer: item i is
 * msgs[off[i] .. off[i] + len[i]).  Host buffers; each call copies them to
 * `device`, runs there and waits.  The curve results are parity-unpinned
 * against a real ed25519-dalek run (oracle/ed25519_sha3.py is pinned by RFC
 * 8032's SHA-512 vectors). */
/* SHA3-512 digests (64 bytes each) of count byte strings. */
gs_status   gs_sha3_512(int device, uint32_t count, const uint8_t *data, const uint32_t *off,
                        const uint32_t *len, uint8_t *out);
/* Message::deserialise's check (src/messages.rs:38): ok[i] = 1 iff sigs[i]
 * (64 bytes) is a valid signature of message i under pubs[i] (32 bytes, the
 * peer's Id). */
gs_status   gs_ed25519_verify(int device, uint32_t count, const uint8_t *pubs, const uint8_t *sigs,
                              const uint8_t *msgs, const uint32_t *off, const uint32_t *len, uint8_t *ok);
/* Message::serialise's signature (src/messages.rs:32) for 32-byte secret
 * seeds (Gossiper::default's Keypair): pubs[i] (32) and sigs[i] (64) out. */
gs_status   gs_ed25519_sign(int device, uint32_t count, const uint8_t *seeds, const uint8_t *msgs,
                            const uint32_t *off, const uint32_t *len, uint8_t *pubs, uint8_t *sigs);
/* gs_handle_received for a SIGNED frame (Message wrapper): the signature is
 * verified under peer_key (the peer's Id = its public key,
 * src/gossiper.rs:84-88); a bad one returns GS_ERR_SIG_FAILURE and applies
 * nothing (handle_received_message drops the frame).  With node_seed (the
 * node's secret seed; NULL: unsigned responses) the Pull responses come back
 * signed by the node, as Gossiper::prepare_to_send does (src/gossiper.rs:117-127). */
gs_status   gs_handle_received_signed(gs_engine *e, uint32_t node, uint32_t peer, const uint8_t peer_key[32],
                                      const uint8_t node_seed[32], const uint8_t *msg, uint32_t msg_len,
                                      uint8_t *out, uint32_t cap, uint32_t *out_len, uint32_t *out_count);
/* gs_push_batch with every Push frame signed by the node (node_seed). */
gs_status   gs_push_batch_signed(gs_engine *e, uint32_t node, const uint8_t node_seed[32], uint8_t *out,
                                 uint32_t cap, uint32_t *len, uint32_t *count);

/* Injected peer schedule: the peer node `node` chooses in `round`. */
uint32_t    gs_peer(uint64_t seed, uint32_t epoch, uint32_t round, uint32_t node, uint32_t n);
/* Origin for rumor `rumor` in the benchmark / harness schedules. */
uint32_t    gs_origin(uint64_t seed, uint32_t epoch, uint32_t rumor, uint32_t n);
/* Harness coin (rng.gen::<bool>(), src/gossiper.rs:204). */
uint32_t    gs_coin(uint64_t seed, uint32_t epoch, uint32_t round, uint32_t node);
/* Fault bits of (round, node) for the given thresholds: 1 offline (churn),
 * 2 push batch dropped, 4 pull batch dropped (gs_config.churn/drop_*). */
uint32_t    gs_fault(uint64_t seed, uint32_t epoch, uint32_t round, uint32_t node,
                     uint32_t churn, uint32_t drop_push, uint32_t drop_pull);
/* Parameter derivation of Gossip::add_peer for network_size = n. */
void        gs_derive_params(uint32_t n, uint8_t out[3]);
const char *gs_status_string(gs_status s);

#ifdef __cplusplus
}
#endif
#endif /* SAFE_GOSSIP_H */
