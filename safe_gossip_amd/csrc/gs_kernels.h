// gs_kernels.h -- launch interface of the round kernels (gs_kernels.hip).
#pragma once
#include "gs_common.h"

namespace gs {

// The exchange layout a round kernel needs (ShardPlan's fields of the same
// names; the slot helpers below take either).
struct ShardRows {
    uint32_t G, P, W, capP, idrows, rw, rwb, codes, chunk, n;
};

struct RoundArgs {
    const u64 *Scur;          // state planes, round t (post phase 0)
    u64 *Snext;               // state planes, round t+1 (post phase 0)
    const InRec *IN8;         // round t, per node y: in-list record (gs_common.h)
    const SibRec *SIB8;       // round t, per source x: pushers of t(x) ahead of x
    const DlvRec *DR;         // round t delivery records (DLV path; IN8/SIB8 unused)
    const uint32_t *dtail;    //   push codes of pushers >= kDlvInline
    const uint32_t *pull;     //   PULL[x]: the pull batch t(x) returned to x
    uint32_t *pc_out;         // DLV: push code of every node's round-(t+1) push batch
    uint16_t *kn_out;         // single-engine DLV: every node's round-(t+1) known mask (state != A)
    uint32_t dlv_tlog, dlv_tper;  // DLV: tail regions of the records' sort parts (gs_common.h DlvRec)
    // counters of the in-list build that follows this kernel on its stream,
    // cleared here (grid-stride) instead of by a memset launch (null: none)
    uint32_t *zero_buf;
    uint32_t zero_words;
    u64 *zero_rows;
    const uint4 *IN;          // shard engine: per node {first edge, k | zi<<16, e0, e1}
    const uint32_t *IN2;      // shard engine: per node e2 (third pusher's receive row)
    const uint32_t *src;      // round t in-list tails (shard engine: receive rows)
    const uint32_t *tg;       // round t target words (target_word: target + flags)
    const uint32_t *tg_next;  // shard engine: round t+1 target words of the owned nodes
    uint32_t serial;          // build serial of the round-t lists (SIB validity)
    uint32_t *st32;           // [n][4] u32 Statistics deltas (empty_pull, empty_push,
                              //   full_sent, full_received); u16 with st16
    uint32_t st16;            // 1: u16 deltas (gs_device.h load_stats); external RPCs'
                              //   counts then go straight to st64
    const u64 *st64;          // [n][4] folded u64 totals (observation only)
    u64 obs_rounds;           // Statistics.rounds of every node (observation)
    const u64 *inj_key;       // sorted segment keys with injections (round t+1)
    const u64 *inj_mask;      //   rumor masks in segment coordinates
    uint32_t n_inj;
    uint32_t *flags;          // [2] device limit
    // any_live of round t+1: kLiveSlots words per round parity, kLiveStride
    // apart (separate 128-B lines); a block with a live node stores 1 into
    // word bid % kLiveSlots (a plain store: no read at the block's end, no
    // returning atomic), the host ORs them; block 0 of the kernel of round
    // t+1 clears round t's words
    uint32_t *live;
    // observation outputs (mode OBSERVE); any may be null
    u64 *obs_known;           // [n][KW]
    u64 *obs_stats;           // [n][5]
    uint16_t *obs_state;      // [n][R]
    uint16_t *obs_rec;        // [n][R]
    uint32_t *obs_psize;      // [n]
    u64 *obs_digest;          // [n] state digest (gs_common.h digest_*)
    // Digest parts of a rumor slice (gs_state_digest_part): this engine's word
    // sums before the final mix (digest_sum), added with atomics into
    // obs_dpart[n][dp_words] at the network's words of rumors [dp_lo, dp_lo + R)
    u64 *obs_dpart;
    uint32_t dp_lo, dp_words;
    // shard engine only (null otherwise): exchange rows, see gs_shard.hip
    const u64 *recvA;         // round-t push rows of this shard's pushers [slot][2][W]
    const u64 *recvB;         // round-t pull rows for this shard's nodes [slot][2][W]
    u64 *sendA;               // round-(t+1) push rows of this shard's nodes [slot][2][W]
    // code rows: round-(t+1) receive buffer of exchange A, where rows to this
    // rank's own nodes go directly (its own block is not exchanged)
    u64 *recvA_next;
    const uint32_t *spos_cur; // slot of x in recvB (exchange B of round t)
    const uint32_t *spos_next;// slot of x in sendA (exchange A of round t+1)
    ShardRows sp;             // its layout
    // harness-injected faults (gs_common.h); pend/offc exist iff f.churn != 0
    Faults f;
    u64 *pend;                // [n][2][W]: votes (bump, anyC) of nodes frozen offline
    uint32_t *offc;           // [n] rounds each node was offline (Statistics.rounds)
    uint32_t node_lo;         // global id of local node 0 (shard engine; else 0)
    // SEQ schedule (gs_seq.hip): pull batch of every node as a 2-plane class
    // code [n][2][W], and per node got << 7 | dep << 6 | level
    const u64 *Wb;
    const uint8_t *sinfo;
    // External RPCs of round t (gs_handle_received), applied after every
    // internal delivery: sorted keys node << 32 | info, info = rumor (12 bits)
    // | counter << 12 | push << 20 | new peer << 21 | record << 22 | empty << 23
    const u64 *ext;
    uint32_t n_ext;
    // launch only blocks [blk_off, blk_off + blk_count) (0: all), and with
    // obs_only != ~0 observe only that node (its codes at obs_state[0..R));
    // observation launches may instead run the blocks blk_list[0..blk_count)
    // and observe the n_obs nodes of the sorted obs_list (node obs_list[j]'s
    // codes at obs_state[j*R .. (j+1)*R))
    uint32_t blk_off, blk_count, obs_only;
    const uint32_t *blk_list, *obs_list;
    uint32_t n_obs;
    u64 *acct;                // filtered timed launches: acct[0] += *rows_cnt (block 0)
    // Live-filtered gathers (gs_common.h kSkipBit; null: every row gathered):
    // zlm = a bit per source "t(x) is live" of round t (in-list build), and
    // the node maps of the round-(t+1) planes this launch writes (transition
    // modes), read by the next build: lvm "live", cpm "complete".
    const u64 *zlm;
    u64 *lvm, *cpm;
    const u64 *rows_cnt;      // filtered, timed launches: node class rows the round's
                              // build flagged for gathering (added to acct[0] once)
    // Rumor-sliced network (gs_slice_*): this engine holds one slice of the
    // rumors of every node, so a node's RPC is empty only when it is empty in
    // every slice.  The kernels then leave empty_pull / empty_push out of st32
    // and write this slice's per-node counts instead, emin[2x] (empty pulls x
    // sent) and emin[2x + 1] (1: x's push is empty); the caller reduces them
    // with MIN over the slices, byte by byte, and adds them back.
    // Observation launches write their pending empty pulls to emin[x].
    // eadd: a reduced buffer of an earlier round, added to st32 by this
    // transition launch (gs_slice_defer: no separate apply pass).
    uint8_t *emin;
    const uint8_t *eadd;
    uint32_t w32;             // 1: eligible launches run round_kernel_w32 (gs_w32.hip)
    // a second range cleared at the start (the coarse fills of the set the
    // previous round's build consumed)
    uint32_t *zero_buf2;
    uint32_t zero_words2;
    uint32_t dlv_pack;        // DLV transition launches: 0 one node per lane, 1 a 32-bit lane
                              // word of several nodes, 2 a 64-bit one (gs_dlv4.hip)
    Geometry g;
    uint64_t seed;
    uint32_t epoch;
    uint32_t round_new;       // t+1
    uint32_t cmax, maxc, maxr;
};
constexpr uint32_t kExtPush = 1u << 20, kExtNew = 1u << 21, kExtRec = 1u << 22, kExtEmpty = 1u << 23;
// Node bit maps of the live-filtered gathers: u64 words (+ one spare word).
inline u64 node_map_words(uint32_t n) { return ((u64)n + 63u) / 64u + 1u; }
__host__ __device__ inline bool map_test(const u64 *m, uint32_t i) { return ((m[i >> 6] >> (i & 63u)) & 1ull) != 0; }

// mode: 0 = transition only (first round), 1 = deliver round t + transition
// to t+1, 2 = deliver round t and write observation outputs only,
// 3 = observe without pending deliveries.
hipError_t launch_round(const RoundArgs &a, int mode, hipStream_t s);
// DLV transition launches (modes 0 and 1, no external RPCs) with four nodes
// per lane (gs_dlv4.hip).
hipError_t launch_round_dlv4(const RoundArgs &a, int mode, hipStream_t s);
constexpr uint32_t kLiveSlots = 64, kLiveStride = 32;
// The any-live words of round t+1 (RoundArgs::live) at the end of a
// transition launch's block.
__device__ __forceinline__ void mark_any_live(uint32_t *live, uint32_t round_new, uint32_t bid, bool blk_live) {
    if (bid == 0 && threadIdx.x < kLiveSlots)  // round t's words, read by the host already
        __hip_atomic_store(&live[(((round_new + 1u) & 1u) * kLiveSlots + threadIdx.x) * kLiveStride], 0u,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0 && blk_live)
        __hip_atomic_store(&live[((round_new & 1u) * kLiveSlots + (bid & (kLiveSlots - 1u))) * kLiveStride], 1u,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Per-node arrays (planes, InRec, SibRec, target words, Statistics deltas)
// are allocated for n rounded up to whole 64-node tiles (round 3's pipelined
// round kernel read whole tiles; kept as headroom).
constexpr uint32_t kTileNodes = 64;
inline uint64_t tile_padded(uint64_t n) { return (n + kTileNodes - 1) / kTileNodes * kTileNodes; }
// The 2P gather path with a 32-bit lane word (gs_w32.hip): modes 0 and 1,
// R_pad 32 (a lane per node; the engine's default there) or 64..256 (half a
// 64-rumor word per lane; only when SAFE_GOSSIP_AMD_W32=1 forces it),
// live-filtered gathers, no external RPCs, the whole grid.
bool w32_eligible(const RoundArgs &a, int mode);
hipError_t launch_round_w32(const RoundArgs &a, int mode, hipStream_t s);

// Plan of the in-list build (gs_inlist.hip).
struct CsrPlan {
    uint32_t n;       // nodes (= edges)
    uint32_t binned;  // 1: binned two-launch path; 0: generic CSR path
    uint32_t bin;     // target nodes per bin (power of two)
    uint32_t logbin;
    uint32_t nb;      // bins
    uint32_t ba;      // source chunks
    uint32_t chunk;   // sources per chunk
    uint32_t tailcap; // binned: capacity of the in-degree > kInline tail list
    uint32_t dlv;     // delivery records (DlvRec) instead of InRec / SibRec
    // binned, small networks: the partition writes 2^sub parts per bin, each
    // in its own region of kBinCap >> sub slots with its fill count at
    // scratch[fill_off + part], so each sort block reads only its part
    // (sub = 0: whole bins, fills at scratch[0, nb))
    uint32_t sub;
    uint32_t fill_off;
};
CsrPlan csr_plan(uint32_t n);
// The plan of the DLV path (binned only; tails sized for kDlvInline), or one
// with binned == 0 when n is too large for it.
CsrPlan dlv_plan(uint32_t n);
struct InListSizes {
    size_t src_words, region_words, scratch_words;  // u32 words
};
InListSizes inlist_sizes(const CsrPlan &p);
void inlist_zero_range(const CsrPlan &p, size_t *first, size_t *words);
// DLV: the coarse shard fills (cleared one round later than the other counters).
void inlist_cfill_range(const CsrPlan &p, size_t *first, size_t *words);

struct InListArgs {
    CsrPlan p;
    uint32_t *tg;       // [n] targets of the round
    // DLV path (dlv != 0, binned, R_pad <= 16): records carry push codes read
    // from the round's planes S (small-segment geometry g)
    uint32_t dlv;
    const u64 *S;
    const uint32_t *PC;     // push codes of the round (written by the round kernel)
    // known masks of the round (state != A, R_pad bits; single engine): with
    // PC[y] they are all a target's planes say about its pull batch
    const uint16_t *KN;
    uint32_t prezeroed;     // 1: the round kernel before cleared the counters (RoundArgs::zero_*)
    Geometry g;
    DlvRec *DR;         // [n]
    uint32_t *dtail;    // [tailcap] push codes of pushers >= kDlvInline
    uint32_t *pull;     // [n] PULL: pull batch of every pusher
    InRec *IN8;         // [n]
    SibRec *SIB8;       // [n]
    uint32_t *src;      // tails (binned) or the full CSR (generic)
    uint32_t *region;   // binned: [nb][cap] (source, target in the bin) records; generic: u64 pairs[n]
    uint32_t *scratch;  // binned: fill[nb], tailcnt (zero between builds); generic: M, tot, base
    uint32_t *flags;    // flags[2]: device-limit bit
    uint32_t serial;
    uint64_t seed;
    uint32_t epoch, round;
    Faults f;           // edges that are not delivered are left out of the lists
    // Live-filtered gathers (binned path; null: no skip flags): node maps of
    // the round's planes ("live", "complete", written by the round kernel
    // before) and the per-source map zl = "t(x) is live" written here.
    const u64 *lvm, *cpm;
    u64 *zl;
    u64 *rows;          // + node class rows the flags leave to gather (zeroed by the caller)
    // Code-row shard engine (DLV build over received rows; null otherwise):
    // the sources are the slot keys [0, nkeys) of exchange A (ascending key =
    // ascending source id, gs_shard.hip), their (target, push code) come from
    // the rows rowsA, the targets are the ntargets local nodes (p.n =
    // max(nkeys, ntargets)), and the pull batches go to pullB at each key's
    // exchange-B slot; t(y)'s pusher is the one whose row has kRowMutual.
    const uint32_t *rowsA;
    uint32_t *pullB;
    ShardRows sr;
    uint32_t nkeys, ntargets;
    // This rank's own block is not exchanged (the self block of a send
    // buffer and of a receive buffer have the same slots): its rows were
    // written straight into rowsA by the round kernel, their count per part
    // is self_cnt[h] (the plan's, no empty-slot marks), and the pulls answering
    // them go straight to pullB_self (the exchange-B receive buffer).
    uint32_t self_rank;
    const uint32_t *self_cnt;
    uint32_t *pullB_self;
};
// Peer choices of `round` (into tg) and their in-lists (IN8, SIB8 tagged with
// `serial`).  Depends on nothing but the Philox stream, so it runs on its own
// stream concurrently with the round kernel of the round before.
hipError_t launch_build_inlists(const InListArgs &a, hipStream_t s);
// A DLV plan's sort parts hold 2^*log targets and own *per tail slots each
// (the decoding of DlvRec::mf, RoundArgs::dlv_tlog / dlv_tper).
void dlv_tail_parts(const CsrPlan &p, uint32_t *log, uint32_t *per);
hipError_t launch_stats_fold(uint32_t *st32, u64 *st64, uint32_t n, uint32_t st16, hipStream_t s);
// Rumor slices: st32 empty_pull / empty_push += emin[2x] / emin[2x + 1].
hipError_t launch_slice_apply(uint32_t *st32, const uint8_t *emin, uint32_t n, uint32_t st16, hipStream_t s);

// ---------------------------------------------------------------- SEQ
// The literal harness order (gs_seq.hip): per round, seq_levels classifies
// every node (does it get a pull, does its pull depend on t(x)'s, the depth of
// that chain), then one pull pass per level builds W(x) for the nodes of that
// level from W(t(x)) of the level before.
struct SeqArgs {
    const u64 *S;             // round-t planes
    const InRec *IN8;
    const SibRec *SIB8;
    const uint32_t *src;
    const uint32_t *tg;
    uint32_t serial;
    uint8_t *sinfo;           // [n] got << 7 | dep << 6 | level
    u64 *Wb;                  // [n][2][W] pull batches (2-plane class code)
    uint32_t *flags;          // flags[2] device limit, flags[3] deepest level
    Geometry g;
    // per-level node lists: bcnt [blocks][kSeqLists] counts -> offsets,
    // ltot [kSeqLists] list sizes, lists [n] node ids grouped by level
    uint32_t *bcnt, *ltot, *lists;
};
constexpr uint32_t kSeqLists = 16;  // levels >= 15 share the last list
inline uint32_t seq_blocks(uint32_t n) { return (n + 255u) / 256u; }
// seq_levels + the per-level lists (ltot read back by the caller)
hipError_t launch_seq_levels(const SeqArgs &a, hipStream_t s);
// pass `level` over the `count` nodes listed from `start` of lists
hipError_t launch_seq_pull_pass(const SeqArgs &a, uint32_t level, uint32_t start, uint32_t count,
                                hipStream_t s);

// ---------------------------------------------------------------- shards
// One rank's slice of a network sharded over G ranks (gs_shard.hip).
constexpr uint32_t kMaxShards = 64;
constexpr uint32_t kMaxParts = 4;  // pipeline parts of a rank's node range
struct ShardPlan {
    uint32_t n;         // global nodes
    uint32_t G, g;      // ranks, this rank
    uint32_t chunk;     // nodes per rank (multiple of 256)
    uint32_t lo, m;     // owned range [lo, lo+m)
    uint32_t nblk_own;  // 256-source plan blocks over the owned range
    uint32_t W;         // words per plane of a row (rows are 2W words)
    // Pipeline parts: the owned range is cut into P parts of mP nodes (a
    // multiple of 256, the same on every rank); the round kernel of part h
    // runs while the exchanges of the other parts are in flight.  Each
    // exchange is stored part-major: part h's region holds one sub-block of
    // capP row slots per rank (exchange A: the last part's sub-blocks also
    // carry idrows rows of next-round source ids), so the exchange of one part
    // is ONE equal-split all-to-all over a contiguous region.
    uint32_t P, mP, bP; // parts, nodes per part, plan blocks per part
    uint32_t capP;      // row slots per (source rank, destination rank, part)
    uint32_t idrows;    // rows of u32 ids per block of the last part of A (P*capP ids)
    // Row format: u32 words per row of exchange A (rw) and B (rwb).  Class
    // rows (R_pad >= 32, or forced): the 2-plane class code as 2W u64 words,
    // rw = rwb = 4W, and the id rows of next round's sources.  Code rows
    // (codes = 1: delivery-record shards, R_pad <= 16, 2P): an A row is the
    // push code (b0 | b1 << 16, gs_common.h DlvRec) and the pusher's target
    // local to the receiving rank with bit 31 set when the pusher is its
    // target's own target (kRowMutual; an empty slot's target word is
    // 0xFFFFFFFF), rw = 2; a B row is the pull code, rwb = 1; no id rows (the
    // receiver needs no in-lists ahead: its build sorts the arrived rows).
    uint32_t rw, rwb, codes;
};
constexpr uint32_t kRowMutual = 1u << 31;
// Row slot of (rank block s, part h, index i) in an exchange-A / -B buffer.
template <class SP>
__host__ __device__ inline uint32_t shard_blockA(const SP &P, uint32_t h) {
    return P.capP + (h + 1u == P.P ? P.idrows : 0u);
}
template <class SP>
__host__ __device__ inline uint32_t shard_a_slot(const SP &P, uint32_t s, uint32_t h, uint32_t i) {
    return h * P.G * P.capP + s * shard_blockA(P, h) + i;
}
template <class SP>
__host__ __device__ inline uint32_t shard_b_slot(const SP &P, uint32_t s, uint32_t h, uint32_t i) {
    return (h * P.G + s) * P.capP + i;
}
template <class SP>
__host__ __device__ inline uint32_t shard_slotsA(const SP &P) {
    return P.G * (P.P * P.capP + P.idrows);
}
template <class SP>
__host__ __device__ inline uint32_t shard_slotsB(const SP &P) { return P.G * P.P * P.capP; }
struct SlotPos {
    uint32_t s, h, i;  // i >= capP: an id row
};
template <class SP>
__host__ __device__ inline SlotPos shard_a_decode(const SP &P, uint32_t e) {
    const uint32_t reg = P.G * P.capP;
    uint32_t h = e / reg;
    if (h > P.P - 1u) h = P.P - 1u;
    const uint32_t r = e - h * reg, ba = shard_blockA(P, h);
    const uint32_t s = r / ba;
    return SlotPos{s, h, r - s * ba};
}
// Pushers are listed in ascending source order = ascending (s, h, i).
template <class SP>
__host__ __device__ inline uint32_t shard_slot_key(const SP &P, const SlotPos &q) {
    return (q.s * P.P + q.h) * P.capP + q.i;
}
template <class SP>
__host__ __device__ inline uint32_t shard_key_slot(const SP &P, uint32_t key) {
    const uint32_t per = P.P * P.capP;
    const uint32_t s = key / per, r = key - s * per, h = r / P.capP;
    return shard_a_slot(P, s, h, r - h * P.capP);
}
template <class SP>
__host__ __device__ inline uint32_t shard_key_bslot(const SP &P, uint32_t key) {
    const uint32_t per = P.P * P.capP;
    const uint32_t s = key / per, r = key - s * per, h = r / P.capP;
    return shard_b_slot(P, s, h, r - h * P.capP);
}
// u32-word offsets inside one plan set (round r: targets and send slots of
// the owned sources) and one in-list set (round r: receive-slot in-lists).
struct ShardPlanLayout {
    size_t tg, SPOSA, SPOSB, bc_d, cnt;
};
struct ShardEdgeLayout {
    size_t fill, region, EP, IN, IN2;
};
// codes: one u32 code per row (delivery-record shards; no row flags), and
// parts of whole 1024-node blocks (the packed DLV round kernel's blocks)
ShardPlan shard_plan(uint32_t n, uint32_t G, uint32_t g, uint32_t W, uint32_t parts, bool codes = false);
size_t shard_plan_words(const ShardPlan &P, ShardPlanLayout *L);
size_t shard_edge_words(const ShardPlan &P, ShardEdgeLayout *L);
// A class-row shard's next-round in-list build (edge_bin) keeps 8 B of LDS
// per 2 K-node bin: ranks of up to 16256 bins (33.3 M nodes) fit gfx950's
// 160 KiB; check_config refuses larger ones (GS_ERR_UNSUPPORTED).
constexpr size_t kEdgeBinMaxLds = 159u * 1024u;  // (1 KiB left for its static LDS)
bool shard_edges_fit(const ShardPlan &P);
// Plan of `round`: owned targets, send slots, and the ids of every block of
// the exchange-A buffer bufA (which carries them one round ahead).
hipError_t launch_shard_plan(const ShardPlan &P, const ShardPlanLayout &L, uint32_t *words, u64 *bufA,
                             uint64_t seed, uint32_t epoch, uint32_t round, const Faults &f,
                             uint32_t *flags, hipStream_t s);
// In-lists of `round` from the ids received in recvA; tg = the plan's owned targets.
hipError_t launch_shard_edges(const ShardPlan &P, const ShardEdgeLayout &L, uint32_t *words,
                              const u64 *recvA, const uint32_t *tg, uint64_t seed, uint32_t epoch,
                              uint32_t round, const Faults &f, uint32_t *flags, hipStream_t s);

struct PullArgs {
    const u64 *S;          // round-t planes of the owned nodes
    const uint4 *IN;       // round-t in-lists of receive slots
    const uint32_t *IN2;   // their third pushers
    const uint32_t *EP;
    const u64 *recvA;      // round-t push rows received (slots of 2W words)
    u64 *sendB;            // pull rows out (exchange-B slots: A slot (s, h, i) -> B slot (s, h, i))
    ShardPlan P;
    Geometry g;            // local geometry (n = m)
};
hipError_t launch_pull(const PullArgs &a, hipStream_t s);
// Code-row shards, observers: pull[x] = the pull code x received in round t
// (recvB at x's exchange-B slot spos[x]; 0 without one).
hipError_t launch_shard_pull_unpack(const uint32_t *spos, const uint32_t *recvB, uint32_t *pull, uint32_t m,
                                    hipStream_t s);

// ---------------------------------------------------------------- signatures
// gs_verify.hip: SHA3-512 and ed25519 over SHA3-512, one item per lane;
// item i's bytes are data[off[i] .. off[i] + len[i]) (device buffers).
hipError_t launch_sha3_512(const uint8_t *data, const uint32_t *off, const uint32_t *len, uint32_t count,
                           uint8_t *out, hipStream_t s);
hipError_t launch_ed25519_verify(const uint8_t *pub, const uint8_t *sig, const uint8_t *msg, const uint32_t *off,
                                 const uint32_t *len, uint32_t count, uint8_t *ok, hipStream_t s);
hipError_t launch_ed25519_sign(const uint8_t *seed, const uint8_t *msg, const uint32_t *off, const uint32_t *len,
                               uint32_t count, uint8_t *pub, uint8_t *sig, hipStream_t s);

// Reductions for observers.
// nodes_complete counts nodes knowing >= min_known rumors.
hipError_t launch_known_reduce(const u64 *known, uint32_t n, uint32_t KW, uint32_t min_known,
                               u64 *partials /* [2*blocks] */, uint32_t blocks,
                               hipStream_t s);
// Per node: |known| (popcount over KW words) into counts[n].
hipError_t launch_known_popc(const u64 *known, uint32_t n, uint32_t KW, uint32_t *counts, hipStream_t s);
// Observation of queued injections (node << 32 | rumor): known bit set, state
// B{0,1}, records dropped; state/rec may be null.
hipError_t launch_obs_pending(const u64 *pairs, uint32_t m, uint32_t R, u64 *known, uint16_t *state,
                              uint16_t *rec, hipStream_t s);
// The digests of a sliced network (gs_digest_finish): per node the mixed word
// sums of dpart[n][words] plus the node term of psize and stats[n][5].
hipError_t launch_digest_finish(const u64 *dpart, uint32_t n, uint32_t words, const uint32_t *psize,
                                const u64 *stats, u64 *out, hipStream_t s);
hipError_t launch_stats_reduce(const u64 *stats, uint32_t n, int op,
                               u64 *partials /* [5*blocks] */, uint32_t blocks,
                               hipStream_t s);

}  // namespace gs
