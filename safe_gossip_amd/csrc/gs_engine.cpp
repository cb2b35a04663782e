// gs_engine.cpp -- host side of the C ABI (include/safe_gossip.h): device
// memory, round sequencing, injections and observers.  All compute is in
// gs_kernels.hip; there is no CPU fallback -- every entry point fails with
// GS_ERR_HIP when the device path cannot run.
#include "../../include/safe_gossip.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "gs_common.h"
#include "gs_kernels.h"

using gs::u64;

struct gs_engine {
    gs::Geometry g{};
    uint64_t seed = 0;
    uint32_t epoch = 0;
    gs::Faults faults{};
    bool seq = false;              // GS_SCHED_SEQ (gs_seq.hip)
    u64 *Wb = nullptr;             // SEQ: pull batch of every node [n][2][W]
    uint8_t *sinfo = nullptr;      // SEQ: got/dep/level per node
    uint32_t *seqw = nullptr;      // SEQ: block counts, list sizes, level lists
    uint32_t seq_round = ~0u;      // round whose pull batches Wb holds
    u64 *pend = nullptr;       // churn: votes of frozen (offline) nodes [n][2][W]
    uint32_t *offc = nullptr;  // churn: rounds offline per node
    uint8_t cmax = 0, maxc = 0, maxr = 0;
    int device = 0;
    hipStream_t stream = nullptr;
    u64 *S[2] = {nullptr, nullptr};
    int cur = 0;
    // In-edge lists, double-buffered: set (r & 1) holds round r's lists.  The
    // set of round r+1 is built on the engine stream right after the round
    // kernel of round r (beside it measured slower).
    struct CsrSet {
        uint32_t *src = nullptr, *tg = nullptr, *scratch = nullptr, *region = nullptr;
        gs::InRec *IN8 = nullptr;
        gs::SibRec *SIB8 = nullptr;
        gs::DlvRec *DR = nullptr;  // DLV path: delivery records (src holds the tails' codes)
        uint32_t *pull = nullptr;  // DLV path: PULL[x]
        u64 *zl = nullptr;         // live-filtered gathers: per source "t(x) is live"
        uint32_t serial = 0;
        uint32_t wraps = 0;        // serial wraps this set's SibRecs were cleared for
    } csr[2];
    uint32_t serial_wraps = 0;
    // Live-filtered gathers (gs_common.h kSkipBit): node maps "live" and
    // "complete" of the planes the last transition launch wrote, read by the
    // in-list build that follows it on the same stream.  On for the 2P gather
    // path with binned in-lists (W <= 8); SAFE_GOSSIP_AMD_FILTER=0 disables.
    bool filt = false;
    u64 *lvm = nullptr, *cpm = nullptr;
    u64 *rows_dev = nullptr;     // [2] per in-list set: node class rows its flags leave to gather
    uint32_t filt_launches = 0;  // MODE-1 launches counted in acct since set_timing(1)
    bool dlv = false;  // delivery-record path (2P, R_pad <= 16, binned in-lists)
    // its transition launches with several nodes per lane (gs_dlv4.hip):
    // SAFE_GOSSIP_AMD_DLV_PACK = 0 one node per lane, u64 four 16-bit nodes
    // per 64-bit lane word, otherwise (default) a 32-bit lane word
    uint32_t dlv_pack = 1;
    bool w32 = false;  // 2P gather path: the 32-bit lane round kernel on eligible launches (gs_w32.hip)
    u64 *acct = nullptr;       // filtered timed launches: class rows counted by the builds (acct[0])
    uint32_t *pc = nullptr;  // DLV: push codes of the current round [n]
    uint16_t *kn = nullptr;  // single-engine DLV: known masks of the current round [n]
    hipStream_t cstream = nullptr;  // shard engines: plan / in-list side stream
    uint32_t build_serial = 0;
    uint32_t *flags = nullptr;
    gs::CsrPlan plan{};
    // Shard engine (gs_shard_create): this rank's node range of a network
    // sharded over `world` ranks.  The plan of round r (owned targets, send
    // slots) lives in set r % 3, the in-lists of round r in set r % 2, and
    // exchange A of round t (rows of round t + ids of round t+1) in buffer
    // set t % 2 (gs_shard.hip).
    bool shard = false;
    uint32_t n_global = 0;
    // Rumor slice (cfg.rumor_slice): this engine holds a slice of the rumors
    // of all n nodes; the round kernel writes this slice's empty-RPC counts to
    // eb[0..2] (2n bytes, round t writes eb[t % 3]) and eb[3] (n bytes,
    // observations), caller-owned (gs_slice_bind), reduced with MIN over the
    // slices; eb_defer = a reduced buffer the next transition launch adds.
    bool slice = false;
    uint8_t *eb[4] = {nullptr, nullptr, nullptr, nullptr};
    int eb_defer = -1;
    gs::ShardPlan sp{};
    gs::ShardPlanLayout spl{};
    gs::ShardEdgeLayout sel{};
    uint32_t *planw[3] = {nullptr, nullptr, nullptr};
    uint32_t *edgew[2] = {nullptr, nullptr};
    hipEvent_t ev_plan[3] = {nullptr, nullptr, nullptr};  // plan set i built
    hipEvent_t ev_edges[2] = {nullptr, nullptr};          // in-list set i built
    hipEvent_t ev_main = nullptr;                          // engine stream position (cstream waits)
    u64 *sendA[2] = {nullptr, nullptr}, *recvA[2] = {nullptr, nullptr};
    u64 *sendB = nullptr, *recvB = nullptr;
    // (code-row shards, dlv && shard: round t's delivery records are built
    // into csr[0] from the rows exchange A delivered, gs_shard_pull)
    uint32_t pulled_round = 0;  // round whose gs_shard_pull ran (its plan of t+2 is launched)
    // Pipeline parts of the round in progress (gs_shard_round_part): parts
    // [0, parts_done) are launched with the arguments `ra` (mode ra_mode).
    uint32_t parts_done = 0;
    gs::RoundArgs ra{};
    int ra_mode = 0;
    bool ra_prezeroed = false;  // the round kernel clears the next build's counters
    uint32_t *st32 = nullptr;  // [n][4] u32 deltas (u16 with st16)
    bool st16 = false;         // delivery-record engines: u16 deltas (gs_device.h load_stats)
    u64 *st64 = nullptr;       // [n][4] folded totals
    uint32_t *live = nullptr;  // any-live words (gs_kernels.h RoundArgs::live)
    uint32_t fold_every = 1, since_fold = 0;
    u64 *inj_key = nullptr, *inj_mask = nullptr;
    u64 *inj_host = nullptr;  // pinned staging [2*cap]
    uint32_t inj_cap = 0;
    std::vector<std::pair<uint32_t, uint32_t>> pending;
    // Wire format (gs_wire.cpp): the message bytes (BTreeMap key) of every
    // rumor slot, and the external RPCs of the pending round (gs_handle_received)
    std::vector<std::string> keys;
    std::map<std::string, uint32_t> key_rumor;
    std::vector<uint32_t> key_order;        // rumor slots in key (byte) order
    struct Ext {
        uint32_t node, seq, info, peer;
    };
    std::vector<Ext> ext;                   // in call order
    std::set<std::pair<uint32_t, uint32_t>> ext_peers;  // (node, peer) heard from this round
    std::map<uint32_t, uint32_t> ext_fp;  // rumor slices: answered external first Pushes per node this round
    uint32_t ext_limit = 0;               // rumor slices: the network's bound on them (0: this slice's own)
    u64 *ext_dev = nullptr;
    uint32_t ext_cap = 0, ext_uploaded = 0;
    uint16_t *node_state = nullptr;         // one node's observed codes [R]
    // gs_handle_received_batch scratch, grown only (a hipFree would
    // synchronise the device at every batch): block + node lists, codes
    uint32_t *batch_lists = nullptr;
    uint16_t *batch_codes = nullptr;
    size_t batch_lists_cap = 0, batch_codes_cap = 0;
    uint32_t round = 0;
    bool deliver_pending = false;
    // observation buffers (lazy)
    u64 *obs_known = nullptr, *obs_stats = nullptr, *partials = nullptr;
    uint16_t *obs_state = nullptr, *obs_rec = nullptr;
    uint32_t *obs_psize = nullptr;
    u64 *obs_digest = nullptr;
    u64 *obs_pend = nullptr;       // queued send_new (node << 32 | rumor) shown to observers
    uint32_t obs_pend_cap = 0;
    bool obs_valid = false;
    bool started = false;          // some send_new since the last clear (Error::AlreadyStarted)
    hipEvent_t lt0 = nullptr, lt1 = nullptr;  // the last round's first / last timing event
    bool timing = false, timed = false;
    // per-round kernel timing ring (gs_round_kernel_times): kMaxParts event
    // pairs per round (one per pipeline part; the round's time is their sum)
    std::vector<hipEvent_t> tev;
    std::vector<uint8_t> tparts;  // parts timed per slot
    uint32_t tcount = 0;
    uint32_t tslot = ~0u;  // timing slot of the round in progress
};

namespace {

constexpr uint32_t kReduceBlocks = 1024;
constexpr uint32_t kTimingSlots = 4096;

// A failing HIP call returns GS_ERR_HIP; SAFE_GOSSIP_AMD_DEBUG=1 also names
// it on stderr (call, line, HIP error).
void report_hip(hipError_t err, const char *what, int line) {
    static const bool on = [] {
        const char *v = std::getenv("SAFE_GOSSIP_AMD_DEBUG");
        return v && *v && *v != '0';
    }();
    if (on) std::fprintf(stderr, "safe_gossip_amd: %s failed at gs_engine.cpp:%d: %s\n", what, line,
                         hipGetErrorString(err));
}
#define GS_HIP(expr)                                   \
    do {                                               \
        hipError_t _e = (expr);                        \
        if (_e != hipSuccess) {                        \
            report_hip(_e, #expr, __LINE__);           \
            return GS_ERR_HIP;                         \
        }                                              \
    } while (0)

uint32_t next_pow2(uint32_t v) {
    uint32_t p = 1;
    while (p < v) p <<= 1;
    return p;
}
uint32_t ilog2(uint32_t v) {
    uint32_t l = 0;
    while ((1u << l) < v) ++l;
    return l;
}

gs_status set_device(gs_engine *e) {
    return hipSetDevice(e->device) == hipSuccess ? GS_OK : GS_ERR_HIP;
}

template <typename T>
hipError_t dalloc(T **p, size_t count) {
    return hipMalloc((void **)p, std::max<size_t>(count, 1) * sizeof(T));
}

void release(gs_engine *e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    if (e->cstream) (void)hipStreamSynchronize(e->cstream);
    for (auto &c : e->csr) {
        void *cb[] = {c.src, c.tg, c.scratch, c.region, c.IN8, c.SIB8, c.DR, c.pull, c.zl};
        for (void *b : cb)
            if (b) (void)hipFree(b);
    }
    for (int i = 0; i < 3; ++i) {
        if (e->planw[i]) (void)hipFree(e->planw[i]);
        if (e->ev_plan[i]) (void)hipEventDestroy(e->ev_plan[i]);
    }
    for (int i = 0; i < 2; ++i) {
        if (e->edgew[i]) (void)hipFree(e->edgew[i]);
        if (e->ev_edges[i]) (void)hipEventDestroy(e->ev_edges[i]);
    }
    if (e->ev_main) (void)hipEventDestroy(e->ev_main);
    if (e->cstream) (void)hipStreamDestroy(e->cstream);
    void *bufs[] = {e->lvm, e->cpm, e->rows_dev, e->acct, e->pc, e->kn, e->Wb, e->sinfo, e->seqw, e->pend, e->offc, e->S[0], e->S[1], e->flags, e->live, e->st32, e->st64, e->inj_key, e->inj_mask, e->obs_known, e->obs_stats,
                    e->partials, e->obs_state, e->obs_rec, e->obs_psize, e->obs_digest, e->obs_pend, e->ext_dev,
                    e->node_state, e->batch_lists, e->batch_codes};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    if (e->inj_host) (void)hipHostFree(e->inj_host);
    for (hipEvent_t ev : e->tev) (void)hipEventDestroy(ev);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
}

gs_status reset_state(gs_engine *e) {
    const gs::Geometry &g = e->g;
    GS_HIP(hipStreamSynchronize(e->cstream));
    const size_t sw = (size_t)g.units * gs::kPlanes * g.W;
    GS_HIP(hipMemsetAsync(e->S[0], 0, sw * sizeof(u64), e->stream));
    GS_HIP(hipMemsetAsync(e->S[1], 0, sw * sizeof(u64), e->stream));
    GS_HIP(hipMemsetAsync(e->st32, 0, (size_t)4 * g.n * sizeof(uint32_t), e->stream));
    GS_HIP(hipMemsetAsync(e->st64, 0, (size_t)4 * g.n * sizeof(u64), e->stream));
    if (e->offc) GS_HIP(hipMemsetAsync(e->offc, 0, (size_t)g.n * sizeof(uint32_t), e->stream));
    e->since_fold = 0;
    GS_HIP(hipMemsetAsync(e->flags, 0, 4 * sizeof(uint32_t), e->stream));
    GS_HIP(hipMemsetAsync(e->live, 0, (size_t)2 * gs::kLiveSlots * gs::kLiveStride * sizeof(uint32_t), e->stream));
    if (e->dlv) {  // both sets' coarse fills (the round kernels clear them a round late)
        size_t first = 0, words = 0;
        gs::inlist_cfill_range(e->plan, &first, &words);
        for (auto &c : e->csr)
            if (words && c.scratch) GS_HIP(hipMemsetAsync(c.scratch + first, 0, words * sizeof(uint32_t), e->stream));
    }
    e->cur = 0;
    e->round = 0;
    e->eb_defer = -1;  // (Statistics restart from zero)
    e->seq_round = ~0u;
    e->pulled_round = 0;
    e->parts_done = 0;
    e->deliver_pending = false;
    e->pending.clear();
    e->obs_valid = false;
    e->started = false;
    e->ext.clear();
    e->ext_peers.clear();
    e->ext_fp.clear();
    e->ext_uploaded = 0;
    return GS_OK;
}

// The pending round's external RPCs, sorted by (node, call order), on the device.
gs_status upload_ext(gs_engine *e) {
    const uint32_t m = (uint32_t)e->ext.size();
    if (m == e->ext_uploaded) return GS_OK;
    if (m > e->ext_cap) {
        GS_HIP(hipStreamSynchronize(e->stream));
        if (e->ext_dev) (void)hipFree(e->ext_dev);
        e->ext_dev = nullptr;
        e->ext_cap = 0;
        const uint32_t cap = std::max<uint32_t>(1024, 2 * m);
        GS_HIP(dalloc(&e->ext_dev, cap));
        e->ext_cap = cap;
    }
    std::vector<gs_engine::Ext> v(e->ext);
    std::stable_sort(v.begin(), v.end(), [](const gs_engine::Ext &a, const gs_engine::Ext &b) {
        return a.node != b.node ? a.node < b.node : a.seq < b.seq;
    });
    std::vector<u64> keys(m);
    for (uint32_t i = 0; i < m; ++i) keys[i] = ((u64)v[i].node << 32) | v[i].info;
    GS_HIP(hipStreamSynchronize(e->stream));  // the previous upload may still be read
    // on the engine stream, waited for (keys is a host temporary; a hipMemcpy
    // on the null stream is not ordered before the non-blocking engine stream)
    GS_HIP(hipMemcpyAsync(e->ext_dev, keys.data(), m * sizeof(u64), hipMemcpyHostToDevice, e->stream));
    GS_HIP(hipStreamSynchronize(e->stream));
    e->ext_uploaded = m;
    return GS_OK;
}

// flags[2]: a device limit was hit since the last clear (in-degree > kMaxIn,
// in-list bin / tail overflow, SEQ level overflow, shard receive capacity).
gs_status device_limit(gs_engine *e) {
    uint32_t fl = 0;
    GS_HIP(hipStreamSynchronize(e->cstream));  // in-list builds may run there
    GS_HIP(hipMemcpyAsync(&fl, e->flags + 2, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
    GS_HIP(hipStreamSynchronize(e->stream));
    return fl ? GS_ERR_DEVICE_LIMIT : GS_OK;
}

gs::RoundArgs base_args(gs_engine *e) {
    gs::RoundArgs a{};
    a.Scur = e->S[e->cur];
    a.Snext = e->S[e->cur ^ 1];
    if (e->dlv) gs::dlv_tail_parts(e->plan, &a.dlv_tlog, &a.dlv_tper);  // (DlvRec tail offsets)
    if (e->shard) {
        const uint32_t t = e->round;
        uint32_t *cur = e->planw[t % 3], *nxt = e->planw[(t + 1) % 3], *ed = e->edgew[t % 2];
        a.IN = reinterpret_cast<const uint4 *>(ed + e->sel.IN);
        a.IN2 = ed + e->sel.IN2;
        a.src = ed + e->sel.EP;
        a.spos_cur = cur + e->spl.SPOSB;
        a.spos_next = nxt + e->spl.SPOSA;
        a.tg = cur + e->spl.tg;
        a.node_lo = e->sp.lo;
        a.tg_next = nxt + e->spl.tg;
        a.recvA = e->recvA[t % 2];
        a.recvB = e->recvB;
        a.sendA = e->sendA[(t + 1) % 2];
        a.sp = gs::ShardRows{e->sp.G,  e->sp.P,   e->sp.W,     e->sp.capP,  e->sp.idrows,
                             e->sp.rw, e->sp.rwb, e->sp.codes, e->sp.chunk, e->sp.n};
        if (e->dlv) {  // code rows: the delivery records built from exchange A (gs_shard_pull)
            a.DR = e->csr[0].DR;
            a.dtail = e->csr[0].src;
            a.recvA_next = e->recvA[(t + 1) % 2];  // (rows to this rank's own nodes)
        }
    } else {
        const auto &cs = e->csr[e->round & 1u];  // round-t lists (t = e->round)
        a.IN8 = cs.IN8;
        a.SIB8 = cs.SIB8;
        a.DR = cs.DR;
        a.dtail = e->dlv ? cs.src : nullptr;
        a.pull = cs.pull;
        a.pc_out = e->pc;
        a.kn_out = e->kn;
        a.src = cs.src;
        a.tg = cs.tg;
        a.serial = cs.serial;
        if (e->filt) {
            a.zlm = cs.zl;
            a.lvm = e->lvm;
            a.cpm = e->cpm;
        }
    }
    a.st32 = e->st32;
    a.st16 = e->st16 ? 1u : 0u;
    a.st64 = e->st64;
    a.f = e->faults;
    a.pend = e->pend;
    a.offc = e->offc;
    if (e->seq) {
        a.Wb = e->Wb;
        a.sinfo = e->sinfo;
    }
    a.obs_rounds = e->round;
    a.flags = e->flags;
    a.live = e->live;
    if (e->deliver_pending && !e->ext.empty()) {  // uploaded by the caller (upload_ext)
        a.ext = e->ext_dev;
        a.n_ext = e->ext_uploaded;
    }
    a.obs_only = 0xFFFFFFFFu;
    a.dlv_pack = e->dlv_pack;
    a.w32 = e->w32 ? 1u : 0u;
    a.g = e->g;
    a.seed = e->seed;
    a.epoch = e->epoch;
    a.round_new = e->round + 1;
    a.cmax = e->cmax;
    a.maxc = e->maxc;
    a.maxr = e->maxr;
    return a;
}

gs_status upload_injections(gs_engine *e, uint32_t *n_inj) {
    *n_inj = 0;
    if (e->pending.empty()) return GS_OK;
    const gs::Geometry &g = e->g;
    std::vector<std::pair<u64, u64>> km;
    km.reserve(e->pending.size());
    for (auto &p : e->pending) {
        const uint32_t x = p.first, r = p.second;
        if (g.small) km.emplace_back((u64)x, 1ull << r);
        else km.emplace_back((u64)x * g.W + (r >> 6), 1ull << (r & 63));
    }
    std::sort(km.begin(), km.end());
    std::vector<std::pair<u64, u64>> merged;
    for (auto &v : km) {
        if (!merged.empty() && merged.back().first == v.first) merged.back().second |= v.second;
        else merged.push_back(v);
    }
    const uint32_t m = (uint32_t)merged.size();
    if (m > e->inj_cap) {
        GS_HIP(hipStreamSynchronize(e->stream));
        if (e->inj_key) (void)hipFree(e->inj_key);
        if (e->inj_mask) (void)hipFree(e->inj_mask);
        if (e->inj_host) (void)hipHostFree(e->inj_host);
        e->inj_key = e->inj_mask = e->inj_host = nullptr;
        uint32_t cap = std::max<uint32_t>(m, 1024);
        GS_HIP(dalloc(&e->inj_key, cap));
        GS_HIP(dalloc(&e->inj_mask, cap));
        GS_HIP(hipHostMalloc((void **)&e->inj_host, 2 * (size_t)cap * sizeof(u64), 0));
        e->inj_cap = cap;
    }
    // The staging buffer may still feed a copy of an earlier round.
    GS_HIP(hipStreamSynchronize(e->stream));
    for (uint32_t i = 0; i < m; ++i) {
        e->inj_host[i] = merged[i].first;
        e->inj_host[e->inj_cap + i] = merged[i].second;
    }
    GS_HIP(hipMemcpyAsync(e->inj_key, e->inj_host, m * sizeof(u64), hipMemcpyHostToDevice, e->stream));
    GS_HIP(hipMemcpyAsync(e->inj_mask, e->inj_host + e->inj_cap, m * sizeof(u64),
                          hipMemcpyHostToDevice, e->stream));
    e->pending.clear();
    *n_inj = m;
    return GS_OK;
}

gs_status ensure_obs(gs_engine *e, bool dumps) {
    const gs::Geometry &g = e->g;
    const uint32_t KW = (g.R + 63) / 64;
    if (!e->obs_known) {
        GS_HIP(dalloc(&e->obs_known, (size_t)g.n * KW));
        GS_HIP(dalloc(&e->obs_stats, (size_t)g.n * 5));
        GS_HIP(dalloc(&e->partials, (size_t)kReduceBlocks * 5));
        GS_HIP(dalloc(&e->obs_psize, (size_t)g.n));
    }
    if (dumps && !e->obs_state) {
        GS_HIP(dalloc(&e->obs_state, (size_t)g.n * g.R));
        GS_HIP(dalloc(&e->obs_rec, (size_t)g.n * g.R));
    }
    return GS_OK;
}

// SEQ: the pull batches of the pending round (levels, then one pass per
// level), once per round, on the engine stream.
gs_status seq_prepare(gs_engine *e) {
    if (!e->seq || !e->deliver_pending || e->seq_round == e->round) return GS_OK;
    const auto &cs = e->csr[e->round & 1u];
    gs::SeqArgs sa{};
    sa.S = e->S[e->cur];
    sa.IN8 = cs.IN8;
    sa.SIB8 = cs.SIB8;
    sa.src = cs.src;
    sa.tg = cs.tg;
    sa.serial = cs.serial;
    sa.sinfo = e->sinfo;
    sa.Wb = e->Wb;
    sa.flags = e->flags;
    sa.g = e->g;
    const size_t nb = (size_t)gs::seq_blocks(e->g.n) * gs::kSeqLists;
    sa.bcnt = e->seqw;
    sa.ltot = e->seqw + nb;
    sa.lists = e->seqw + nb + gs::kSeqLists;
    GS_HIP(hipMemsetAsync(e->flags + 3, 0, sizeof(uint32_t), e->stream));
    GS_HIP(gs::launch_seq_levels(sa, e->stream));
    uint32_t maxlev = 0, ltot[gs::kSeqLists];
    GS_HIP(hipMemcpyAsync(&maxlev, e->flags + 3, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
    GS_HIP(hipMemcpyAsync(ltot, sa.ltot, sizeof(ltot), hipMemcpyDeviceToHost, e->stream));
    GS_HIP(hipStreamSynchronize(e->stream));
    uint32_t lstart[gs::kSeqLists], run = 0;
    for (uint32_t l = 0; l < gs::kSeqLists; ++l) {
        lstart[l] = run;
        run += ltot[l];
    }
    for (uint32_t l = 0; l <= maxlev; ++l) {
        const uint32_t li = std::min(l, gs::kSeqLists - 1u);
        GS_HIP(gs::launch_seq_pull_pass(sa, l, lstart[li], ltot[li], e->stream));
    }
    e->seq_round = e->round;
    return GS_OK;
}

// Code-row shards: an observation launch runs the per-node DLV kernel over
// the pull codes unpacked into node order (the delivery records are the pull
// kernel's, gs_shard_pull).
hipError_t code_rows_obs(gs_engine *e, gs::RoundArgs &a) {
    if (!(e->shard && e->dlv)) return hipSuccess;
    if (e->deliver_pending) {
        const hipError_t he = gs::launch_shard_pull_unpack(a.spos_cur, reinterpret_cast<const uint32_t *>(e->recvB),
                                                           e->pc, e->g.n, e->stream);
        if (he != hipSuccess) return he;
    }
    a.recvA = nullptr;
    a.pull = e->pc;
    return hipSuccess;
}

// Fill the observation buffers with the state after the last delivery.
gs_status observe(gs_engine *e, bool dumps, bool digest = false, u64 *dpart = nullptr, uint32_t dp_lo = 0,
                  uint32_t dp_words = 0) {
    if (e->obs_valid && !dumps && !digest && !dpart) return GS_OK;
    if (e->slice && !e->eb[3]) return GS_ERR_INVALID_ARGUMENT;  // gs_slice_bind first
    if (e->slice && e->eb_defer >= 0) {  // a deferred reduced buffer: add it now
        GS_HIP(gs::launch_slice_apply(e->st32, e->eb[e->eb_defer], e->g.n, e->st16 ? 1u : 0u, e->stream));
        e->eb_defer = -1;
    }
    gs_status st = ensure_obs(e, dumps);
    if (st == GS_OK && digest && !e->obs_digest && dalloc(&e->obs_digest, e->g.n) != hipSuccess) st = GS_ERR_HIP;
    if (st == GS_OK && e->deliver_pending) st = upload_ext(e);
    if (st != GS_OK) return st;
    gs::RoundArgs a = base_args(e);
    a.obs_known = e->obs_known;
    a.obs_stats = e->obs_stats;
    a.obs_psize = e->obs_psize;
    if (dumps) {
        a.obs_state = e->obs_state;
        a.obs_rec = e->obs_rec;
    }
    if (digest) a.obs_digest = e->obs_digest;
    a.obs_dpart = dpart;
    a.dp_lo = dp_lo;
    a.dp_words = dp_words;
    if (e->slice) a.emin = e->eb[3];  // pending empty pulls of this slice
    if (e->deliver_pending) {
        if (e->shard && !e->dlv) GS_HIP(hipStreamWaitEvent(e->stream, e->ev_edges[e->round % 2], 0));
        st = seq_prepare(e);
        if (st != GS_OK) return st;
    }
    GS_HIP(code_rows_obs(e, a));
    GS_HIP(gs::launch_round(a, e->deliver_pending ? 2 : 3, e->stream));
    if (!e->pending.empty()) {
        // Queued send_new calls: Gossip::new_message inserts MessageState::new
        // into the map at once (src/gossip.rs:71-75), so observers show the
        // rumor as known, in state B{round 0, our_counter 1}, records dropped.
        const uint32_t m = (uint32_t)e->pending.size();
        if (m > e->obs_pend_cap) {
            if (e->obs_pend) (void)hipFree(e->obs_pend);
            e->obs_pend = nullptr;
            e->obs_pend_cap = 0;
            GS_HIP(dalloc(&e->obs_pend, m));
            e->obs_pend_cap = m;
        }
        std::vector<u64> pv(m);
        for (uint32_t i = 0; i < m; ++i) pv[i] = ((u64)e->pending[i].first << 32) | e->pending[i].second;
        GS_HIP(hipMemcpyAsync(e->obs_pend, pv.data(), m * sizeof(u64), hipMemcpyHostToDevice, e->stream));
        GS_HIP(gs::launch_obs_pending(e->obs_pend, m, e->g.R, e->obs_known, a.obs_state, a.obs_rec,
                                      e->stream));
        GS_HIP(hipStreamSynchronize(e->stream));  // pv is a host temporary
    }
    gs_status st2 = device_limit(e);
    if (st2 != GS_OK) return st2;
    e->obs_valid = true;
    return GS_OK;
}

}  // namespace

extern "C" {

#ifndef GS_BUILD_ID
#define GS_BUILD_ID "unknown"
#endif
uint32_t gs_abi_version(void) { return GS_ABI_VERSION; }
const char *gs_build_id(void) { return GS_BUILD_ID; }

const char *gs_status_string(gs_status s) {
    switch (s) {
    case GS_OK: return "ok";
    case GS_ERR_NO_PEERS: return "There are no connected peers with which to gossip.";
    case GS_ERR_ALREADY_STARTED: return "Connections to all other nodes must be made before sending any messages.";
    case GS_ERR_SIG_FAILURE: return "The message or signature might be corrupted, or the signer is wrong.";
    case GS_ERR_IO: return "I/O error";
    case GS_ERR_SERIALISATION: return "Serialisation error";
    case GS_ERR_INVALID_ARGUMENT: return "invalid argument";
    case GS_ERR_UNSUPPORTED: return "parameters outside the packed state layout (counter_max<=3, max_c_rounds<=3, max_rounds<=32, R<=4096), or a shard layout the engine cannot hold (class-row rank above 33.3 M nodes)";
    case GS_ERR_HIP: return "HIP runtime error (no usable MI355X device?)";
    case GS_ERR_OUT_OF_MEMORY: return "out of device memory";
    case GS_ERR_DEVICE_LIMIT: return "device limit hit (in-degree > 30, in-list or receive-row capacity, SEQ depth)";
    }
    return "unknown";
}

void gs_derive_params(uint32_t n, uint8_t out[3]) {
    // Gossip::add_peer (src/gossip.rs:59-64): network_size == n after the
    // full mesh is built; f64 ln, ceil, `as u8` (saturating), max(1, .).
    if (n <= 1) {
        out[0] = out[1] = out[2] = 0;  // Gossip::new
        return;
    }
    auto as_u8 = [](double v) -> uint8_t {
        if (!(v > 0.0)) return 0;
        if (v >= 255.0) return 255;
        return (uint8_t)v;
    };
    const double ns = (double)n;
    const uint8_t lnln = as_u8(std::ceil(std::log(std::log(ns))));
    const uint8_t ln = as_u8(std::ceil(std::log(ns)));
    out[0] = std::max<uint8_t>(1, lnln);
    out[1] = std::max<uint8_t>(1, lnln);
    out[2] = std::max<uint8_t>(1, ln);
}

uint32_t gs_peer(uint64_t seed, uint32_t epoch, uint32_t round, uint32_t node, uint32_t n) {
    return gs::peer_of(seed, epoch, round, node, n);
}
uint32_t gs_origin(uint64_t seed, uint32_t epoch, uint32_t rumor, uint32_t n) {
    return gs::origin_of(seed, epoch, rumor, n);
}
uint32_t gs_coin(uint64_t seed, uint32_t epoch, uint32_t round, uint32_t node) {
    return gs::coin_of(seed, epoch, round, node);
}
uint32_t gs_fault(uint64_t seed, uint32_t epoch, uint32_t round, uint32_t node, uint32_t churn,
                  uint32_t drop_push, uint32_t drop_pull) {
    const gs::Ph4 w = gs::philox4(round, node, gs::kStreamFault, epoch, seed);
    return (w.w0 < churn ? 1u : 0u) | (w.w1 < drop_push ? 2u : 0u) | (w.w2 < drop_pull ? 4u : 0u);
}

}  // extern "C"

namespace {

// The exchange layout of rank `rank` of `world` (gs_shard.hip shard_plan).
gs::ShardPlan plan_of(const gs_config *cfg, uint32_t rank, uint32_t world, uint32_t parts) {
    const uint32_t R = cfg->n_rumors;
    // code rows (one u32 push / pull code per row, delivery records and the
    // packed DLV round kernel) at R_pad <= 16 in the 2P schedule;
    // SAFE_GOSSIP_AMD_NO_DLV=1 keeps class rows (every rank must agree)
    const char *nd = std::getenv("SAFE_GOSSIP_AMD_NO_DLV");
    const bool codes = !(nd && *nd && *nd != '0') && next_pow2(R) <= 16 && cfg->schedule == GS_SCHED_2P;
    return gs::shard_plan(cfg->n_nodes, world, rank, R >= 64 ? (next_pow2(R) / 64) : 1u, parts, codes);
}

// Slot keys of exchange A (sources of a code-row shard's DLV build).
uint32_t shard_keys(const gs::ShardPlan &sp) { return sp.G * sp.P * sp.capP; }

void fill_shard_info(const gs::ShardPlan &sp, uint32_t info[14]) {
    info[0] = sp.lo;
    info[1] = sp.m;
    info[2] = sp.capP;  // row slots per rank sub-block of a part
    info[3] = sp.idrows;
    // u32 words per exchange-A row: the 2-plane class code (2W u64 = 4W u32),
    // or (code rows, R_pad <= 16) the push code and the target word
    info[4] = sp.rw;
    info[5] = sp.G;
    info[6] = sp.g;
    info[7] = sp.chunk;
    info[8] = sp.P;
    info[9] = sp.mP;
    info[10] = gs::shard_slotsA(sp);  // rows of an exchange-A buffer
    info[11] = gs::shard_slotsB(sp);  // rows of an exchange-B buffer
    info[12] = sp.rwb;                // u32 words per exchange-B row
    info[13] = sp.codes;              // 1: code rows
}

// The checks of a configuration (a whole network: world == 0, or rank `rank`
// of `world` node shards with `parts` pipeline parts): the shard layout and
// the protocol parameters.  gs_create / gs_shard_create_parts and
// gs_shard_plan_info run the same checks, so a reported layout is one an
// engine can be created with.
gs_status check_config(const gs_config *cfg, uint32_t rank, uint32_t world, uint32_t parts, gs::ShardPlan *sp,
                       uint8_t p[3]) {
    const uint32_t nglob = cfg->n_nodes, R = cfg->n_rumors;
    if (nglob == 0 || nglob == 0xffffffffu || R == 0 || R > 4096) return GS_ERR_INVALID_ARGUMENT;
    if (world && (rank >= world || world > gs::kMaxShards)) return GS_ERR_INVALID_ARGUMENT;
    if (world && (parts == 0 || parts > gs::kMaxParts)) return GS_ERR_INVALID_ARGUMENT;
    if (cfg->schedule > GS_SCHED_SEQ) return GS_ERR_INVALID_ARGUMENT;
    // Target words pack t(x) into 29 bits below the delivery flags
    // (gs_common.h kTgMask), whatever the parameters.
    if (nglob > gs::kTgMask + 1u) return GS_ERR_UNSUPPORTED;
    gs_derive_params(nglob, p);
    if (cfg->counter_max) p[0] = cfg->counter_max;
    if (cfg->max_c_rounds) p[1] = cfg->max_c_rounds;
    if (cfg->max_rounds) p[2] = cfg->max_rounds;
    if (nglob >= 2 && (p[0] > 3 || p[1] > 3 || p[2] > 32 || !p[0] || !p[1] || !p[2]))
        return GS_ERR_UNSUPPORTED;
    if (world && cfg->schedule == GS_SCHED_SEQ) return GS_ERR_UNSUPPORTED;  // chains cross ranks
    // rumor slices are single engines (node shards slice nodes instead); both
    // schedules: which pushes a node answers, and when, depends on the peer
    // schedule only, and "has a live entry" only turns on within a round, so
    // its empty pulls are a nondecreasing function of the first time it is
    // live and the network's count is the MIN over the slices under SEQ too
    // (tests/test_sliced_gloo.py: the oracle per slice against one oracle)
    if (cfg->rumor_slice && world) return GS_ERR_UNSUPPORTED;
    *sp = gs::ShardPlan{};
    if (world) {
        *sp = plan_of(cfg, rank, world, parts);
        // code rows run the delivery-record build over max(owned nodes, slot
        // keys) sources: only on its binned plan
        if (sp->codes && !gs::dlv_plan(std::max(sp->m, shard_keys(*sp))).binned) return GS_ERR_UNSUPPORTED;
        // class rows build the next round's in-lists in LDS bins (gs_shard.hip edge_bin)
        if (!gs::shard_edges_fit(*sp)) return GS_ERR_UNSUPPORTED;
    }
    return GS_OK;
}

// Common constructor: a whole network (world == 0) or the node range of rank
// `rank` of a network sharded over `world` ranks.
gs_status create_engine(const gs_config *cfg, uint32_t rank, uint32_t world, uint32_t parts, gs_engine **out) {
    if (!cfg || !out) return GS_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    gs::ShardPlan sp{};
    uint8_t p[3];
    const gs_status cst = check_config(cfg, rank, world, parts, &sp, p);
    if (cst != GS_OK) return cst;
    const uint32_t nglob = cfg->n_nodes, R = cfg->n_rumors;
    const uint32_t n = world ? sp.m : nglob;  // nodes owned by this engine

    gs_engine *e = new gs_engine();
    e->shard = world != 0;
    e->slice = cfg->rumor_slice != 0;
    e->n_global = nglob;
    e->sp = sp;
    e->seed = cfg->seed;
    e->epoch = cfg->epoch;
    e->faults = gs::Faults{cfg->churn, cfg->drop_push, cfg->drop_pull};
    e->seq = cfg->schedule == GS_SCHED_SEQ;
    e->cmax = p[0];
    e->maxc = p[1];
    e->maxr = p[2];
    int dev = cfg->device;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) {
        delete e;
        return GS_ERR_HIP;
    }
    e->device = dev;
    if (hipSetDevice(dev) != hipSuccess) {
        delete e;
        return GS_ERR_HIP;
    }
    gs::Geometry &g = e->g;
    g.n = n;
    g.R = R;
    g.rpad = next_pow2(R);
    g.logr = ilog2(g.rpad);
    if (g.rpad >= 64) {
        g.small = 0;
        g.W = g.rpad / 64;
        g.lognpu = 0;
        g.units = n;
        g.nseg = (uint64_t)n * g.W;
    } else {
        g.small = 1;
        g.W = 1;
        g.lognpu = 6 - g.logr;
        const uint64_t npu = 1ull << g.lognpu;
        g.units = (n + npu - 1) / npu;
        g.nseg = n;
    }
    {
        // Delivery records (DLV) for small R in the 2P schedule: every
        // class-plane gather but one is replaced by records of the in-list
        // build.  SAFE_GOSSIP_AMD_NO_DLV=1 forces gathers.
        const char *v = std::getenv("SAFE_GOSSIP_AMD_NO_DLV");
        const bool off = v && *v && *v != '0';
        e->dlv = e->shard ? e->sp.codes != 0
                          : !off && !e->seq && g.small && g.rpad <= 16 && gs::dlv_plan(n).binned;
    }
    {
        const char *v = std::getenv("SAFE_GOSSIP_AMD_DLV_PACK");
        const std::string m = v ? v : "";
        e->dlv_pack = m == "0" ? 0u : (m == "u64" ? 2u : (m == "u32x1" ? 3u : 1u));
    }
    // (code-row shards: the DLV build's sources are the slot keys of
    // exchange A, its targets the owned nodes)
    e->plan = e->dlv ? gs::dlv_plan(e->shard ? std::max(n, shard_keys(e->sp)) : n) : gs::csr_plan(n);
    if (e->dlv && !e->plan.binned) {  // (n <= 2^27: every shard of a network the state layout holds)
        delete e;
        return GS_ERR_UNSUPPORTED;
    }
    // Default message bytes of rumor slot r: bincode of a 4-byte Vec<u8>
    // holding r big-endian (u64 length 4, then the bytes), so key order is
    // slot order.  gs_set_rumor_key replaces them.
    e->keys.resize(R);
    e->key_order.resize(R);
    for (uint32_t r = 0; r < R; ++r) {
        const char k[12] = {4, 0, 0, 0, 0, 0, 0, 0, (char)(r >> 24), (char)(r >> 16), (char)(r >> 8), (char)r};
        e->keys[r] = std::string(k, 12);
        e->key_rumor[e->keys[r]] = r;
        e->key_order[r] = r;
    }
    {
        // The 32-bit lane round kernel (gs_w32.hip) by default where a lane
        // holds one node (R_pad 32: 2^24 x 32, 1.24 -> 1.10 ms/step); at R_pad
        // 64..256 its duplicated per-node work costs more than its occupancy
        // gains (config 4: 2.61 -> 3.03 ms per launch).
        // SAFE_GOSSIP_AMD_W32=0/1 forces the 64-bit / 32-bit lane kernel.
        const char *w = std::getenv("SAFE_GOSSIP_AMD_W32");
        e->w32 = (w && *w) ? *w != '0' : (e->g.small && e->g.rpad == 32u);
    }
    {
        // SAFE_GOSSIP_AMD_FILTER=0 keeps the unfiltered kernel (parity tests)
        const char *v = std::getenv("SAFE_GOSSIP_AMD_FILTER");
        const bool off = v && *v == '0';
        e->filt = !off && !e->shard && !e->seq && !e->dlv && e->plan.binned && (g.small || g.W <= 8);
    }
    // Per round a node's Statistics deltas of internal deliveries grow by at
    // most 32*R_pad + 32 (in-degree <= 30 is enforced); fold them into u64
    // well before a wrap.  The delivery-record engines (R_pad <= 16) keep them
    // in 16 bits (8 B per node and round less to read and write; external
    // RPCs' counts go straight to the totals): a fold every >= 60 rounds.
    e->st16 = e->dlv;
    e->fold_every = (uint32_t)std::max<uint64_t>(1, (e->st16 ? 0xFFFFull : 0xFFFFFFFFull) / (32ull * g.rpad + 32) / 2);
    bool ok;
    if (e->shard) {
        // Shard engines share the device with the process group's collective
        // stream (normal priority): the engine stream takes a high-priority
        // and the plan / in-list side stream a low-priority hardware queue, so
        // neither is serialised behind an exchange on a shared queue (HIP
        // round-robins streams of one priority over GPU_MAX_HW_QUEUES queues).
        int least = 0, greatest = 0;
        ok = hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess &&
             hipStreamCreateWithPriority(&e->stream, hipStreamNonBlocking, greatest) == hipSuccess &&
             hipStreamCreateWithPriority(&e->cstream, hipStreamNonBlocking, least) == hipSuccess;
    } else {
        ok = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) == hipSuccess &&
             hipStreamCreateWithFlags(&e->cstream, hipStreamNonBlocking) == hipSuccess;
    }
    for (int i = 0; i < 3 && ok && e->shard; ++i) {
        const size_t words = gs::shard_plan_words(e->sp, &e->spl);
        ok = hipEventCreateWithFlags(&e->ev_plan[i], hipEventDisableTiming) == hipSuccess &&
             dalloc(&e->planw[i], words) == hipSuccess;
    }
    for (int i = 0; i < 2 && ok && e->shard && !e->dlv; ++i) {  // (code rows need no in-lists ahead)
        const size_t words = gs::shard_edge_words(e->sp, &e->sel);
        ok = hipEventCreateWithFlags(&e->ev_edges[i], hipEventDisableTiming) == hipSuccess &&
             dalloc(&e->edgew[i], words) == hipSuccess &&
             hipMemsetAsync(e->edgew[i], 0, words * sizeof(uint32_t), e->stream) == hipSuccess;  // (counters zero between builds)
    }
    if (ok && e->shard) ok = hipEventCreateWithFlags(&e->ev_main, hipEventDisableTiming) == hipSuccess;
    if (ok && e->shard && e->dlv) {  // one build set: built and read on the engine stream, in order
        const gs::InListSizes dz = gs::inlist_sizes(e->plan);
        auto &c = e->csr[0];
        ok = dalloc(&c.src, dz.src_words) == hipSuccess && dalloc(&c.region, dz.region_words) == hipSuccess &&
             dalloc(&c.scratch, dz.scratch_words) == hipSuccess && dalloc(&c.DR, e->plan.n) == hipSuccess;
    }
    const gs::InListSizes isz = gs::inlist_sizes(e->plan);
    // per-node arrays the pipelined round kernel reads by whole 64-node tiles
    const size_t npad = gs::tile_padded(n);
    const size_t sw_pad = (size_t)gs::tile_padded(g.units) * gs::kPlanes * g.W;
    for (int i = 0; i < 2 && ok && !e->shard; ++i) {
        auto &c = e->csr[i];
        ok = dalloc(&c.src, isz.src_words) == hipSuccess && dalloc(&c.tg, npad) == hipSuccess &&
             dalloc(&c.region, isz.region_words) == hipSuccess &&
             dalloc(&c.scratch, isz.scratch_words) == hipSuccess &&
             hipMemsetAsync(c.scratch, 0, std::max<size_t>(isz.scratch_words, 1) * sizeof(uint32_t), e->stream) == hipSuccess;
        if (ok && e->dlv) {
            ok = dalloc(&c.DR, n) == hipSuccess && dalloc(&c.pull, n) == hipSuccess;
        } else if (ok) {
            ok = dalloc(&c.IN8, npad) == hipSuccess && dalloc(&c.SIB8, npad) == hipSuccess &&
                 hipMemsetAsync(c.SIB8, 0, std::max<size_t>(n, 1) * sizeof(gs::SibRec), e->stream) == hipSuccess;
            if (ok && e->filt) ok = dalloc(&c.zl, gs::node_map_words(n)) == hipSuccess;
        }
    }
    ok = ok && dalloc(&e->S[0], sw_pad) == hipSuccess && dalloc(&e->S[1], sw_pad) == hipSuccess &&
         dalloc(&e->flags, 4) == hipSuccess && dalloc(&e->live, (size_t)2 * gs::kLiveSlots * gs::kLiveStride) == hipSuccess && dalloc(&e->st32, (size_t)4 * npad) == hipSuccess &&
         dalloc(&e->st64, (size_t)4 * n) == hipSuccess;
    if (ok && e->dlv) ok = dalloc(&e->pc, n) == hipSuccess && (e->shard || dalloc(&e->kn, n) == hipSuccess);
    if (ok && e->filt)
        ok = dalloc(&e->lvm, gs::node_map_words(n)) == hipSuccess &&
             dalloc(&e->cpm, gs::node_map_words(n)) == hipSuccess &&
             dalloc(&e->rows_dev, 2) == hipSuccess &&
             dalloc(&e->acct, 1) == hipSuccess && hipMemsetAsync(e->acct, 0, sizeof(u64), e->stream) == hipSuccess;
    if (ok && e->seq)
        ok = dalloc(&e->Wb, (size_t)n * 2 * g.W) == hipSuccess && dalloc(&e->sinfo, n) == hipSuccess &&
             dalloc(&e->seqw, (size_t)gs::seq_blocks(n) * gs::kSeqLists + gs::kSeqLists + n) == hipSuccess;
    if (ok && e->faults.churn)
        ok = dalloc(&e->pend, (size_t)n * 2 * g.W) == hipSuccess && dalloc(&e->offc, n) == hipSuccess;
    if (!ok) {
        hipError_t le = hipGetLastError();
        release(e);
        return le == hipErrorOutOfMemory ? GS_ERR_OUT_OF_MEMORY : GS_ERR_HIP;
    }
    // (the zeroing above and reset_state's run on the engine stream: a plain
    // hipMemset goes to the null stream, which non-blocking streams do not
    // wait for; every buffer is zero once this synchronisation returns)
    if (reset_state(e) != GS_OK || hipStreamSynchronize(e->stream) != hipSuccess) {
        release(e);
        return GS_ERR_HIP;
    }
    *out = e;
    return GS_OK;
}

// Plan of round r on the side stream: owned targets and send slots (set
// r % 3), and the ids exchange A of round r-1 carries (buffer set (r-1) % 2);
// code rows carry no ids: the plan marks the empty row slots of round r's own
// buffer set (r % 2) instead.
gs_status launch_plan(gs_engine *e, uint32_t r) {
    GS_HIP(gs::launch_shard_plan(e->sp, e->spl, e->planw[r % 3], e->sendA[(e->dlv ? r : r + 1) % 2], e->seed,
                                 e->epoch, r, e->faults, e->flags, e->cstream));
    GS_HIP(hipEventRecord(e->ev_plan[r % 3], e->cstream));
    return GS_OK;
}

// In-lists of round r from the ids received by exchange A of round r-1
// (buffer set (r-1) % 2), on the side stream.
gs_status launch_edges(gs_engine *e, uint32_t r) {
    GS_HIP(gs::launch_shard_edges(e->sp, e->sel, e->edgew[r % 2], e->recvA[(r + 1) % 2],
                                  e->planw[r % 3] + e->spl.tg, e->seed, e->epoch, r, e->faults, e->flags,
                                  e->cstream));
    GS_HIP(hipEventRecord(e->ev_edges[r % 2], e->cstream));
    return GS_OK;
}

// Code-row shard, after exchange A of round t: the plan of round t+2 on the
// side stream (its ids are not exchanged: code rows carry their targets),
// then on the engine stream the delivery-record build of round t over the
// arrived rows (gs_inlist.hip, sources = slot keys): every owned node's
// record and each pusher's pull code into sendB at its exchange-B slot.
gs_status shard_build(gs_engine *e) {
    const uint32_t t = e->round;
    GS_HIP(hipEventRecord(e->ev_main, e->stream));
    GS_HIP(hipStreamWaitEvent(e->cstream, e->ev_main, 0));
    gs_status st = launch_plan(e, t + 2);
    if (st != GS_OK) return st;
    e->pulled_round = t;
    auto &c = e->csr[0];
    gs::InListArgs la{};
    la.p = e->plan;
    la.dlv = 1;
    la.S = e->S[e->cur];
    la.g = e->g;
    la.DR = c.DR;
    la.dtail = c.src;
    la.src = c.src;
    la.region = c.region;
    la.scratch = c.scratch;
    la.flags = e->flags;
    la.seed = e->seed;
    la.epoch = e->epoch;
    la.round = t;
    la.f = e->faults;
    la.rowsA = reinterpret_cast<const uint32_t *>(e->recvA[t % 2]);
    la.pullB = reinterpret_cast<uint32_t *>(e->sendB);
    la.sr = gs::ShardRows{e->sp.G,  e->sp.P,   e->sp.W,     e->sp.capP,  e->sp.idrows,
                          e->sp.rw, e->sp.rwb, e->sp.codes, e->sp.chunk, e->sp.n};
    la.nkeys = shard_keys(e->sp);
    la.ntargets = e->g.n;
    // this rank's own block: written in place by the round kernel, counted by
    // round t's plan, answered in place in exchange B's receive buffer
    la.self_rank = e->sp.g;
    la.self_cnt = e->planw[t % 3] + e->spl.cnt + (size_t)e->sp.g * e->sp.P;
    la.pullB_self = reinterpret_cast<uint32_t *>(e->recvB);
    GS_HIP(gs::launch_build_inlists(la, e->stream));
    return GS_OK;
}

}  // namespace

extern "C" {

gs_status gs_create(const gs_config *cfg, gs_engine **out) { return create_engine(cfg, 0, 0, 0, out); }

gs_status gs_shard_create(const gs_config *cfg, uint32_t rank, uint32_t world, gs_engine **out) {
    if (world == 0) return GS_ERR_INVALID_ARGUMENT;
    return create_engine(cfg, rank, world, 1, out);
}

gs_status gs_shard_create_parts(const gs_config *cfg, uint32_t rank, uint32_t world, uint32_t parts,
                                gs_engine **out) {
    if (world == 0) return GS_ERR_INVALID_ARGUMENT;
    return create_engine(cfg, rank, world, parts, out);
}

gs_status gs_shard_info(const gs_engine *e, uint32_t info[14]) {
    if (!e || !info || !e->shard) return GS_ERR_INVALID_ARGUMENT;
    fill_shard_info(e->sp, info);
    return GS_OK;
}

gs_status gs_shard_plan_info(const gs_config *cfg, uint32_t rank, uint32_t world, uint32_t parts, uint32_t info[14]) {
    if (!cfg || !info || world == 0) return GS_ERR_INVALID_ARGUMENT;
    gs::ShardPlan sp{};
    uint8_t p[3];
    const gs_status st = check_config(cfg, rank, world, parts, &sp, p);  // (as gs_shard_create_parts)
    if (st != GS_OK) return st;
    fill_shard_info(sp, info);
    return GS_OK;
}

gs_status gs_shard_bind(gs_engine *e, void *sendA0, void *sendA1, void *recvA0, void *recvA1, void *sendB,
                        void *recvB) {
    if (!e || !e->shard || !sendA0 || !sendA1 || !recvA0 || !recvA1 || !sendB || !recvB)
        return GS_ERR_INVALID_ARGUMENT;
    e->sendA[0] = (u64 *)sendA0;
    e->sendA[1] = (u64 *)sendA1;
    e->recvA[0] = (u64 *)recvA0;
    e->recvA[1] = (u64 *)recvA1;
    e->sendB = (u64 *)sendB;
    e->recvB = (u64 *)recvB;
    return GS_OK;
}

gs_status gs_shard_pull(gs_engine *e) {
    if (!e || !e->shard || e->round == 0 || !e->recvB) return GS_ERR_INVALID_ARGUMENT;
    gs_status st = set_device(e);
    if (st != GS_OK) return st;
    const uint32_t t = e->round;
    if (e->dlv) return shard_build(e);
    // Exchange A of round t (and, in round 1, the ids-only exchange A of
    // round 0) is complete on the engine stream: build the in-lists of round
    // t+1 (and of round 1) on the side stream, behind this round's work.
    GS_HIP(hipEventRecord(e->ev_main, e->stream));
    GS_HIP(hipStreamWaitEvent(e->cstream, e->ev_main, 0));
    if (t == 1) {
        st = launch_edges(e, 1);
        if (st != GS_OK) return st;
    }
    GS_HIP(hipStreamWaitEvent(e->stream, e->ev_edges[t % 2], 0));
    st = launch_edges(e, t + 1);
    if (st != GS_OK) return st;
    // Plan of round t+2 into set (t+2)%3 (last read by the round kernel of
    // round t-1) and its ids into exchange-A buffer (t+1)%2 (last sent by
    // exchange A of round t-1): it has this round's pull rows, exchange B and
    // round kernel to finish before exchange A of round t+1 needs it.
    st = launch_plan(e, t + 2);
    if (st != GS_OK) return st;
    e->pulled_round = t;
    uint32_t *ed = e->edgew[t % 2];
    gs::PullArgs a{};
    a.S = e->S[e->cur];
    a.IN = reinterpret_cast<const uint4 *>(ed + e->sel.IN);
    a.IN2 = ed + e->sel.IN2;
    a.EP = ed + e->sel.EP;
    a.recvA = e->recvA[t % 2];
    a.sendB = e->sendB;
    a.P = e->sp;
    a.g = e->g;
    GS_HIP(gs::launch_pull(a, e->stream));
    return GS_OK;
}

uint64_t gs_stream(const gs_engine *e) { return e ? (uint64_t)(uintptr_t)e->stream : 0; }

int gs_device(const gs_engine *e) { return e ? e->device : 0; }

void gs_destroy(gs_engine *e) { release(e); }

gs_status gs_get_params(const gs_engine *e, uint8_t out[3]) {
    if (!e || !out) return GS_ERR_INVALID_ARGUMENT;
    out[0] = e->cmax;
    out[1] = e->maxc;
    out[2] = e->maxr;
    return GS_OK;
}

uint32_t gs_round(const gs_engine *e) { return e ? e->round : 0; }

gs_status gs_send_new(gs_engine *e, uint32_t node, uint32_t rumor) {
    if (!e) return GS_ERR_INVALID_ARGUMENT;
    if ((e->shard ? e->n_global : e->g.n) < 2) return GS_ERR_NO_PEERS;  // src/gossiper.rs:56-58
    if (e->shard) {  // global node id; must be owned by this rank
        if (node < e->sp.lo || node - e->sp.lo >= e->sp.m) return GS_ERR_INVALID_ARGUMENT;
        node -= e->sp.lo;
    }
    if (node >= e->g.n || rumor >= e->g.R) return GS_ERR_INVALID_ARGUMENT;
    e->pending.emplace_back(node, rumor);
    e->obs_valid = false;
    e->started = true;
    return GS_OK;
}

gs_status gs_set_params(gs_engine *e, const uint8_t params[3]) {
    if (!e || !params) return GS_ERR_INVALID_ARGUMENT;
    // Gossiper::add_peer (src/gossiper.rs:45-52): the parameters may only
    // change before any message exists.
    if (e->started) return GS_ERR_ALREADY_STARTED;
    uint8_t p[3];
    gs_derive_params(e->shard ? e->n_global : e->g.n, p);
    for (int i = 0; i < 3; ++i)
        if (params[i]) p[i] = params[i];
    if ((e->shard ? e->n_global : e->g.n) >= 2 && (p[0] > 3 || p[1] > 3 || p[2] > 32 || !p[0] || !p[1] || !p[2]))
        return GS_ERR_UNSUPPORTED;
    e->cmax = p[0];
    e->maxc = p[1];
    e->maxr = p[2];
    e->obs_valid = false;
    return GS_OK;
}

}  // extern "C"

namespace {

// ------------------------------------------------------------ round
// A round is launched as one or more pipeline parts (shard engines: the
// node-range parts of gs_shard_create_parts; otherwise one part = the whole
// grid): round_begin sequences the round and fixes its arguments, launch_part
// launches one part's blocks, round_end does the bookkeeping after the last.
// A new build serial for in-list set c (SibRecs of older builds read as
// stale).  When the 24-bit serial wraps, every set's SibRecs are cleared at
// that set's next build, on the build stream, after its last reader.
gs_status next_serial(gs_engine *e, gs_engine::CsrSet &c, hipStream_t bs) {
    c.serial = ++e->build_serial & gs::kSerialMask;
    if (c.serial == 0) {
        ++e->serial_wraps;
        c.serial = ++e->build_serial & gs::kSerialMask;
    }
    if (c.wraps != e->serial_wraps) {
        if (c.SIB8) GS_HIP(hipMemsetAsync(c.SIB8, 0, (size_t)e->g.n * sizeof(gs::SibRec), bs));
        c.wraps = e->serial_wraps;
    }
    return GS_OK;
}

// Arguments of the build of round `round`'s in-lists into set c.
gs::InListArgs inlist_args(gs_engine *e, gs_engine::CsrSet &c, uint32_t round) {
    gs::InListArgs la{};
    la.p = e->plan;
    la.tg = c.tg;
    la.IN8 = c.IN8;
    la.SIB8 = c.SIB8;
    la.src = c.src;
    la.region = c.region;
    la.scratch = c.scratch;
    la.flags = e->flags;
    la.serial = c.serial;
    la.seed = e->seed;
    la.epoch = e->epoch;
    la.round = round;
    la.f = e->faults;
    if (e->filt) {  // skip flags from the maps the round kernel just wrote
        la.lvm = e->lvm;
        la.cpm = e->cpm;
        la.zl = c.zl;
        la.rows = e->rows_dev + (round & 1u);
    }
    if (e->dlv) {  // records carry the push codes of the new round's planes
        la.dlv = 1;
        la.S = e->S[e->cur];
        la.PC = e->pc;
        la.KN = e->kn;
        la.g = e->g;
        la.DR = c.DR;
        la.dtail = c.src;
        la.pull = c.pull;
    }
    return la;
}

gs_status round_begin(gs_engine *e) {
    gs_status st = GS_OK;
    if (e->shard) {
        // cstream work launched below may reuse buffers read before this point
        GS_HIP(hipEventRecord(e->ev_main, e->stream));
        GS_HIP(hipStreamWaitEvent(e->cstream, e->ev_main, 0));
        if (e->round == 0) {
            st = launch_plan(e, 1);  // send slots of round 1's push rows, ids for exchange A(0)
            if (st != GS_OK) return st;
        }
    }
    uint32_t n_inj = 0;
    st = upload_injections(e, &n_inj);
    if (st == GS_OK && e->deliver_pending) st = upload_ext(e);
    if (st != GS_OK) return st;
    gs::RoundArgs a = base_args(e);
    a.inj_key = e->inj_key;
    a.inj_mask = e->inj_mask;
    a.n_inj = n_inj;
    const uint32_t R0 = e->round;
    if (e->slice) {
        a.emin = e->eb[(R0 + 1u) % 3u];  // round R0+1's buffer
        if (e->eb_defer >= 0) a.eadd = e->eb[e->eb_defer];
        e->eb_defer = -1;
    }
    if (e->filt && e->deliver_pending && e->timing) {  // rows gathered, for gs_round_traffic
        a.acct = e->acct;
        a.rows_cnt = e->rows_dev + (R0 & 1u);  // counted by the build of round t's lists
        e->filt_launches++;
    }
    if (e->shard) {
        GS_HIP(hipStreamWaitEvent(e->stream, e->ev_plan[(R0 + 1) % 3], 0));
        if (e->deliver_pending && !e->dlv) GS_HIP(hipStreamWaitEvent(e->stream, e->ev_edges[R0 % 2], 0));
    } else if (e->deliver_pending) {
        st = seq_prepare(e);  // SEQ: pull batches of round t (no-op for 2P)
        if (st != GS_OK) return st;
    }
    // the build of round t+1 runs right behind this kernel on its stream: the
    // kernel clears that build's counters (no memset launch)
    e->ra_prezeroed = !e->shard;
    if (e->ra_prezeroed) {
        auto &c = e->csr[(R0 + 1u) & 1u];
        size_t first = 0, words = 0;
        gs::inlist_zero_range(e->plan, &first, &words);
        if (words) {
            a.zero_buf = c.scratch + first;
            a.zero_words = (uint32_t)words;
        }
        if (e->filt) a.zero_rows = e->rows_dev + ((R0 + 1u) & 1u);
        // DLV: the coarse fills of the set round t's build used (consumed by
        // its dl_fine) are cleared now, a round before that set is
        // partitioned into again; the next set's were cleared a round ago, so
        // this launch may reserve in them
        gs::inlist_cfill_range(e->plan, &first, &words);
        if (words) {
            a.zero_buf2 = e->csr[R0 & 1u].scratch + first;
            a.zero_words2 = (uint32_t)words;
        }
    }
    e->ra = a;
    e->ra_mode = e->deliver_pending ? 1 : 0;
    e->tslot = ~0u;
    if (e->timing && e->tcount < kTimingSlots) {
        e->tslot = e->tcount++;
        e->tparts[e->tslot] = 0;
    }
    return GS_OK;
}

// Nodes per lane of the packed DLV round kernel (gs_dlv4.hip launch_round_dlv4).
uint32_t dlv_nodes_per_lane(const gs_engine *e) {
    if (e->dlv_pack == 3) return 1u;
    if (e->g.rpad < 16) return 4u;
    return e->dlv_pack == 2 ? 4u : 2u;
}

gs_status launch_part(gs_engine *e, uint32_t h) {
    gs::RoundArgs a = e->ra;
    if (e->shard && e->sp.P > 1) {  // blocks of part h (blk_count 0 would mean the whole grid)
        // (code rows: the packed DLV kernel's blocks of 256 lanes of npl
        // nodes; parts are whole 1024-node blocks, gs_shard.hip shard_plan)
        const u64 bn = e->dlv ? 256ull * dlv_nodes_per_lane(e) : 256ull;
        const u64 nblk = e->dlv ? ((u64)e->g.n + bn - 1) / bn : (e->g.nseg + 255) / 256;
        const u64 per = e->dlv ? (u64)e->sp.mP / bn : e->g.small ? (u64)e->sp.bP : (u64)e->sp.mP * e->g.W / 256;
        const u64 b0 = std::min<u64>((u64)h * per, nblk), b1 = std::min<u64>(b0 + per, nblk);
        if (b1 == b0) return GS_OK;
        a.blk_off = (uint32_t)b0;
        a.blk_count = (uint32_t)(b1 - b0);
    }
    hipEvent_t t0 = nullptr, t1 = nullptr;
    if (e->timing && e->tslot != ~0u) {
        t0 = e->tev[2 * ((size_t)e->tslot * gs::kMaxParts + h)];
        t1 = e->tev[2 * ((size_t)e->tslot * gs::kMaxParts + h) + 1];
        if (!e->tparts[e->tslot]) e->lt0 = t0;  // first timed part
        e->tparts[e->tslot] |= (uint8_t)(1u << h);
        e->lt1 = t1;
    }
    if (t0) GS_HIP(hipEventRecord(t0, e->stream));
    GS_HIP(gs::launch_round(a, e->ra_mode, e->stream));
    if (t1) GS_HIP(hipEventRecord(t1, e->stream));
    return GS_OK;
}

gs_status round_end(gs_engine *e, gs_round_report *report) {
    gs_status st = GS_OK;
    const uint32_t R0 = e->round;
    e->timed = e->timing;
    e->round += 1;
    e->cur ^= 1;
    e->deliver_pending = true;
    e->ext.clear();  // delivered by this round kernel (upload_ext syncs before reuse)
    e->ext_peers.clear();
    e->ext_fp.clear();
    e->ext_uploaded = 0;
    e->obs_valid = false;
    if (++e->since_fold >= e->fold_every) {
        GS_HIP(gs::launch_stats_fold(e->st32, e->st64, e->g.n, e->st16 ? 1u : 0u, e->stream));
        e->since_fold = 0;
    }
    if (e->shard) {
        // Exchange A of round t+1 (next on the engine stream) carries the ids
        // of the plan of round t+2, launched by gs_shard_pull (or, for round
        // 2, here); the in-lists of round t+1 are built by then.
        if (R0 == 0) {
            st = launch_plan(e, 2);
            if (st != GS_OK) return st;
        }
        GS_HIP(hipStreamWaitEvent(e->stream, e->ev_plan[(R0 + 2) % 3], 0));
    } else {
        // Lists of the new round t+1 into the other set, whose last reader
        // was the round kernel before this one.  Built on the round stream
        // right after the round kernel: both are HBM-bound, and the in-list
        // kernels hold whole CUs (1024 threads, >100 KiB LDS), so running them
        // beside the round kernel measured slower than in sequence (DESIGN.md
        // section 4); the DLV and filtered builds also read what this round
        // kernel writes (push codes, node maps).
        auto &c = e->csr[e->round & 1u];
        st = next_serial(e, c, e->stream);
        if (st != GS_OK) return st;
        gs::InListArgs la = inlist_args(e, c, e->round);
        la.prezeroed = e->ra_prezeroed ? 1u : 0u;
        GS_HIP(gs::launch_build_inlists(la, e->stream));
    }
    if (report) {
        uint32_t fl[4];
        static thread_local uint32_t lw[gs::kLiveSlots * gs::kLiveStride];
        GS_HIP(hipMemcpyAsync(fl, e->flags, sizeof(fl), hipMemcpyDeviceToHost, e->stream));
        GS_HIP(hipMemcpyAsync(lw, e->live + (size_t)(e->round & 1u) * gs::kLiveSlots * gs::kLiveStride, sizeof(lw),
                              hipMemcpyDeviceToHost, e->stream));
        GS_HIP(hipStreamSynchronize(e->stream));
        report->round = e->round;
        uint32_t any = 0;
        for (uint32_t i = 0; i < gs::kLiveSlots; ++i) any |= lw[i * gs::kLiveStride];
        report->any_live = any;
        if (fl[2]) return GS_ERR_DEVICE_LIMIT;
    }
    return GS_OK;
}

gs_status round_checks(gs_engine *e) {
    if ((e->shard ? e->n_global : e->g.n) < 2) return GS_ERR_NO_PEERS;  // src/gossiper.rs:71-74
    if (e->shard && !e->sendB) return GS_ERR_INVALID_ARGUMENT;  // gs_shard_bind first
    if (e->slice && !e->eb[0]) return GS_ERR_INVALID_ARGUMENT;  // gs_slice_bind first
    // a shard delivers round t only after its exchanges (gs_shard_pull)
    if (e->shard && e->round > 0 && e->pulled_round != e->round) return GS_ERR_INVALID_ARGUMENT;
    return set_device(e);
}

}  // namespace

extern "C" {

gs_status gs_shard_round_part(gs_engine *e, uint32_t part) {
    if (!e || !e->shard || part != e->parts_done || part >= e->sp.P) return GS_ERR_INVALID_ARGUMENT;
    gs_status st = round_checks(e);
    if (st == GS_OK && part == 0) st = round_begin(e);
    if (st == GS_OK) st = launch_part(e, part);
    if (st != GS_OK) {
        e->parts_done = 0;
        return st;
    }
    e->parts_done = part + 1;
    return GS_OK;
}

gs_status gs_next_round(gs_engine *e, gs_round_report *report) {
    if (!e) return GS_ERR_INVALID_ARGUMENT;
    gs_status st = round_checks(e);
    if (st == GS_OK && e->parts_done == 0) st = round_begin(e);
    const uint32_t parts = e->shard ? e->sp.P : 1u;
    for (uint32_t h = e->parts_done; st == GS_OK && h < parts; ++h) st = launch_part(e, h);
    e->parts_done = 0;
    if (st != GS_OK) return st;
    return round_end(e, report);
}

gs_status gs_slice_bind(gs_engine *e, void *buf0, void *buf1, void *buf2, void *obs) {
    if (!e || !e->slice || !buf0 || !buf1 || !buf2 || !obs) return GS_ERR_INVALID_ARGUMENT;
    e->eb[0] = static_cast<uint8_t *>(buf0);
    e->eb[1] = static_cast<uint8_t *>(buf1);
    e->eb[2] = static_cast<uint8_t *>(buf2);
    e->eb[3] = static_cast<uint8_t *>(obs);
    return GS_OK;
}

gs_status gs_slice_defer(gs_engine *e, uint32_t which) {
    if (!e || !e->slice || which > 2 || !e->eb[which]) return GS_ERR_INVALID_ARGUMENT;
    if (e->eb_defer == (int)which) return GS_ERR_INVALID_ARGUMENT;  // would be added twice
    gs_status st = set_device(e);
    if (st != GS_OK) return st;
    if (e->eb_defer >= 0)  // one deferred buffer at a time: add the older one now
        GS_HIP(gs::launch_slice_apply(e->st32, e->eb[e->eb_defer], e->g.n, e->st16 ? 1u : 0u, e->stream));
    e->eb_defer = (int)which;
    e->obs_valid = false;
    return GS_OK;
}

gs_status gs_slice_apply(gs_engine *e, uint32_t which) {
    if (!e || !e->slice || which > 2) return GS_ERR_INVALID_ARGUMENT;
    gs_status st = set_device(e);
    if (st != GS_OK) return st;
    if (!e->eb[which]) return GS_ERR_INVALID_ARGUMENT;
    if (e->eb_defer == (int)which) e->eb_defer = -1;  // deferred: added now instead, once
    GS_HIP(gs::launch_slice_apply(e->st32, e->eb[which], e->g.n, e->st16 ? 1u : 0u, e->stream));
    e->obs_valid = false;
    return GS_OK;
}

gs_status gs_statistics_all(gs_engine *e, uint64_t *out) {
    if (!e || !out) return GS_ERR_INVALID_ARGUMENT;
    gs_status st = set_device(e);
    if (st == GS_OK) st = observe(e, false);
    if (st != GS_OK) return st;
    GS_HIP(hipMemcpy(out, e->obs_stats, (size_t)e->g.n * 5 * sizeof(u64), hipMemcpyDeviceToHost));
    return GS_OK;
}

gs_status gs_statistics(gs_engine *e, uint32_t node, gs_statistics_t *out) {
    if (!e || !out || node >= e->g.n) return GS_ERR_INVALID_ARGUMENT;
    gs_status st = set_device(e);
    if (st == GS_OK) st = observe(e, false);
    if (st != GS_OK) return st;
    u64 v[5];
    GS_HIP(hipMemcpy(v, e->obs_stats + (size_t)node * 5, sizeof(v), hipMemcpyDeviceToHost));
    out->rounds = v[0];
    out->empty_pull_sent = v[1];
    out->empty_push_sent = v[2];
    out->full_message_sent = v[3];
    out->full_message_received = v[4];
    return GS_OK;
}

gs_status gs_statistics_reduce(gs_engine *e, gs_reduce_op op, gs_statistics_t *out) {
    if (!e || !out || (int)op < 0 || (int)op > 2) return GS_ERR_INVALID_ARGUMENT;
    gs_status st = set_device(e);
    if (st == GS_OK) st = observe(e, false);
    if (st != GS_OK) return st;
    GS_HIP(gs::launch_stats_reduce(e->obs_stats, e->g.n, (int)op, e->partials, kReduceBlocks, e->stream));
    std::vector<u64> part((size_t)kReduceBlocks * 5);
    GS_HIP(hipMemcpyAsync(part.data(), e->partials, part.size() * sizeof(u64), hipMemcpyDeviceToHost,
                          e->stream));
    GS_HIP(hipStreamSynchronize(e->stream));
    u64 acc[5];
    for (int f = 0; f < 5; ++f) acc[f] = op == GS_REDUCE_MIN ? ~0ull : 0ull;
    for (uint32_t b = 0; b < kReduceBlocks; ++b)
        for (int f = 0; f < 5; ++f) {
            const u64 v = part[(size_t)b * 5 + f];
            acc[f] = op == GS_REDUCE_SUM ? acc[f] + v : (op == GS_REDUCE_MIN ? std::min(acc[f], v) : std::max(acc[f], v));
        }
    out->rounds = acc[0];
    out->empty_pull_sent = acc[1];
    out->empty_push_sent = acc[2];
    out->full_message_sent = acc[3];
    out->full_message_received = acc[4];
    return GS_OK;
}

gs_status gs_messages(gs_engine *e, uint32_t node, uint64_t *words) {
    if (!e || !words || node >= e->g.n) return GS_ERR_INVALID_ARGUMENT;
    gs_status st = set_device(e);
    if (st == GS_OK) st = observe(e, false);
    if (st != GS_OK) return st;
    const uint32_t KW = (e->g.R + 63) / 64;
    GS_HIP(hipMemcpy(words, e->obs_known + (size_t)node * KW, KW * sizeof(u64), hipMemcpyDeviceToHost));
    return GS_OK;
}

gs_status gs_known_all(gs_engine *e, uint64_t *words) {
    if (!e || !words) return GS_ERR_INVALID_ARGUMENT;
    gs_status st = set_device(e);
    if (st == GS_OK) st = observe(e, false);
    if (st != GS_OK) return st;
    const uint32_t KW = (e->g.R + 63) / 64;
    GS_HIP(hipMemcpy(words, e->obs_known, (size_t)e->g.n * KW * sizeof(u64), hipMemcpyDeviceToHost));
    return GS_OK;
}

gs_status gs_known_counts(gs_engine *e, uint64_t *known_total, uint64_t *nodes_complete) {
    return gs_known_counts_min(e, e ? e->g.R : 0, known_total, nodes_complete);
}

gs_status gs_known_counts_min(gs_engine *e, uint32_t min_known, uint64_t *known_total,
                              uint64_t *nodes_complete) {
    if (!e) return GS_ERR_INVALID_ARGUMENT;
    gs_status st = set_device(e);
    if (st == GS_OK) st = observe(e, false);
    if (st != GS_OK) return st;
    const uint32_t KW = (e->g.R + 63) / 64;
    GS_HIP(gs::launch_known_reduce(e->obs_known, e->g.n, KW, min_known, e->partials, kReduceBlocks / 2,
                                   e->stream));
    std::vector<u64> part(kReduceBlocks);
    GS_HIP(hipMemcpyAsync(part.data(), e->partials, part.size() * sizeof(u64), hipMemcpyDeviceToHost,
                          e->stream));
    GS_HIP(hipStreamSynchronize(e->stream));
    u64 t = 0, c = 0;
    for (uint32_t b = 0; b < kReduceBlocks / 2; ++b) {
        t += part[2 * b];
        c += part[2 * b + 1];
    }
    if (known_total) *known_total = t;
    if (nodes_complete) *nodes_complete = c;
    return GS_OK;
}

gs_status gs_known_popcounts(gs_engine *e, uint32_t *counts) {
    if (!e || !counts) return GS_ERR_INVALID_ARGUMENT;
    gs_status st = set_device(e);
    if (st == GS_OK) st = observe(e, false);
    if (st != GS_OK) return st;
    const uint32_t KW = (e->g.R + 63) / 64;
    // obs_psize is free scratch here ([n] u32; rewritten by the next observe)
    GS_HIP(gs::launch_known_popc(e->obs_known, e->g.n, KW, e->obs_psize, e->stream));
    GS_HIP(hipMemcpyAsync(counts, e->obs_psize, (size_t)e->g.n * sizeof(uint32_t), hipMemcpyDeviceToHost,
                          e->stream));
    GS_HIP(hipStreamSynchronize(e->stream));
    e->obs_valid = false;  // obs_psize overwritten
    return GS_OK;
}

gs_status gs_dump_state(gs_engine *e, uint16_t *out) {
    if (!e || !out) return GS_ERR_INVALID_ARGUMENT;
    gs_status st = set_device(e);
    if (st == GS_OK) st = observe(e, true);
    if (st != GS_OK) return st;
    GS_HIP(hipMemcpy(out, e->obs_state, (size_t)e->g.n * e->g.R * sizeof(uint16_t), hipMemcpyDeviceToHost));
    return GS_OK;
}

gs_status gs_state_digest(gs_engine *e, uint64_t *out) {
    if (!e || !out) return GS_ERR_INVALID_ARGUMENT;
    if (!e->pending.empty()) return GS_ERR_INVALID_ARGUMENT;  // queued send_new: observe before injecting
    gs_status st = set_device(e);
    if (st == GS_OK) st = observe(e, false, true);
    if (st != GS_OK) return st;
    GS_HIP(hipMemcpy(out, e->obs_digest, (size_t)e->g.n * sizeof(u64), hipMemcpyDeviceToHost));
    return GS_OK;
}

gs_status gs_state_digest_part(gs_engine *e, uint32_t rumor_lo, uint32_t words, uint64_t *dpart) {
    if (!e || !dpart || words == 0 || (uint64_t)rumor_lo + e->g.R > 64ull * words) return GS_ERR_INVALID_ARGUMENT;
    if (!e->pending.empty()) return GS_ERR_INVALID_ARGUMENT;  // queued send_new: observe before injecting
    gs_status st = set_device(e);
    if (st == GS_OK) st = observe(e, false, false, reinterpret_cast<u64 *>(dpart), rumor_lo, words);
    if (st != GS_OK) return st;
    GS_HIP(hipStreamSynchronize(e->stream));
    return GS_OK;
}

gs_status gs_digest_finish(gs_engine *e, const uint64_t *dpart, uint32_t words, const uint64_t *stats,
                           uint64_t *out) {
    if (!e || !dpart || !stats || !out || words == 0) return GS_ERR_INVALID_ARGUMENT;
    if (!e->obs_psize) return GS_ERR_INVALID_ARGUMENT;  // gs_state_digest_part first
    gs_status st = set_device(e);
    if (st != GS_OK) return st;
    if (!e->obs_digest) GS_HIP(dalloc(&e->obs_digest, e->g.n));
    // the Statistics rows go through obs_stats (rewritten by the next observation)
    GS_HIP(hipMemcpyAsync(e->obs_stats, stats, (size_t)e->g.n * 5 * sizeof(u64), hipMemcpyHostToDevice, e->stream));
    GS_HIP(gs::launch_digest_finish(reinterpret_cast<const u64 *>(dpart), e->g.n, words, e->obs_psize, e->obs_stats,
                                    e->obs_digest, e->stream));
    GS_HIP(hipMemcpyAsync(out, e->obs_digest, (size_t)e->g.n * sizeof(u64), hipMemcpyDeviceToHost, e->stream));
    GS_HIP(hipStreamSynchronize(e->stream));
    e->obs_valid = false;  // obs_stats overwritten
    return GS_OK;
}

gs_status gs_dump_records(gs_engine *e, uint16_t *rec, uint32_t *psize) {
    if (!e || !rec) return GS_ERR_INVALID_ARGUMENT;
    gs_status st = set_device(e);
    if (st == GS_OK) st = observe(e, true);
    if (st != GS_OK) return st;
    GS_HIP(hipMemcpy(rec, e->obs_rec, (size_t)e->g.n * e->g.R * sizeof(uint16_t), hipMemcpyDeviceToHost));
    if (psize)
        GS_HIP(hipMemcpy(psize, e->obs_psize, (size_t)e->g.n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return GS_OK;
}

gs_status gs_clear(gs_engine *e, uint32_t epoch) {
    if (!e) return GS_ERR_INVALID_ARGUMENT;
    gs_status st = set_device(e);
    if (st != GS_OK) return st;
    // A device limit hit since the last clear is reported here rather than
    // dropped with the flags (gs_next_round(e, NULL) never reads them).
    const gs_status lim = device_limit(e);
    if (lim != GS_OK && lim != GS_ERR_DEVICE_LIMIT) return lim;
    e->epoch = epoch;
    st = reset_state(e);
    if (st != GS_OK) return st;
    GS_HIP(hipStreamSynchronize(e->stream));
    return lim;
}

gs_status gs_sync(gs_engine *e) {
    if (!e) return GS_ERR_INVALID_ARGUMENT;
    gs_status st = set_device(e);
    if (st != GS_OK) return st;
    GS_HIP(hipStreamSynchronize(e->stream));
    GS_HIP(hipStreamSynchronize(e->cstream));
    return device_limit(e);
}

void gs_set_timing(gs_engine *e, int enable) {
    if (!e) return;
    e->timing = enable != 0;
    if (e->timing && e->tev.empty()) {
        (void)hipSetDevice(e->device);
        e->tev.resize(2 * (size_t)kTimingSlots * gs::kMaxParts, nullptr);
        e->tparts.assign(kTimingSlots, 0);
        // timing only: no system-scope fence (an L2 write-back and invalidate
        // at every record) around the kernel being timed
        for (auto &ev : e->tev)
            if (hipEventCreateWithFlags(&ev, hipEventDisableSystemFence) != hipSuccess) {
                e->timing = false;
                return;
            }
    }
    e->tcount = 0;
    if (e->timing && e->filt) {  // restart the traffic accounting with the ring
        (void)hipSetDevice(e->device);
        if (hipMemsetAsync(e->acct, 0, sizeof(u64), e->stream) == hipSuccess) e->filt_launches = 0;
    }
}

int32_t gs_round_kernel_times(gs_engine *e, float *out_ms, uint32_t max) {
    if (!e || !out_ms) return -1;
    if (hipStreamSynchronize(e->stream) != hipSuccess) return -1;
    const uint32_t m = std::min(max, e->tcount);
    for (uint32_t i = 0; i < m; ++i) {
        float sum = 0.0f;
        for (uint32_t h = 0; h < gs::kMaxParts; ++h) {
            if (!(e->tparts[i] & (1u << h))) continue;
            const size_t k = 2 * ((size_t)i * gs::kMaxParts + h);
            float ms = -1.0f;
            if (hipEventElapsedTime(&ms, e->tev[k], e->tev[k + 1]) != hipSuccess) return -1;
            sum += ms;
        }
        out_ms[i] = sum;
    }
    e->tcount = 0;
    return (int32_t)m;
}

float gs_last_round_kernel_ms(gs_engine *e) {
    if (!e || !e->timed || !e->lt0 || !e->lt1) return -1.0f;
    if (hipEventSynchronize(e->lt1) != hipSuccess) return -1.0f;
    float ms = -1.0f;
    if (hipEventElapsedTime(&ms, e->lt0, e->lt1) != hipSuccess) return -1.0f;
    return ms;
}

// ------------------------------------------------------------ wire format
gs_status gs_set_rumor_key(gs_engine *e, uint32_t rumor, const uint8_t *key, uint32_t len) {
    if (!e || (len && !key) || rumor >= e->g.R) return GS_ERR_INVALID_ARGUMENT;
    const std::string k(reinterpret_cast<const char *>(key), len);
    auto it = e->key_rumor.find(k);
    if (it != e->key_rumor.end()) return it->second == rumor ? GS_OK : GS_ERR_INVALID_ARGUMENT;
    e->key_rumor.erase(e->keys[rumor]);
    e->keys[rumor] = k;
    e->key_rumor[k] = rumor;
    std::sort(e->key_order.begin(), e->key_order.end(),
              [e](uint32_t x, uint32_t y) { return e->keys[x] < e->keys[y]; });  // BTreeMap<Vec<u8>> order
    return GS_OK;
}

gs_status gs_rumor_key(const gs_engine *e, uint32_t rumor, uint8_t *out, uint32_t cap, uint32_t *len) {
    if (!e || !len || rumor >= e->g.R) return GS_ERR_INVALID_ARGUMENT;
    const std::string &k = e->keys[rumor];
    *len = (uint32_t)k.size();
    if (!out || cap < k.size()) return GS_ERR_SERIALISATION;
    std::memcpy(out, k.data(), k.size());
    return GS_OK;
}

}  // extern "C"

namespace {

// Appends one length-prefixed frame (u32 LE size, then the bincode GossipRpc).
gs_status append_frame(int pull, const std::string &msg, uint8_t counter, uint8_t *out, uint32_t cap,
                       uint32_t *len) {
    uint32_t need = 0;
    gs_rpc_encode(pull, nullptr, 0, 0, nullptr, 0, &need);
    need += (uint32_t)msg.size();
    const uint32_t at = *len;
    *len += 4 + need;
    if (!out || *len > cap) return GS_ERR_SERIALISATION;  // keep counting the size needed
    for (int i = 0; i < 4; ++i) out[at + i] = (uint8_t)(need >> (8 * i));
    uint32_t w = 0;
    return gs_rpc_encode(pull, reinterpret_cast<const uint8_t *>(msg.data()), (uint32_t)msg.size(), counter,
                         out + at + 4, need, &w);
}

// External RPCs (gs_handle_received*) are accepted once a round has run and
// been delivered: a shard after gs_shard_pull, whose pull rows (exchange B)
// the caller has waited for.
gs_status ext_ready(const gs_engine *e) {
    if (e->round == 0 || !e->deliver_pending) return GS_ERR_INVALID_ARGUMENT;  // after a next_round
    if (e->shard && e->pulled_round != e->round) return GS_ERR_INVALID_ARGUMENT;
    return GS_OK;
}

// A node of this engine (shards: a global id owned by this rank) and a peer
// outside the simulated network.
bool ext_ids(const gs_engine *e, uint32_t node, uint32_t peer) {
    if (e->shard) return node >= e->sp.lo && node - e->sp.lo < e->sp.m && peer >= e->n_global;
    return node < e->g.n && peer >= e->g.n;
}

// Rumor slices: each slice counts an external first Push answered with an
// empty Pull into the node's per-round empty count, which the slices reduce
// as one byte (MIN) and the u16 Statistics deltas take between folds (sized
// for 32 * R_pad + 32 per round, the internal count being at most 30): at
// most this many first Pushes per node and round (GS_ERR_DEVICE_LIMIT).
// The bound must be the same on every slice of a network (a batch is refused
// on all of them or applied on all of them, and |peers_in_this_round| stays
// equal on every slice): the caller sets the network's, the smallest over its
// slices (gs_slice_set_ext_limit; SlicedNetwork does).
uint32_t slice_own_ext_limit(const gs_engine *e) { return std::min<uint32_t>(200u, 32u * e->g.rpad); }
uint32_t slice_ext_limit(const gs_engine *e) { return e->ext_limit ? e->ext_limit : slice_own_ext_limit(e); }

// Post-delivery state codes of one node (gs_dump_state's codes), external
// RPCs queued so far included: the observation kernel over the node's block.
gs_status observe_node(gs_engine *e, uint32_t node, std::vector<uint16_t> &codes) {
    gs_status st = upload_ext(e);
    if (st != GS_OK) return st;
    if (!e->node_state) GS_HIP(dalloc(&e->node_state, e->g.R));
    gs::RoundArgs a = base_args(e);
    a.obs_state = e->node_state;
    a.obs_only = node;
    const u64 seg0 = e->g.small ? (u64)node : (u64)node * e->g.W;
    a.blk_off = (uint32_t)(seg0 / 256);
    a.blk_count = 1;
    if (e->deliver_pending) {
        if (e->shard && !e->dlv) GS_HIP(hipStreamWaitEvent(e->stream, e->ev_edges[e->round % 2], 0));  // its in-lists
        st = seq_prepare(e);  // SEQ: the round's pull batches (no-op for 2P)
        if (st != GS_OK) return st;
    }
    GS_HIP(code_rows_obs(e, a));
    GS_HIP(gs::launch_round(a, e->deliver_pending ? 2 : 3, e->stream));
    codes.resize(e->g.R);
    GS_HIP(hipMemcpyAsync(codes.data(), e->node_state, e->g.R * sizeof(uint16_t), hipMemcpyDeviceToHost,
                          e->stream));
    GS_HIP(hipStreamSynchronize(e->stream));
    return GS_OK;
}

// Post-delivery state codes of several nodes at once (sorted, distinct): one
// observation launch over the blocks holding them, codes of nodes[j] at
// codes[j*R ..], external RPCs queued so far included.
gs_status observe_nodes(gs_engine *e, const std::vector<uint32_t> &nodes, std::vector<uint16_t> &codes) {
    const uint32_t m = (uint32_t)nodes.size();
    codes.assign((size_t)m * e->g.R, 0);
    if (!m) return GS_OK;
    gs_status st = upload_ext(e);
    if (st != GS_OK) return st;
    std::vector<uint32_t> blocks;
    for (uint32_t x : nodes) {
        const uint32_t b = (uint32_t)((e->g.small ? (u64)x : (u64)x * e->g.W) / 256);
        if (blocks.empty() || blocks.back() != b) blocks.push_back(b);
    }
    // grow-only scratch on the engine (engine stream order protects its reuse)
    const size_t lw = blocks.size() + m, cw = (size_t)m * e->g.R;
    if (lw > e->batch_lists_cap) {
        GS_HIP(hipStreamSynchronize(e->stream));
        if (e->batch_lists) (void)hipFree(e->batch_lists);
        e->batch_lists = nullptr;
        e->batch_lists_cap = 0;
        GS_HIP(dalloc(&e->batch_lists, 2 * lw));
        e->batch_lists_cap = 2 * lw;
    }
    if (cw > e->batch_codes_cap) {
        GS_HIP(hipStreamSynchronize(e->stream));
        if (e->batch_codes) (void)hipFree(e->batch_codes);
        e->batch_codes = nullptr;
        e->batch_codes_cap = 0;
        GS_HIP(dalloc(&e->batch_codes, 2 * cw));
        e->batch_codes_cap = 2 * cw;
    }
    uint32_t *dev = e->batch_lists;  // [blocks | nodes]
    uint16_t *dcodes = e->batch_codes;
    gs::RoundArgs a = base_args(e);
    a.obs_state = dcodes;
    a.blk_list = dev;
    a.blk_count = (uint32_t)blocks.size();
    a.obs_list = dev + blocks.size();
    a.n_obs = m;
    hipError_t he = hipMemcpyAsync(dev, blocks.data(), blocks.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                                   e->stream);
    if (he == hipSuccess)
        he = hipMemcpyAsync(dev + blocks.size(), nodes.data(), m * sizeof(uint32_t), hipMemcpyHostToDevice,
                            e->stream);
    if (he == hipSuccess && e->deliver_pending && e->shard && !e->dlv)  // a class-row shard's in-lists
        he = hipStreamWaitEvent(e->stream, e->ev_edges[e->round % 2], 0);
    if (he == hipSuccess && e->deliver_pending && seq_prepare(e) != GS_OK)
        he = hipErrorUnknown;  // SEQ: the round's pull batches
    if (he == hipSuccess) he = code_rows_obs(e, a);
    if (he == hipSuccess) he = gs::launch_round(a, e->deliver_pending ? 2 : 3, e->stream);
    if (he == hipSuccess)
        he = hipMemcpyAsync(codes.data(), dcodes, codes.size() * sizeof(uint16_t), hipMemcpyDeviceToHost, e->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream);  // (codes, blocks and nodes are host temporaries)
    return he == hipSuccess ? GS_OK : GS_ERR_HIP;
}

}  // namespace

extern "C" {

gs_status gs_slice_set_ext_limit(gs_engine *e, uint32_t limit) {
    if (!e || !e->slice || limit == 0 || limit > slice_own_ext_limit(e)) return GS_ERR_INVALID_ARGUMENT;
    e->ext_limit = limit;
    return GS_OK;
}

gs_status gs_handle_received_batch(gs_engine *e, uint32_t count, const uint32_t *nodes, const uint32_t *peers,
                                   const uint8_t *msgs, const uint32_t *off, const uint32_t *len, uint8_t *out,
                                   uint32_t cap, uint32_t *out_len, uint32_t *resp_off) {
    if (!e || !out_len || (count && (!nodes || !peers || !msgs || !off || !len || !resp_off)))
        return GS_ERR_INVALID_ARGUMENT;
    *out_len = 0;
    gs_status st = ext_ready(e);
    if (st != GS_OK) return st;
    // Decode and check every RPC first: the batch is applied whole or not at all.
    struct Item {
        uint32_t node, peer, rumor;
        uint8_t counter;
        bool pull, empty, offline, is_new;
    };
    std::vector<Item> it(count);
    std::set<std::pair<uint32_t, uint32_t>> peers_seen(e->ext_peers);
    std::map<uint32_t, uint32_t> fp;  // slices: first Pushes per node, this batch included
    std::vector<uint32_t> obs;
    for (uint32_t i = 0; i < count; ++i) {
        Item &v = it[i];
        if (!ext_ids(e, nodes[i], peers[i])) return GS_ERR_INVALID_ARGUMENT;
        v.node = nodes[i] - (e->shard ? e->sp.lo : 0u);  // (shards: global ids, owned by this rank)
        v.peer = peers[i];
        int pull = 0;
        uint32_t mo = 0, ml = 0;
        st = gs_rpc_decode(msgs + off[i], len[i], &pull, &mo, &ml, &v.counter);
        if (st != GS_OK) return st;  // Message::deserialise failure (src/gossiper.rs:89-94)
        v.pull = pull != 0;
        v.empty = ml == 0 && v.counter == 0;  // src/gossip.rs:153-154
        v.rumor = 0;
        if (!v.empty) {
            auto k = e->key_rumor.find(std::string(reinterpret_cast<const char *>(msgs + off[i] + mo), ml));
            if (k == e->key_rumor.end()) return GS_ERR_INVALID_ARGUMENT;  // no rumor slot for this message
            v.rumor = k->second;
        }
        // churn: a node the harness took offline this round drops it
        v.offline = e->faults.churn && gs::offline_of(e->seed, e->epoch, e->round, nodes[i], e->faults.churn);
        v.is_new = !v.offline && peers_seen.insert({v.node, v.peer}).second;  // src/gossip.rs:125
        if (v.is_new && !v.pull) {
            obs.push_back(v.node);
            if (e->slice) {  // (see slice_ext_limit)
                auto f = fp.find(v.node);
                if (f == fp.end()) {
                    auto h = e->ext_fp.find(v.node);
                    f = fp.emplace(v.node, h == e->ext_fp.end() ? 0u : h->second).first;
                }
                if (++f->second > slice_ext_limit(e)) return GS_ERR_DEVICE_LIMIT;
            }
        }
    }
    std::sort(obs.begin(), obs.end());
    obs.erase(std::unique(obs.begin(), obs.end()), obs.end());
    st = set_device(e);
    if (st != GS_OK) return st;
    // the answering nodes' state with every RPC queued before this batch (one
    // launch), then this batch's copies applied in call order on the host:
    // a copy only ever creates an absent entry (B{0,1}, or C when its counter
    // >= counter_max: src/message_state.rs:62-74) -- records never change
    // which entries are live, so the Pull responses follow from the codes
    std::vector<uint16_t> codes;
    st = observe_nodes(e, obs, codes);
    if (st != GS_OK) return st;
    auto codes_of = [&](uint32_t x) {
        const size_t j = (size_t)(std::lower_bound(obs.begin(), obs.end(), x) - obs.begin());
        return codes.data() + j * e->g.R;
    };
    uint32_t need = 0;
    auto frames = [&](bool write) {  // responses in call order; returns false when out is too small
        need = 0;
        // per answering node, the entries this batch's earlier copies created
        std::map<uint32_t, std::vector<std::pair<uint32_t, uint16_t>>> over;
        for (uint32_t i = 0; i < count; ++i) {
            const Item &v = it[i];
            if (write) resp_off[i] = need;
            if (v.offline) continue;
            if (v.is_new && !v.pull) {  // Pull responses: the node's live entries now (src/gossip.rs:126-148)
                const uint16_t *c = codes_of(v.node);
                auto &ov = over[v.node];
                auto code_at = [&](uint32_t r) {
                    for (auto &o : ov)
                        if (o.first == r) return o.second;
                    return c[r];
                };
                uint32_t cnt = 0;
                for (uint32_t r : e->key_order) {
                    const uint16_t cr = code_at(r);
                    const uint32_t tag = cr >> 14;
                    if (tag == 1 || tag == 2) {
                        const uint8_t ctr = tag == 1 ? (uint8_t)((cr >> 7) & 0x7Fu) : 255;
                        if (append_frame(1, e->keys[r], ctr, write ? out : nullptr, write ? cap : 0, &need) != GS_OK &&
                            write)
                            return false;
                        ++cnt;
                    }
                }
                if (cnt == 0 &&
                    append_frame(1, std::string(), 0, write ? out : nullptr, write ? cap : 0, &need) != GS_OK && write)
                    return false;
            }
            if (!v.empty && std::binary_search(obs.begin(), obs.end(), v.node)) {
                // the copy creates an absent entry at once (Gossip::receive,
                // src/gossip.rs:153-163): later responses of this node show it
                auto &ov = over[v.node];
                uint16_t cur = codes_of(v.node)[v.rumor];
                for (auto &o : ov)
                    if (o.first == v.rumor) cur = o.second;
                if ((cur >> 14) == 0)  // A: absent -> B{0,1}, or C{0,0} for a counter >= counter_max
                    ov.emplace_back(v.rumor, v.counter >= e->cmax ? (uint16_t)(2u << 14)
                                                                   : (uint16_t)((1u << 14) | (1u << 7)));
            }
        }
        if (write) resp_off[count] = need;
        return true;
    };
    frames(false);
    *out_len = need;
    if (!out || need > cap) return GS_ERR_SERIALISATION;  // nothing applied; *out_len holds the size needed
    frames(true);
    // queue every RPC as gs_handle_received does, in call order
    for (auto &f : fp) e->ext_fp[f.first] = f.second;
    for (uint32_t i = 0; i < count; ++i) {
        const Item &v = it[i];
        if (v.offline) continue;
        e->ext_peers.insert({v.node, v.peer});
        uint32_t info = (v.pull ? 0u : gs::kExtPush) | (v.is_new ? gs::kExtNew : 0u);
        if (v.empty) {
            info |= gs::kExtEmpty;
        } else {
            e->started = true;
            info |= v.rumor | ((uint32_t)v.counter << 12) | gs::kExtRec;
            for (auto &x : e->ext)  // only the last copy from a peer is kept in peer_counters
                if (x.node == v.node && x.peer == v.peer && !(x.info & gs::kExtEmpty) && (x.info & 0xFFFu) == v.rumor)
                    x.info &= ~gs::kExtRec;
        }
        e->ext.push_back({v.node, (uint32_t)e->ext.size(), info, v.peer});
    }
    if (count) {
        e->ext_uploaded = (uint32_t)-1;  // re-upload
        e->obs_valid = false;
    }
    return GS_OK;
}

gs_status gs_push_batch(gs_engine *e, uint32_t node, uint8_t *out, uint32_t cap, uint32_t *len,
                        uint32_t *count) {
    if (!e || !len || !count) return GS_ERR_INVALID_ARGUMENT;
    const uint32_t gnode = node;  // (shards: a global id, owned by this rank)
    if (e->shard) {
        if (node < e->sp.lo || node - e->sp.lo >= e->sp.m) return GS_ERR_INVALID_ARGUMENT;
        node -= e->sp.lo;
    }
    if (node >= e->g.n) return GS_ERR_INVALID_ARGUMENT;
    *len = 0;
    *count = 0;
    if (e->round == 0) return GS_OK;  // no round run yet: no next_round call, no push batch
    gs_status st = set_device(e);
    if (st != GS_OK) return st;
    if (e->faults.churn && gs::offline_of(e->seed, e->epoch, e->round, gnode, e->faults.churn))
        return GS_OK;  // the harness skipped this node's next_round
    // the planes of round t after phase 0 = Gossip::next_round's push list
    const gs::Geometry &g = e->g;
    std::vector<u64> w((size_t)gs::kPlanes * g.W);
    uint32_t sh = 0;
    // (on the engine stream: a non-blocking stream the legacy default stream
    // does not wait for, and the round kernel that wrote the planes runs there)
    if (g.small) {
        GS_HIP(hipMemcpyAsync(w.data(), e->S[e->cur] + (u64)(node >> g.lognpu) * gs::kPlanes,
                              gs::kPlanes * sizeof(u64), hipMemcpyDeviceToHost, e->stream));
        sh = (node & ((1u << g.lognpu) - 1u)) << g.logr;
    } else {
        GS_HIP(hipMemcpyAsync(w.data(), e->S[e->cur] + (u64)node * gs::kPlanes * g.W, w.size() * sizeof(u64),
                              hipMemcpyDeviceToHost, e->stream));
    }
    GS_HIP(hipStreamSynchronize(e->stream));
    auto bit = [&](int p, uint32_t r) -> uint32_t {
        return g.small ? (uint32_t)((w[p] >> (sh + r)) & 1u) : (uint32_t)((w[(size_t)p * g.W + (r >> 6)] >> (r & 63)) & 1u);
    };
    gs_status res = GS_OK;
    for (uint32_t r : e->key_order) {  // src/gossip.rs:93-98, in map (key) order
        const uint32_t c = bit(0, r), a0 = bit(1, r), a1 = bit(2, r);
        if (!c && (a0 | a1)) {  // B: our_counter
            if (append_frame(0, e->keys[r], (uint8_t)(a0 | (a1 << 1)), out, cap, len) != GS_OK) res = GS_ERR_SERIALISATION;
            ++*count;
        } else if (c && !(a0 & a1)) {  // C: 255
            if (append_frame(0, e->keys[r], 255, out, cap, len) != GS_OK) res = GS_ERR_SERIALISATION;
            ++*count;
        }
    }
    if (*count == 0) {  // an empty Push: a fetch request (src/gossip.rs:104-111)
        if (append_frame(0, std::string(), 0, out, cap, len) != GS_OK) res = GS_ERR_SERIALISATION;
        *count = 1;
    }
    return res;
}

gs_status gs_handle_received(gs_engine *e, uint32_t node, uint32_t peer, const uint8_t *msg, uint32_t msg_len,
                             uint8_t *out, uint32_t cap, uint32_t *out_len, uint32_t *out_count) {
    if (!e || !msg || !out_len || !out_count) return GS_ERR_INVALID_ARGUMENT;
    *out_len = 0;
    *out_count = 0;
    if (!ext_ids(e, node, peer)) return GS_ERR_INVALID_ARGUMENT;
    gs_status st = ext_ready(e);
    if (st != GS_OK) return st;
    const uint32_t gnode = node;  // (shards: a global id, owned by this rank)
    if (e->shard) node -= e->sp.lo;
    int pull = 0;
    uint32_t off = 0, mlen = 0;
    uint8_t counter = 0;
    // Message::deserialise failure: the reference logs it and returns no RPC
    // (src/gossiper.rs:89-94)
    st = gs_rpc_decode(msg, msg_len, &pull, &off, &mlen, &counter);
    if (st != GS_OK) return st;
    const bool empty = mlen == 0 && counter == 0;  // src/gossip.rs:153-154
    uint32_t rumor = 0;
    if (!empty) {
        auto it = e->key_rumor.find(std::string(reinterpret_cast<const char *>(msg + off), mlen));
        if (it == e->key_rumor.end()) return GS_ERR_INVALID_ARGUMENT;  // no rumor slot for this message
        rumor = it->second;
    }
    // churn: a node the harness took offline this round receives nothing (its
    // internal RPCs are dropped too); the RPC is dropped without effect
    if (e->faults.churn && gs::offline_of(e->seed, e->epoch, e->round, gnode, e->faults.churn)) return GS_OK;
    st = set_device(e);
    if (st != GS_OK) return st;
    const bool fresh = !e->ext_peers.count({node, peer});  // src/gossip.rs:125
    if (fresh && !pull && e->slice && e->ext_fp[node] >= slice_ext_limit(e)) return GS_ERR_DEVICE_LIMIT;
    const bool is_new = e->ext_peers.insert({node, peer}).second;
    if (is_new && !pull) {
        // Pull responses: the node's live entries now (src/gossip.rs:126-148)
        std::vector<uint16_t> codes;
        st = observe_node(e, node, codes);
        if (st != GS_OK) return st;
        gs_status res = GS_OK;
        for (uint32_t r : e->key_order) {
            const uint32_t tag = codes[r] >> 14;
            if (tag == 1 || tag == 2) {
                const uint8_t c = tag == 1 ? (uint8_t)((codes[r] >> 7) & 0x7Fu) : 255;
                if (append_frame(1, e->keys[r], c, out, cap, out_len) != GS_OK) res = GS_ERR_SERIALISATION;
                ++*out_count;
            }
        }
        if (*out_count == 0) {
            if (append_frame(1, std::string(), 0, out, cap, out_len) != GS_OK) res = GS_ERR_SERIALISATION;
            *out_count = 1;
        }
        if (res != GS_OK) {  // out too small: nothing is queued; *out_len holds the size needed
            e->ext_peers.erase({node, peer});
            return res;
        }
        ++e->ext_fp[node];
    }
    uint32_t info = (pull ? 0u : gs::kExtPush) | (is_new ? gs::kExtNew : 0u);
    if (empty) {
        info |= gs::kExtEmpty;
    } else {
        // the copy creates or updates an entry: messages() is no longer empty,
        // so Gossiper::add_peer refuses from now on (src/gossiper.rs:45-52)
        e->started = true;
        info |= rumor | ((uint32_t)counter << 12) | gs::kExtRec;
        // only the last copy from a peer is kept in peer_counters (BTreeMap::insert)
        for (auto &x : e->ext)
            if (x.node == node && x.peer == peer && !(x.info & gs::kExtEmpty) && (x.info & 0xFFFu) == rumor)
                x.info &= ~gs::kExtRec;
    }
    e->ext.push_back({node, (uint32_t)e->ext.size(), info, peer});
    e->ext_uploaded = (uint32_t)-1;  // re-upload
    e->obs_valid = false;
    return GS_OK;
}

double gs_round_kernel_bytes(const gs_engine *e) {
    // DESIGN.md "Roofline": per (node, rumor slot) 1 B state read + 1 B state
    // write (8 bit-planes) + 3/8 B class planes of each pusher (mean in-degree
    // 1) + 3/8 B class planes of t(x); per node 68 B: InRec 16 + SibRec 16 +
    // target 4 + Statistics deltas (16 r + 16 w).
    if (!e) return 0.0;
    const double n = e->g.n, rp = e->g.rpad;
    // DLV path: per slot 1 B planes read + 1 B written; per node its delivery
    // record 12 (carrying the node's own delivery flags) + its pull batch 4 +
    // u16 Statistics deltas 8 r + 8 w + the next round's push code 4 and
    // known mask 2: 38 B (the one-node-per-lane kernel,
    // SAFE_GOSSIP_AMD_DLV_PACK=0, also reads the 4-B target word).
    // Code-row shards: record 12 + target word 4 + deltas 16, the pull code
    // read at x's exchange-B slot (slot 4 + code 4 B) and the 8-B row written
    // at its exchange-A slot (slot 4 + next target word 4 + row 8): 56 B.
    if (e->dlv && e->shard) return n * (2.0 * rp + 56.0);
    if (e->dlv) return n * (2.0 * rp + (e->dlv_pack ? 38.0 : 42.0));
    return n * (2.75 * rp + 68.0);
}

const char *gs_round_kernel_name(const gs_engine *e) {
    if (!e) return "";
    if (e->shard && e->dlv) {
        if (e->g.rpad < 16) return "round_kernel_dlv4<1,u32,4,SHARD>";
        return e->dlv_pack == 2 ? "round_kernel_dlv4<1,u64,4,SHARD>"
                                : (e->dlv_pack == 3 ? "round_kernel_dlv4<1,u32,1,SHARD>" : "round_kernel_dlv4<1,u32,2,SHARD>");
    }
    if (e->shard) return e->g.small ? "round_kernel<true,1,SHARD>" : "round_kernel<false,1,SHARD>";
    if (e->seq) return e->g.small ? "round_kernel<true,1,SEQ>" : "round_kernel<false,1,SEQ>";
    if (e->dlv) {
        if (e->dlv_pack == 0) return "round_kernel<true,1,DLV> (one node per lane)";
        if (e->g.rpad < 16) return "round_kernel_dlv4<1,u32,4>";
        return e->dlv_pack == 2 ? "round_kernel_dlv4<1,u64,4>"
                                : (e->dlv_pack == 3 ? "round_kernel_dlv4<1,u32,1>" : "round_kernel_dlv4<1,u32,2>");
    }
    if (e->filt && e->w32 && (e->g.small ? e->g.rpad == 32 : e->g.logr <= 8))
        return "round_kernel_w32<1> (32-bit lanes, live-filtered gathers)";
    if (e->filt) return e->g.small ? "round_kernel<true,1> (live-filtered gathers)"
                                   : "round_kernel<false,1> (live-filtered gathers)";
    return e->g.small ? "round_kernel<true,1>" : "round_kernel<false,1>";
}

gs_status gs_round_traffic(gs_engine *e, double *bytes_per_launch, uint32_t *launches) {
    if (!e || !bytes_per_launch || !launches) return GS_ERR_INVALID_ARGUMENT;
    const double dense = gs_round_kernel_bytes(e);
    if (e->filt) {
        // Live-filtered launches: per node the 68 B of gs_round_kernel_bytes
        // plus its zl bit and the two map bits written, and its planes read
        // and written (2 R_pad B); per node class row the build left to gather
        // (pushers, t(x), t(x)'s earlier pushers) 3 planes of R_pad bits.
        gs_status st = set_device(e);
        if (st != GS_OK) return st;
        *launches = e->filt_launches;
        if (e->filt_launches == 0) {
            *bytes_per_launch = dense;
            return GS_OK;
        }
        u64 rows = 0;
        GS_HIP(hipStreamSynchronize(e->stream));
        GS_HIP(hipMemcpy(&rows, e->acct, sizeof(u64), hipMemcpyDeviceToHost));
        const double n = e->g.n, rp = e->g.rpad;
        *bytes_per_launch = n * (68.0 + 3.0 / 8.0 + 2.0 * rp) + 3.0 * rp / 8.0 * (double)rows / e->filt_launches;
        return GS_OK;
    }
    *bytes_per_launch = dense;
    *launches = 0;
    return GS_OK;
}

}  // extern "C"
