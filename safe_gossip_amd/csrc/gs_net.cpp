// gs_net.cpp -- a whole multi-GPU network behind the C ABI (include/
// safe_gossip.h "gs_net"): the per-round loop that
// safe_gossip_amd/sharded.py and sliced.py drive from Python, in C++, so a
// host without Python (the north star's Rust crate, examples/net_rounds.cpp)
// gets node shards or rumor slices over several GPUs from gs_net_* calls only.
//
// One process per GPU joined through RCCL (gs_net_create): the exchanges are
// RCCL collectives on a communication stream of the rank, ordered against the
// engine stream with events -- issued after the engine stream's work so far,
// waited for by the engine stream (never the host) when their rows are
// needed, so a round is enqueued without a host synchronisation:
//   node shards  -- part h of exchange A / B = one ncclAllToAll over the part's
//                   contiguous region (gs_shard.hip layout), parts pipelined
//                   against the round kernel of other parts;
//   rumor slices -- one ncclAllReduce(MIN) of the 2 B/node empty-RPC counts per
//                   round, folded into a later round kernel (gs_slice_defer).
// RCCL is loaded at run time (dlopen: the library itself has no link-time
// dependency on it; a process that already holds RCCL shares that copy).
//
// gs_net_create_local runs every rank in this process on one device and
// exchanges by device copies with host synchronisation (the "local" transport
// of the Python wrappers): a test transport for the same loop at world > 1 on
// one GPU.  gs_net_create_with takes the collectives from the caller (any
// transport: MPI, sockets, gloo) and runs them on host-staged buffers after a
// synchronisation of the rank -- no RCCL needed, several ranks may share a
// GPU (the rehearsal of the multi-process loop on one box).
#include "../../include/safe_gossip.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string>
#include <utility>
#include <vector>

namespace {

// ------------------------------------------------------------------ RCCL
struct Rccl {
    bool tried = false, ok = false;
    decltype(&ncclGetUniqueId) getUniqueId = nullptr;
    decltype(&ncclCommInitRank) commInitRank = nullptr;
    decltype(&ncclCommDestroy) commDestroy = nullptr;
    decltype(&ncclAllToAll) allToAll = nullptr;
    decltype(&ncclAllReduce) allReduce = nullptr;
    decltype(&ncclAllGather) allGather = nullptr;
    decltype(&ncclGetErrorString) errorString = nullptr;
};

Rccl &rccl() {
    static Rccl r;
    if (r.tried) return r;
    r.tried = true;
    void *h = nullptr;
    // an RCCL the process already holds (e.g. torch's), else the named or
    // the system one
    for (const char *name : {"librccl.so", "librccl.so.1"})
        if (!h) h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
    const char *env = std::getenv("SAFE_GOSSIP_AMD_RCCL");
    if (!h && env && *env) h = dlopen(env, RTLD_NOW);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW);
    if (!h) return r;
    r.getUniqueId = reinterpret_cast<decltype(r.getUniqueId)>(dlsym(h, "ncclGetUniqueId"));
    r.commInitRank = reinterpret_cast<decltype(r.commInitRank)>(dlsym(h, "ncclCommInitRank"));
    r.commDestroy = reinterpret_cast<decltype(r.commDestroy)>(dlsym(h, "ncclCommDestroy"));
    r.allToAll = reinterpret_cast<decltype(r.allToAll)>(dlsym(h, "ncclAllToAll"));
    r.allReduce = reinterpret_cast<decltype(r.allReduce)>(dlsym(h, "ncclAllReduce"));
    r.allGather = reinterpret_cast<decltype(r.allGather)>(dlsym(h, "ncclAllGather"));
    r.errorString = reinterpret_cast<decltype(r.errorString)>(dlsym(h, "ncclGetErrorString"));
    r.ok = r.getUniqueId && r.commInitRank && r.commDestroy && r.allToAll && r.allReduce && r.allGather &&
           r.errorString;
    return r;
}

bool debug_on() {
    static const bool on = [] {
        const char *v = std::getenv("SAFE_GOSSIP_AMD_DEBUG");
        return v && *v && *v != '0';
    }();
    return on;
}

#define NET_HIP(expr)                                                                                    \
    do {                                                                                                 \
        hipError_t _e = (expr);                                                                          \
        if (_e != hipSuccess) {                                                                          \
            if (debug_on())                                                                              \
                std::fprintf(stderr, "safe_gossip_amd: %s failed at gs_net.cpp:%d: %s\n", #expr, __LINE__, \
                             hipGetErrorString(_e));                                                     \
            return GS_ERR_HIP;                                                                           \
        }                                                                                                \
    } while (0)
#define NET_NCCL(expr)                                                                                   \
    do {                                                                                                 \
        ncclResult_t _r = (expr);                                                                        \
        if (_r != ncclSuccess) {                                                                         \
            if (debug_on())                                                                              \
                std::fprintf(stderr, "safe_gossip_amd: %s failed at gs_net.cpp:%d: %s\n", #expr, __LINE__, \
                             rccl().errorString(_r));                                                    \
            return GS_ERR_HIP;                                                                           \
        }                                                                                                \
    } while (0)
#define NET_ST(expr)                  \
    do {                              \
        gs_status _s = (expr);        \
        if (_s != GS_OK) return _s;   \
    } while (0)

// RCCL's all-to-all returns wrong bytes past 2^30 per rank (DESIGN.md section
// 7, "The single-part stall"); SAFE_GOSSIP_AMD_RCCL_MAX_BYTES lowers it (tests).
size_t rccl_max_bytes() {
    const char *v = std::getenv("SAFE_GOSSIP_AMD_RCCL_MAX_BYTES");
    const long long b = v && *v ? std::atoll(v) : 0;
    return b > 0 ? (size_t)b : ((size_t)1 << 30);
}

}  // namespace

// One rank of the network held by this process.
struct NetRank {
    gs_engine *e = nullptr;
    int device = 0;
    hipStream_t stream = nullptr;  // the engine's stream (gs_stream)
    hipStream_t cs = nullptr;      // RCCL: collectives of this rank
    // node shard: layout (gs_shard_info) and exchange buffers
    uint32_t info[14] = {};
    uint32_t *sendA[2] = {nullptr, nullptr}, *recvA[2] = {nullptr, nullptr};
    uint32_t *sendB = nullptr, *recvB = nullptr;
    // rumor slice: rumors [lo, hi), empty-count buffers of rounds t % 3, obs
    uint32_t lo = 0, hi = 0;
    uint8_t *buf[3] = {nullptr, nullptr, nullptr};
    uint8_t *obs = nullptr;
    // RCCL scratch for observers (grown only)
    void *scratch = nullptr;
    size_t scratch_bytes = 0;
};

struct gs_net {
    gs_net_mode mode = GS_NET_SLICES;
    bool dist = false;  // one rank per process (RCCL or the host's collectives); else every rank here
    bool host = false;  // dist over collectives the caller brings (gs_net_create_with), on host buffers
    gs_net_collectives coll{};
    uint32_t world = 1, rank = 0;
    uint32_t n = 0, R = 0, parts = 1;
    bool codes = false;  // node shards: code rows (R_pad <= 16, 2P)
    ncclComm_t comm = nullptr;
    std::vector<NetRank> ranks;
    uint32_t round = 0;
    bool delivered = true;
    // RCCL work not yet waited for by the engine stream: events on cs
    std::vector<hipEvent_t> pendA;
    std::vector<hipEvent_t> pendB;  // per part (nullptr: nothing to wait for)
    std::deque<std::pair<hipEvent_t, uint32_t>> pend_slice;  // (event, round buffer)
    std::vector<hipEvent_t> free_ev;
};

namespace {

// ------------------------------------------------------------ events
gs_status take_event(gs_net *net, hipEvent_t *ev) {
    if (!net->free_ev.empty()) {
        *ev = net->free_ev.back();
        net->free_ev.pop_back();
        return GS_OK;
    }
    NET_HIP(hipEventCreateWithFlags(ev, hipEventDisableTiming));
    return GS_OK;
}

// The engine stream waits for `ev` (recorded on the comm stream); the event
// goes back to the pool (a later record does not affect this wait).
gs_status engine_wait(gs_net *net, NetRank &r, hipEvent_t ev) {
    if (!ev) return GS_OK;
    NET_HIP(hipStreamWaitEvent(r.stream, ev, 0));
    net->free_ev.push_back(ev);
    return GS_OK;
}

// The comm stream waits for the engine stream's work so far.
gs_status comm_after_engine(gs_net *net, NetRank &r) {
    hipEvent_t ev;
    NET_ST(take_event(net, &ev));
    NET_HIP(hipEventRecord(ev, r.stream));
    NET_HIP(hipStreamWaitEvent(r.cs, ev, 0));
    net->free_ev.push_back(ev);
    return GS_OK;
}

gs_status comm_done(gs_net *net, NetRank &r, hipEvent_t *out) {
    NET_ST(take_event(net, out));
    NET_HIP(hipEventRecord(*out, r.cs));
    return GS_OK;
}

gs_status sync_all(gs_net *net) {
    for (auto &r : net->ranks) {
        NET_ST(gs_sync(r.e));
        if (r.cs) {
            NET_HIP(hipSetDevice(r.device));
            NET_HIP(hipStreamSynchronize(r.cs));
        }
    }
    return GS_OK;
}

// ------------------------------------------------------------ host collectives
// gs_net_create_with: the caller's collectives on host buffers the library
// stages; every call follows a synchronisation of this rank's engine (its
// engine and side streams), so the exchanged bytes are final and nothing
// still reads the buffers a result lands in.
gs_status host_call(int rc) { return rc == 0 ? GS_OK : GS_ERR_IO; }

// Host bytes into a device buffer the engine's kernels read next: on the
// engine stream, waited for before the host buffer goes.  (A plain hipMemcpy
// runs on the null stream, which a non-blocking engine stream does not wait
// for, and a pageable upload may return before its data lands.)
gs_status upload_to_engine(NetRank &r, void *dst, const void *src, size_t bytes) {
    NET_HIP(hipSetDevice(r.device));
    NET_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, r.stream));
    NET_HIP(hipStreamSynchronize(r.stream));
    return GS_OK;
}

gs_status host_alltoall_dev(gs_net *net, NetRank &r, const void *send, void *recv, size_t bytes_per_rank) {
    NET_ST(gs_sync(r.e));
    NET_HIP(hipSetDevice(r.device));
    std::vector<uint8_t> hs(bytes_per_rank * net->world), hr(bytes_per_rank * net->world);
    NET_HIP(hipMemcpy(hs.data(), send, hs.size(), hipMemcpyDeviceToHost));
    NET_ST(host_call(net->coll.alltoall(net->coll.ctx, hs.data(), hr.data(), bytes_per_rank)));
    return upload_to_engine(r, recv, hr.data(), hr.size());
}

// MIN over the ranks of `bytes` device bytes, in place (host collectives).
gs_status host_min_u8_dev(gs_net *net, NetRank &r, uint8_t *buf, size_t bytes) {
    NET_ST(gs_sync(r.e));
    NET_HIP(hipSetDevice(r.device));
    std::vector<uint8_t> h(bytes);
    NET_HIP(hipMemcpy(h.data(), buf, bytes, hipMemcpyDeviceToHost));
    NET_ST(host_call(net->coll.allreduce(net->coll.ctx, h.data(), bytes, GS_NET_U8, GS_NET_MIN)));
    return upload_to_engine(r, buf, h.data(), bytes);
}

// ------------------------------------------------------------ node shards
// Part h of exchange A (buffer set k) or B: (first u32 word, u32 words per
// rank sub-block); the part's `world` sub-blocks are contiguous.
std::pair<size_t, size_t> region(const NetRank &r, bool A, uint32_t h) {
    const uint32_t capP = r.info[2], idrows = r.info[3], world = r.info[5], P = r.info[8];
    const uint32_t wa = r.info[4], wb = r.info[12];
    const size_t rows = capP + (A && h == P - 1 ? idrows : 0u);
    const size_t w = A ? wa : wb;
    return {(size_t)h * world * capP * w, rows * w};
}

// Issue part h of exchange A (set k) or B.  RCCL: one all-to-all on the comm
// stream after the engine stream's work so far; *ev = its completion (null:
// nothing moved).  Local: every rank's sub-blocks copied at once, after every
// engine finished.
gs_status exchange(gs_net *net, bool A, uint32_t h, uint32_t k, hipEvent_t *ev) {
    *ev = nullptr;
    const bool own = net->codes && net->world == 1;  // one code-row rank: rows written in place
    if (!net->dist) {
        // (every engine idle: the sources are final and no reader of the
        // receive buffers is left; each copy runs on its destination's engine
        // stream, ahead of the kernels that read it)
        NET_ST(sync_all(net));
        for (uint32_t d = 0; d < net->world; ++d)
            for (uint32_t s = 0; s < net->world; ++s) {
                if (own && s == d) continue;
                NetRank &src = net->ranks[s], &dst = net->ranks[d];
                const auto rg = region(src, A, h);
                const uint32_t *sb = A ? src.sendA[k] : src.sendB;
                uint32_t *rb = A ? dst.recvA[k] : dst.recvB;
                NET_HIP(hipSetDevice(dst.device));
                NET_HIP(hipMemcpyAsync(rb + rg.first + s * rg.second, sb + rg.first + d * rg.second,
                                       rg.second * sizeof(uint32_t), hipMemcpyDeviceToDevice, dst.stream));
            }
        return GS_OK;
    }
    if (own) return GS_OK;
    NetRank &r = net->ranks[0];
    const auto rg = region(r, A, h);
    const uint32_t *sb = (A ? r.sendA[k] : r.sendB) + rg.first;
    uint32_t *rb = (A ? r.recvA[k] : r.recvB) + rg.first;
    if (net->host) return host_alltoall_dev(net, r, sb, rb, rg.second * sizeof(uint32_t));
    NET_HIP(hipSetDevice(r.device));
    NET_ST(comm_after_engine(net, r));
    const size_t limit = rccl_max_bytes() / sizeof(uint32_t);
    if (net->world * rg.second <= limit) {
        NET_NCCL(rccl().allToAll(sb, rb, rg.second, ncclUint32, net->comm, r.cs));
    } else {
        // one rank: its span is its own block, moved in pieces (checked at
        // creation: several ranks never need this)
        for (size_t a = 0; a < rg.second; a += limit)
            NET_NCCL(rccl().allToAll(sb + a, rb + a, std::min(limit, rg.second - a), ncclUint32, net->comm, r.cs));
    }
    return comm_done(net, r, ev);
}

gs_status wait_list(gs_net *net, std::vector<hipEvent_t> &evs) {
    for (hipEvent_t ev : evs)
        if (ev) NET_ST(engine_wait(net, net->ranks[0], ev));
    evs.clear();
    return GS_OK;
}

// Exchange A of the current round complete (round 1, class rows: also the
// ids of round 1), the pull rows, and every part of exchange B issued.
gs_status shard_deliver(gs_net *net) {
    if (net->delivered || net->round == 0) return GS_OK;
    const uint32_t t = net->round;
    if (t == 1 && !net->codes) {
        hipEvent_t ev;
        NET_ST(exchange(net, true, net->parts - 1, 0, &ev));
        net->pendA.push_back(ev);
    }
    NET_ST(wait_list(net, net->pendA));
    for (auto &r : net->ranks) NET_ST(gs_shard_pull(r.e));
    net->pendB.assign(net->parts, nullptr);
    for (uint32_t h = 0; h < net->parts; ++h) NET_ST(exchange(net, false, h, 0, &net->pendB[h]));
    net->delivered = true;
    return GS_OK;
}

gs_status wait_b(gs_net *net, uint32_t h) {
    if (h >= net->pendB.size()) return GS_OK;
    hipEvent_t ev = net->pendB[h];
    net->pendB[h] = nullptr;
    return ev ? engine_wait(net, net->ranks[0], ev) : GS_OK;
}

gs_status shard_wait_all(gs_net *net) {
    NET_ST(wait_list(net, net->pendA));
    for (uint32_t h = 0; h < net->pendB.size(); ++h) NET_ST(wait_b(net, h));
    net->pendB.clear();
    return GS_OK;
}

gs_status shard_round(gs_net *net, bool report, bool *live) {
    NET_ST(shard_deliver(net));
    const uint32_t k = (net->round + 1) % 2;
    for (uint32_t h = 0; h + 1 < net->parts; ++h) {
        NET_ST(wait_b(net, h));
        for (auto &r : net->ranks) NET_ST(gs_shard_round_part(r.e, h));
        hipEvent_t ev;
        NET_ST(exchange(net, true, h, k, &ev));
        net->pendA.push_back(ev);
    }
    NET_ST(wait_b(net, net->parts - 1));
    net->pendB.clear();
    *live = false;
    for (auto &r : net->ranks) {
        gs_round_report rep{};
        NET_ST(gs_next_round(r.e, report ? &rep : nullptr));
        *live = *live || rep.any_live;
    }
    hipEvent_t ev;
    NET_ST(exchange(net, true, net->parts - 1, k, &ev));
    net->pendA.push_back(ev);
    net->delivered = false;
    return GS_OK;
}

// ------------------------------------------------------------ rumor slices
gs_status slice_apply_pending(gs_net *net, size_t keep) {
    while (net->pend_slice.size() > keep) {
        auto p = net->pend_slice.front();
        net->pend_slice.pop_front();
        NetRank &r = net->ranks[0];
        NET_ST(engine_wait(net, r, p.first));
        NET_ST(keep ? gs_slice_defer(r.e, p.second) : gs_slice_apply(r.e, p.second));
    }
    return GS_OK;
}

// MIN over the local slices' device byte buffers buf_of(rank), into each
// (host-staged: the in-process test transport).
template <typename BufOf>
gs_status local_min_u8(gs_net *net, BufOf buf_of, size_t bytes) {
    NET_ST(sync_all(net));
    std::vector<uint8_t> m(bytes, 0xFF), v(bytes);
    for (auto &r : net->ranks) {
        NET_HIP(hipMemcpy(v.data(), buf_of(r), bytes, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < bytes; ++i) m[i] = std::min(m[i], v[i]);
    }
    for (auto &r : net->ranks) NET_ST(upload_to_engine(r, buf_of(r), m.data(), bytes));
    return GS_OK;
}

gs_status slice_round(gs_net *net, bool report, bool *live) {
    *live = false;
    for (auto &r : net->ranks) {
        gs_round_report rep{};
        NET_ST(gs_next_round(r.e, report ? &rep : nullptr));
        *live = *live || rep.any_live;
    }
    const uint32_t b = (net->round + 1) % 3;  // the round just run wrote buf[t % 3]
    if (!net->dist) {
        NET_ST(local_min_u8(net, [b](NetRank &r) { return r.buf[b]; }, 2 * (size_t)net->n));
        for (auto &r : net->ranks) NET_ST(gs_slice_defer(r.e, b));  // added by the next round kernel
        return GS_OK;
    }
    NetRank &r = net->ranks[0];
    if (net->host) {  // reduced now, added by the next round kernel
        NET_ST(host_min_u8_dev(net, r, r.buf[b], 2 * (size_t)net->n));
        return gs_slice_defer(r.e, b);
    }
    NET_HIP(hipSetDevice(r.device));
    NET_ST(comm_after_engine(net, r));
    NET_NCCL(rccl().allReduce(r.buf[b], r.buf[b], 2 * (size_t)net->n, ncclUint8, ncclMin, net->comm, r.cs));
    hipEvent_t ev;
    NET_ST(comm_done(net, r, &ev));
    net->pend_slice.emplace_back(ev, b);
    return slice_apply_pending(net, 1);  // round t-1's counts: folded into round t+1's kernel
}

gs_status flush(gs_net *net) {
    if (net->mode == GS_NET_SHARDS) return shard_wait_all(net);
    return slice_apply_pending(net, 0);
}

// Before an observer: the pending round delivered (node shards: exchange A
// in, pull rows, exchange B waited for -- observers show the state after the
// round's deliveries, as on one engine) and every reduction applied.
gs_status observe_ready(gs_net *net) {
    if (net->mode == GS_NET_SHARDS) NET_ST(shard_deliver(net));
    return flush(net);
}

// ------------------------------------------------------------ RCCL helpers
gs_status grow_scratch(NetRank &r, size_t bytes) {
    if (r.scratch_bytes >= bytes) return GS_OK;
    NET_HIP(hipSetDevice(r.device));
    if (r.scratch) {
        NET_HIP(hipStreamSynchronize(r.cs));
        NET_HIP(hipFree(r.scratch));
    }
    r.scratch = nullptr;
    r.scratch_bytes = 0;
    NET_HIP(hipMalloc(&r.scratch, bytes));
    r.scratch_bytes = bytes;
    return GS_OK;
}

// In-place all-reduce of host data over the ranks (RCCL; synchronous).
gs_status host_allreduce(gs_net *net, void *data, size_t count, ncclDataType_t dt, size_t elem, ncclRedOp_t op) {
    if (!net->dist || net->world == 1) return GS_OK;
    if (net->host) {
        const int hdt = dt == ncclUint8 ? GS_NET_U8 : (dt == ncclUint32 ? GS_NET_U32 : GS_NET_U64);
        const int hop = op == ncclSum ? GS_NET_SUM : (op == ncclMin ? GS_NET_MIN : GS_NET_MAX);
        return host_call(net->coll.allreduce(net->coll.ctx, data, count, hdt, hop));
    }
    NetRank &r = net->ranks[0];
    NET_ST(grow_scratch(r, count * elem));
    NET_HIP(hipSetDevice(r.device));
    NET_HIP(hipMemcpyAsync(r.scratch, data, count * elem, hipMemcpyHostToDevice, r.cs));
    NET_NCCL(rccl().allReduce(r.scratch, r.scratch, count, dt, op, net->comm, r.cs));
    NET_HIP(hipMemcpyAsync(data, r.scratch, count * elem, hipMemcpyDeviceToHost, r.cs));
    NET_HIP(hipStreamSynchronize(r.cs));
    return GS_OK;
}

// Every rank's `bytes` (host) gathered in rank order into out (host, world*bytes).
gs_status host_allgather(gs_net *net, const void *mine, size_t bytes, void *out) {
    if (!net->dist || net->world == 1) {
        std::memcpy(out, mine, bytes);
        return GS_OK;
    }
    if (net->host) return host_call(net->coll.allgather(net->coll.ctx, mine, out, bytes));
    NetRank &r = net->ranks[0];
    NET_ST(grow_scratch(r, bytes * (net->world + 1)));
    uint8_t *s = static_cast<uint8_t *>(r.scratch), *g = s + bytes;
    NET_HIP(hipSetDevice(r.device));
    NET_HIP(hipMemcpyAsync(s, mine, bytes, hipMemcpyHostToDevice, r.cs));
    NET_NCCL(rccl().allGather(s, g, bytes, ncclUint8, net->comm, r.cs));
    NET_HIP(hipMemcpyAsync(out, g, bytes * net->world, hipMemcpyDeviceToHost, r.cs));
    NET_HIP(hipStreamSynchronize(r.cs));
    return GS_OK;
}

// ------------------------------------------------------------ lifecycle
void release(gs_net *net) {
    if (!net) return;
    for (auto &r : net->ranks) {
        if (r.e) (void)gs_sync(r.e);
        (void)hipSetDevice(r.device);
        if (r.cs) (void)hipStreamSynchronize(r.cs);
    }
    if (net->comm) (void)rccl().commDestroy(net->comm);
    for (auto &r : net->ranks) {
        (void)hipSetDevice(r.device);
        void *bufs[] = {r.sendA[0], r.sendA[1], r.recvA[0], r.recvA[1], r.sendB, r.recvB,
                        r.buf[0],   r.buf[1],   r.buf[2],   r.obs,      r.scratch};
        for (void *b : bufs)
            if (b) (void)hipFree(b);
        if (r.cs) (void)hipStreamDestroy(r.cs);
        if (r.e) gs_destroy(r.e);
    }
    for (hipEvent_t ev : net->free_ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : net->pendA)
        if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : net->pendB)
        if (ev) (void)hipEventDestroy(ev);
    for (auto &p : net->pend_slice) (void)hipEventDestroy(p.first);
    delete net;
}

template <typename T>
gs_status zalloc(T **p, size_t count) {
    NET_HIP(hipMalloc((void **)p, std::max<size_t>(count, 1) * sizeof(T)));
    NET_HIP(hipMemset(*p, 0, std::max<size_t>(count, 1) * sizeof(T)));
    // (the null stream's memset done before any engine or comm stream --
    // non-blocking, not ordered after it -- touches the buffer)
    NET_HIP(hipDeviceSynchronize());
    return GS_OK;
}

// Rank g's engine and buffers (device cfg->device).
gs_status make_rank(gs_net *net, const gs_config *cfg, uint32_t g, NetRank &r) {
    gs_config c = *cfg;
    if (net->mode == GS_NET_SHARDS) {
        NET_ST(gs_shard_create_parts(&c, g, net->world, net->parts, &r.e));
        NET_ST(gs_shard_info(r.e, r.info));
        const size_t rowsA = r.info[10], rowsB = r.info[11], wa = r.info[4], wb = r.info[12];
        r.device = gs_device(r.e);
        NET_HIP(hipSetDevice(r.device));
        for (int i = 0; i < 2; ++i) {
            NET_ST(zalloc(&r.sendA[i], rowsA * wa));
            NET_ST(zalloc(&r.recvA[i], rowsA * wa));
        }
        NET_ST(zalloc(&r.sendB, rowsB * wb));
        NET_ST(zalloc(&r.recvB, rowsB * wb));
        NET_ST(gs_shard_bind(r.e, r.sendA[0], r.sendA[1], r.recvA[0], r.recvA[1], r.sendB, r.recvB));
    } else {
        r.lo = (uint32_t)((uint64_t)g * net->R / net->world);
        r.hi = (uint32_t)((uint64_t)(g + 1) * net->R / net->world);
        c.n_rumors = r.hi - r.lo;
        c.rumor_slice = 1;
        NET_ST(gs_create(&c, &r.e));
        r.device = gs_device(r.e);
        NET_HIP(hipSetDevice(r.device));
        for (int i = 0; i < 3; ++i) NET_ST(zalloc(&r.buf[i], 2 * (size_t)net->n));
        NET_ST(zalloc(&r.obs, (size_t)net->n));
        NET_ST(gs_slice_bind(r.e, r.buf[0], r.buf[1], r.buf[2], r.obs));
        // one bound on external first Pushes for the whole network: the
        // smallest slice's (gs_slice_set_ext_limit)
        const uint32_t rmin = net->R / net->world;
        uint32_t rp = 1;
        while (rp < rmin) rp <<= 1;
        NET_ST(gs_slice_set_ext_limit(r.e, std::min<uint32_t>(200u, 32u * rp)));
    }
    r.stream = reinterpret_cast<hipStream_t>(gs_stream(r.e));
    if (net->dist && !net->host) NET_HIP(hipStreamCreateWithFlags(&r.cs, hipStreamNonBlocking));
    return GS_OK;
}

gs_status check_net_args(const gs_config *cfg, gs_net_mode mode, uint32_t world, uint32_t parts) {
    if (!cfg || world == 0 || (mode != GS_NET_SLICES && mode != GS_NET_SHARDS)) return GS_ERR_INVALID_ARGUMENT;
    if (mode == GS_NET_SLICES && cfg->n_rumors < world) return GS_ERR_INVALID_ARGUMENT;  // a slice per rank
    if (mode == GS_NET_SHARDS && (parts == 0 || cfg->schedule == GS_SCHED_SEQ)) return GS_ERR_UNSUPPORTED;
    if (cfg->rumor_slice) return GS_ERR_INVALID_ARGUMENT;
    return GS_OK;
}

gs_status finish_create(gs_net *net, const gs_config *cfg) {
    for (uint32_t i = 0; i < (net->dist ? 1u : net->world); ++i) {
        net->ranks.emplace_back();
        NET_ST(make_rank(net, cfg, net->dist ? net->rank : i, net->ranks.back()));
    }
    if (net->mode == GS_NET_SHARDS) {
        const NetRank &r = net->ranks[0];
        net->parts = r.info[8];  // parts that hold nodes (gs_shard_info)
        net->codes = r.info[13] != 0;
        if (net->dist && !net->host && net->world > 1) {  // every exchange within RCCL's exact range
            size_t biggest = 0;
            for (uint32_t h = 0; h < net->parts; ++h)
                for (bool A : {true, false}) biggest = std::max(biggest, net->world * region(r, A, h).second * 4);
            if (biggest > rccl_max_bytes()) return GS_ERR_UNSUPPORTED;  // more pipeline parts needed
        }
    }
    return GS_OK;
}

}  // namespace

extern "C" {

gs_status gs_net_unique_id(uint8_t id[GS_NET_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == GS_NET_ID_BYTES, "RCCL unique id size");
    if (!id) return GS_ERR_INVALID_ARGUMENT;
    if (!rccl().ok) return GS_ERR_UNSUPPORTED;  // no RCCL in this process or on the system
    ncclUniqueId u;
    NET_NCCL(rccl().getUniqueId(&u));
    std::memcpy(id, &u, sizeof(u));
    return GS_OK;
}

gs_status gs_net_create(const gs_config *cfg, gs_net_mode mode, uint32_t rank, uint32_t world, uint32_t parts,
                        const uint8_t id[GS_NET_ID_BYTES], gs_net **out) {
    if (!out || !id || rank >= world) return GS_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    NET_ST(check_net_args(cfg, mode, world, parts));
    if (!rccl().ok) return GS_ERR_UNSUPPORTED;
    gs_net *net = new gs_net();
    net->mode = mode;
    net->dist = true;
    net->world = world;
    net->rank = rank;
    net->n = cfg->n_nodes;
    net->R = cfg->n_rumors;
    net->parts = parts ? parts : 1u;
    gs_status st = GS_OK;
    int dev = cfg->device;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) st = GS_ERR_HIP;
    if (st == GS_OK && hipSetDevice(dev) != hipSuccess) st = GS_ERR_HIP;
    if (st == GS_OK) {
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        if (rccl().commInitRank(&net->comm, (int)world, u, (int)rank) != ncclSuccess) {
            net->comm = nullptr;
            st = GS_ERR_HIP;
        }
    }
    if (st == GS_OK) {
        gs_config c = *cfg;
        c.device = dev;
        st = finish_create(net, &c);
    }
    if (st != GS_OK) {
        release(net);
        return st;
    }
    *out = net;
    return GS_OK;
}

gs_status gs_net_create_local(const gs_config *cfg, gs_net_mode mode, uint32_t world, uint32_t parts, gs_net **out) {
    if (!out) return GS_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    NET_ST(check_net_args(cfg, mode, world, parts));
    gs_net *net = new gs_net();
    net->mode = mode;
    net->world = world;
    net->n = cfg->n_nodes;
    net->R = cfg->n_rumors;
    net->parts = parts ? parts : 1u;
    const gs_status st = finish_create(net, cfg);
    if (st != GS_OK) {
        release(net);
        return st;
    }
    *out = net;
    return GS_OK;
}

gs_status gs_net_create_with(const gs_config *cfg, gs_net_mode mode, uint32_t rank, uint32_t world, uint32_t parts,
                             const gs_net_collectives *coll, gs_net **out) {
    if (!out || !coll || !coll->alltoall || !coll->allreduce || !coll->allgather || rank >= world)
        return GS_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    NET_ST(check_net_args(cfg, mode, world, parts));
    gs_net *net = new gs_net();
    net->mode = mode;
    net->dist = true;
    net->host = true;
    net->coll = *coll;
    net->world = world;
    net->rank = rank;
    net->n = cfg->n_nodes;
    net->R = cfg->n_rumors;
    net->parts = parts ? parts : 1u;
    const gs_status st = finish_create(net, cfg);
    if (st != GS_OK) {
        release(net);
        return st;
    }
    *out = net;
    return GS_OK;
}

void gs_net_destroy(gs_net *net) {
    if (net) (void)flush(net);
    release(net);
}

uint32_t gs_net_local_engines(const gs_net *net) { return net ? (uint32_t)net->ranks.size() : 0u; }

gs_engine *gs_net_engine(gs_net *net, uint32_t i) {
    return net && i < net->ranks.size() ? net->ranks[i].e : nullptr;
}

gs_status gs_net_send_new(gs_net *net, uint32_t node, uint32_t rumor) {
    if (!net) return GS_ERR_INVALID_ARGUMENT;
    if (net->n < 2) return GS_ERR_NO_PEERS;  // src/gossiper.rs:56-58
    if (node >= net->n || rumor >= net->R) return GS_ERR_INVALID_ARGUMENT;
    for (auto &r : net->ranks) {
        if (net->mode == GS_NET_SHARDS) {
            if (node >= r.info[0] && node - r.info[0] < r.info[1]) NET_ST(gs_send_new(r.e, node, rumor));
        } else if (rumor >= r.lo && rumor < r.hi) {
            NET_ST(gs_send_new(r.e, node, rumor - r.lo));
        }
    }
    return GS_OK;
}

gs_status gs_net_next_round(gs_net *net, gs_round_report *report) {
    if (!net) return GS_ERR_INVALID_ARGUMENT;
    bool live = false;
    NET_ST(net->mode == GS_NET_SHARDS ? shard_round(net, report != nullptr, &live)
                                      : slice_round(net, report != nullptr, &live));
    net->round += 1;
    if (!report) return GS_OK;
    uint32_t any = live ? 1u : 0u;
    NET_ST(host_allreduce(net, &any, 1, ncclUint32, sizeof(uint32_t), ncclMax));
    report->round = net->round;
    report->any_live = any;
    return GS_OK;
}

gs_status gs_net_sync(gs_net *net) {
    if (!net) return GS_ERR_INVALID_ARGUMENT;
    NET_ST(flush(net));
    return sync_all(net);
}

gs_status gs_net_clear(gs_net *net, uint32_t epoch) {
    if (!net) return GS_ERR_INVALID_ARGUMENT;
    NET_ST(flush(net));
    NET_ST(sync_all(net));  // no exchange of the old epoch may still write the buffers
    gs_status st = GS_OK;
    for (auto &r : net->ranks) {
        const gs_status s = gs_clear(r.e, epoch);
        if (st == GS_OK) st = s;
    }
    net->round = 0;
    net->delivered = true;
    return st;
}

gs_status gs_net_known_counts(gs_net *net, uint64_t *known_total, uint64_t *nodes_complete) {
    if (!net || !known_total || !nodes_complete) return GS_ERR_INVALID_ARGUMENT;
    NET_ST(observe_ready(net));
    uint64_t v[2] = {0, 0};
    if (net->mode == GS_NET_SHARDS) {
        for (auto &r : net->ranks) {
            uint64_t t = 0, c = 0;
            if (r.info[1]) NET_ST(gs_known_counts(r.e, &t, &c));
            v[0] += t;
            v[1] += c;
        }
        NET_ST(host_allreduce(net, v, 2, ncclUint64, sizeof(uint64_t), ncclSum));
    } else {
        // a node is complete when it knows every rumor of every slice
        std::vector<uint32_t> sum(net->n, 0), cnt(net->n);
        for (auto &r : net->ranks) {
            NET_ST(gs_known_popcounts(r.e, cnt.data()));
            for (uint32_t x = 0; x < net->n; ++x) sum[x] += cnt[x];
        }
        NET_ST(host_allreduce(net, sum.data(), net->n, ncclUint32, sizeof(uint32_t), ncclSum));
        for (uint32_t x = 0; x < net->n; ++x) {
            v[0] += sum[x];
            v[1] += sum[x] == net->R ? 1u : 0u;
        }
    }
    *known_total = v[0];
    *nodes_complete = v[1];
    return GS_OK;
}

gs_status gs_net_statistics_all(gs_net *net, uint64_t *out) {
    if (!net || !out) return GS_ERR_INVALID_ARGUMENT;
    NET_ST(observe_ready(net));
    const size_t n = net->n;
    if (net->mode == GS_NET_SHARDS) {
        // each rank's owned rows, gathered at the uniform chunk stride
        const NetRank &r0 = net->ranks[0];
        const size_t chunk = r0.info[7];
        std::vector<uint64_t> all(chunk * 5 * net->world, 0);
        for (auto &r : net->ranks) {
            const uint32_t g = r.info[6];
            std::vector<uint64_t> mine(chunk * 5, 0);
            if (r.info[1]) NET_ST(gs_statistics_all(r.e, mine.data()));
            if (net->dist) NET_ST(host_allgather(net, mine.data(), mine.size() * sizeof(uint64_t), all.data()));
            else std::copy(mine.begin(), mine.end(), all.begin() + (size_t)g * chunk * 5);
        }
        std::copy(all.begin(), all.begin() + n * 5, out);
        return GS_OK;
    }
    // rumor slices: rounds and the empty counts are the network's on every
    // slice but the pending round's empty pulls (obs: MIN over the slices);
    // full_message_* add over the slices
    std::vector<uint64_t> st(n * 5), full(n * 2, 0);
    for (size_t i = 0; i < net->ranks.size(); ++i) {
        NET_ST(gs_statistics_all(net->ranks[i].e, st.data()));
        if (i == 0) std::copy(st.begin(), st.end(), out);
        for (size_t x = 0; x < n; ++x) {
            full[2 * x] += st[5 * x + 3];
            full[2 * x + 1] += st[5 * x + 4];
        }
    }
    std::vector<uint8_t> pend(n);
    if (!net->dist) {
        NET_ST(local_min_u8(net, [](NetRank &r) { return r.obs; }, n));
    } else if (net->world > 1 && net->host) {
        NET_ST(host_min_u8_dev(net, net->ranks[0], net->ranks[0].obs, n));
    } else if (net->world > 1) {
        NetRank &r = net->ranks[0];
        NET_HIP(hipSetDevice(r.device));
        NET_ST(comm_after_engine(net, r));
        NET_NCCL(rccl().allReduce(r.obs, r.obs, n, ncclUint8, ncclMin, net->comm, r.cs));
        NET_HIP(hipStreamSynchronize(r.cs));
    }
    NET_HIP(hipSetDevice(net->ranks[0].device));
    NET_HIP(hipMemcpy(pend.data(), net->ranks[0].obs, n, hipMemcpyDeviceToHost));
    NET_ST(host_allreduce(net, full.data(), full.size(), ncclUint64, sizeof(uint64_t), ncclSum));
    for (size_t x = 0; x < n; ++x) {
        out[5 * x + 1] += pend[x];
        out[5 * x + 3] = full[2 * x];
        out[5 * x + 4] = full[2 * x + 1];
    }
    return GS_OK;
}

gs_status gs_net_dump_state(gs_net *net, uint16_t *out) {
    if (!net || !out) return GS_ERR_INVALID_ARGUMENT;
    NET_ST(observe_ready(net));
    const size_t n = net->n, R = net->R;
    if (net->mode == GS_NET_SHARDS) {
        const size_t chunk = net->ranks[0].info[7];
        std::vector<uint16_t> all(chunk * R * net->world, 0);
        for (auto &r : net->ranks) {
            std::vector<uint16_t> mine(chunk * R, 0);
            if (r.info[1]) NET_ST(gs_dump_state(r.e, mine.data()));
            if (net->dist) NET_ST(host_allgather(net, mine.data(), mine.size() * sizeof(uint16_t), all.data()));
            else std::copy(mine.begin(), mine.end(), all.begin() + (size_t)r.info[6] * chunk * R);
        }
        std::copy(all.begin(), all.begin() + n * R, out);
        return GS_OK;
    }
    // slices: columns [lo, hi) of each; gathered at the widest slice's width
    const size_t wmax = (R + net->world - 1) / net->world;
    std::vector<uint16_t> all(n * wmax * net->world, 0);
    for (auto &r : net->ranks) {
        const size_t w = r.hi - r.lo;
        std::vector<uint16_t> d(n * w), mine(n * wmax, 0);
        NET_ST(gs_dump_state(r.e, d.data()));
        for (size_t x = 0; x < n; ++x) std::copy(d.begin() + x * w, d.begin() + (x + 1) * w, mine.begin() + x * wmax);
        const uint32_t g = (uint32_t)(&r - &net->ranks[0]) + net->rank;
        if (net->dist) NET_ST(host_allgather(net, mine.data(), mine.size() * sizeof(uint16_t), all.data()));
        else std::copy(mine.begin(), mine.end(), all.begin() + (size_t)g * n * wmax);
    }
    for (uint32_t g = 0; g < net->world; ++g) {
        const size_t lo = (uint64_t)g * R / net->world, hi = (uint64_t)(g + 1) * R / net->world;
        for (size_t x = 0; x < n; ++x)
            for (size_t c = lo; c < hi; ++c) out[x * R + c] = all[(size_t)g * n * wmax + x * wmax + (c - lo)];
    }
    return GS_OK;
}

}  // extern "C"
