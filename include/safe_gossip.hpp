// safe_gossip.hpp -- header-only C++ host API over the C ABI (safe_gossip.h),
// mirroring the reference crate's public surface (src/lib.rs:62-65):
//   Gossiper { id, send_new, next_round, messages, statistics }  (src/gossiper.rs:36-109)
//   Statistics { add, min, max, new_max }                          (src/gossip.rs:209-264)
//   Error { NoPeers, AlreadyStarted, SigFailure, Io, Serialisation } (src/error.rs:23-51)
// A Network owns one gs_engine: n Gossipers on one MI355X.  Errors are thrown
// as safe_gossip::GossipError carrying the reference's Error kind.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "safe_gossip.h"

namespace safe_gossip {

enum class ErrorKind : int {
    NoPeers = GS_ERR_NO_PEERS,
    AlreadyStarted = GS_ERR_ALREADY_STARTED,
    SigFailure = GS_ERR_SIG_FAILURE,
    Io = GS_ERR_IO,
    Serialisation = GS_ERR_SERIALISATION,
    Device = -1,
};

class GossipError : public std::runtime_error {
  public:
    GossipError(gs_status s)
        : std::runtime_error(gs_status_string(s)),
          kind_(s > 0 ? static_cast<ErrorKind>(s) : ErrorKind::Device), status_(s) {}
    ErrorKind kind() const { return kind_; }
    gs_status status() const { return status_; }

  private:
    ErrorKind kind_;
    gs_status status_;
};

inline void check(gs_status s) {
    if (s != GS_OK) throw GossipError(s);
}

struct Statistics {
    uint64_t rounds = 0, empty_pull_sent = 0, empty_push_sent = 0, full_message_sent = 0,
             full_message_received = 0;

    static Statistics new_max() {
        Statistics s;
        s.rounds = s.empty_pull_sent = s.empty_push_sent = s.full_message_sent =
            s.full_message_received = UINT64_MAX;
        return s;
    }
    void add(const Statistics &o) {
        rounds += o.rounds;
        empty_pull_sent += o.empty_pull_sent;
        empty_push_sent += o.empty_push_sent;
        full_message_sent += o.full_message_sent;
        full_message_received += o.full_message_received;
    }
#define SG_FOLD(op)                                                                        \
    rounds = op(rounds, o.rounds);                                                         \
    empty_pull_sent = op(empty_pull_sent, o.empty_pull_sent);                              \
    empty_push_sent = op(empty_push_sent, o.empty_push_sent);                              \
    full_message_sent = op(full_message_sent, o.full_message_sent);                        \
    full_message_received = op(full_message_received, o.full_message_received);
    static uint64_t min_(uint64_t a, uint64_t b) { return a < b ? a : b; }
    static uint64_t max_(uint64_t a, uint64_t b) { return a > b ? a : b; }
    void min(const Statistics &o) { SG_FOLD(min_) }
    void max(const Statistics &o) { SG_FOLD(max_) }
#undef SG_FOLD
    static Statistics from(const gs_statistics_t &s) {
        Statistics r;
        r.rounds = s.rounds;
        r.empty_pull_sent = s.empty_pull_sent;
        r.empty_push_sent = s.empty_push_sent;
        r.full_message_sent = s.full_message_sent;
        r.full_message_received = s.full_message_received;
        return r;
    }
};

class Network;

// Per-node view (the reference's Gossiper).  Id order == index order.
class Gossiper {
  public:
    Gossiper(Network &net, uint32_t idx) : net_(net), idx_(idx) {}
    uint32_t id() const { return idx_; }
    inline void send_new(uint32_t rumor);            // Gossiper::send_new
    inline std::vector<uint32_t> messages() const;   // Gossiper::messages
    inline Statistics statistics() const;            // Gossiper::statistics

  private:
    Network &net_;
    uint32_t idx_;
};

class Network {
  public:
    Network(uint32_t n_nodes, uint32_t n_rumors, uint64_t seed = 0x5AFE6055ull, uint32_t epoch = 0,
            int device = 0, gs_schedule schedule = GS_SCHED_2P) {
        gs_config cfg{};
        cfg.n_nodes = n_nodes;
        cfg.n_rumors = n_rumors;
        cfg.seed = seed;
        cfg.epoch = epoch;
        cfg.device = device;
        cfg.schedule = (uint8_t)schedule;
        check(gs_create(&cfg, &e_));
        n_ = n_nodes;
        r_ = n_rumors;
        seed_ = seed;
        epoch_ = epoch;
    }
    ~Network() { gs_destroy(e_); }
    Network(const Network &) = delete;
    Network &operator=(const Network &) = delete;

    uint32_t size() const { return n_; }
    uint32_t rumors() const { return r_; }
    uint64_t seed() const { return seed_; }
    uint32_t epoch() const { return epoch_; }
    uint32_t round() const { return gs_round(e_); }
    Gossiper gossiper(uint32_t i) { return Gossiper(*this, i); }

    void send_new(uint32_t node, uint32_t rumor) { check(gs_send_new(e_, node, rumor)); }
    // Gossiper::next_round for every node + delivery of every RPC; returns the
    // harness's `processed` flag (some node pushed a live rumor).
    bool next_round() {
        gs_round_report rep{};
        check(gs_next_round(e_, &rep));
        return rep.any_live != 0;
    }
    Statistics statistics(uint32_t node) {
        gs_statistics_t s{};
        check(gs_statistics(e_, node, &s));
        return Statistics::from(s);
    }
    std::vector<uint64_t> statistics_all() {
        std::vector<uint64_t> v((size_t)n_ * 5);
        check(gs_statistics_all(e_, v.data()));
        return v;
    }
    std::vector<uint32_t> messages(uint32_t node) {
        std::vector<uint64_t> w((r_ + 63) / 64);
        check(gs_messages(e_, node, w.data()));
        std::vector<uint32_t> out;
        for (uint32_t r = 0; r < r_; ++r)
            if (w[r >> 6] >> (r & 63) & 1ull) out.push_back(r);
        return out;
    }
    std::vector<uint64_t> known_all() {
        std::vector<uint64_t> w((size_t)n_ * ((r_ + 63) / 64));
        check(gs_known_all(e_, w.data()));
        return w;
    }
    // |Gossiper::messages()| of every node (device popcount)
    std::vector<uint32_t> known_popcounts() {
        std::vector<uint32_t> c(n_);
        check(gs_known_popcounts(e_, c.data()));
        return c;
    }
    // Statistics::add / min / max over every node (device reduction)
    Statistics statistics_reduce(gs_reduce_op op) {
        gs_statistics_t s{};
        check(gs_statistics_reduce(e_, op, &s));
        return Statistics::from(s);
    }
    // Gossiper::add_peer's parameter update: throws AlreadyStarted once a
    // message was sent (src/gossiper.rs:45-52); 0 = derive from n
    void set_params(uint8_t counter_max, uint8_t max_c_rounds, uint8_t max_rounds) {
        const uint8_t p[3] = {counter_max, max_c_rounds, max_rounds};
        check(gs_set_params(e_, p));
    }
    std::vector<uint8_t> params() const {
        std::vector<uint8_t> p(3);
        check(gs_get_params(e_, p.data()));
        return p;
    }
    void sync() { check(gs_sync(e_)); }
    void clear(uint32_t epoch) {
        check(gs_clear(e_, epoch));
        epoch_ = epoch;
    }
    gs_engine *handle() { return e_; }

  private:
    gs_engine *e_ = nullptr;
    uint32_t n_ = 0, r_ = 0, epoch_ = 0;
    uint64_t seed_ = 0;
};

inline void Gossiper::send_new(uint32_t rumor) { net_.send_new(idx_, rumor); }
inline std::vector<uint32_t> Gossiper::messages() const { return net_.messages(idx_); }
inline Statistics Gossiper::statistics() const { return net_.statistics(idx_); }

}  // namespace safe_gossip
