// facade_check -- exercises the C++ host API (include/safe_gossip.hpp), the
// stand-in for the reference crate's public surface (src/lib.rs:62-65), the
// way a caller of the Rust crate would use it.  Prints one "key value" line
// per check; tests/test_gpu_facade.py runs it on the GPU and compares every
// value with the CPU oracle.
//
//   ./examples/facade_check [nodes=300] [rumors=16] [seed=0x5AFE6055]
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "safe_gossip.hpp"

using safe_gossip::ErrorKind;
using safe_gossip::GossipError;
using safe_gossip::Network;
using safe_gossip::Statistics;

static void print_stats(const char *key, const Statistics &s) {
    printf("%s %" PRIu64 " %" PRIu64 " %" PRIu64 " %" PRIu64 " %" PRIu64 "\n", key, s.rounds,
           s.empty_pull_sent, s.empty_push_sent, s.full_message_sent, s.full_message_received);
}

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 300;
    const uint32_t R = argc > 2 ? (uint32_t)atoi(argv[2]) : 16;
    const uint64_t seed = argc > 3 ? strtoull(argv[3], nullptr, 0) : 0x5AFE6055ull;
    try {
        // Error::NoPeers: a lone gossiper (src/gossiper.rs:56-58, :71-74)
        {
            Network lone(1, 1, seed);
            std::string k = "none";
            try {
                lone.gossiper(0).send_new(0);
            } catch (const GossipError &e) {
                k = e.kind() == ErrorKind::NoPeers ? "NoPeers" : "other";
            }
            printf("lone_send_new %s\n", k.c_str());
        }
        Network net(n, R, seed);
        // add_peer before any message: allowed; parameters re-derived
        net.set_params(0, 0, 0);
        const std::vector<uint8_t> p = net.params();
        printf("params %u %u %u\n", p[0], p[1], p[2]);
        // every rumor at its Philox origin, through the Gossiper view
        for (uint32_t r = 0; r < R; ++r) net.gossiper(gs_origin(seed, 0, r, n)).send_new(r);
        // Gossip::new_message inserts at once: the origin knows the rumor
        const uint32_t o0 = gs_origin(seed, 0, 0, n);
        const std::vector<uint32_t> m0 = net.gossiper(o0).messages();
        bool has0 = false;
        for (uint32_t r : m0) has0 |= r == 0;
        printf("origin_knows_rumor0 %d\n", has0 ? 1 : 0);
        // Error::AlreadyStarted: add_peer after a message exists (:45-48)
        std::string k = "none";
        try {
            net.set_params(0, 0, 0);
        } catch (const GossipError &e) {
            k = e.kind() == ErrorKind::AlreadyStarted ? "AlreadyStarted" : "other";
        }
        printf("add_peer_after_send %s\n", k.c_str());
        uint32_t rounds = 0;
        while (net.next_round()) ++rounds;
        ++rounds;  // the final all-empty round
        net.sync();
        printf("rounds %u\n", rounds);
        print_stats("stats_sum", net.statistics_reduce(GS_REDUCE_SUM));
        print_stats("stats_min", net.statistics_reduce(GS_REDUCE_MIN));
        print_stats("stats_max", net.statistics_reduce(GS_REDUCE_MAX));
        // the same reductions through the Gossiper view (Statistics::add/min/max)
        Statistics sum, mn = Statistics::new_max(), mx;
        for (uint32_t x = 0; x < n; ++x) {
            const Statistics s = net.gossiper(x).statistics();
            sum.add(s);
            mn.min(s);
            mx.max(s);
        }
        print_stats("view_sum", sum);
        print_stats("view_min", mn);
        print_stats("view_max", mx);
        uint64_t known = 0;
        for (uint32_t c : net.known_popcounts()) known += c;
        printf("known_total %" PRIu64 "\n", known);
        // clear: parameters may change again
        net.clear(1);
        net.set_params(0, 0, 0);
        printf("add_peer_after_clear ok\n");
    } catch (const GossipError &e) {
        fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
