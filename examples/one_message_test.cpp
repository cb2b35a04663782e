// one_message_test -- the reference's convergence experiment
// (src/gossiper.rs:173-323: send_messages / one_message_test / print_metric)
// driven through the C++ host API on the MI355X engine.  The default schedule
// is SEQ, the reference harness's literal delivery order, whose averages are
// the published table (README.md:5); "2P" buffers pulls after all pushes.
//
//   ./examples/one_message_test [nodes=2000] [iterations=1000] [messages=1] [SEQ|2P]
//
// Prints the AVERAGE / MIN / MAX lines in the reference's format.
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <string>
#include <tuple>
#include <vector>

#include "safe_gossip.hpp"

using safe_gossip::Network;
using safe_gossip::Statistics;

struct Metric {
    uint64_t nodes_missed, msgs_missed;
    Statistics stats;
};

// send_messages (src/gossiper.rs:173-259): first rumor at a Philox-chosen
// node, then 50%/node/round while rumors remain; stop after a round with no
// live push; empties of the final confirmation round subtracted.
static Metric send_messages(Network &net, uint32_t num_msgs) {
    const uint32_t n = net.size();
    uint32_t next = 0;
    net.send_new(gs_origin(net.seed(), net.epoch(), 0, n), next++);
    bool processed = true;
    while (processed) {
        const uint32_t rnd = net.round() + 1;
        for (uint32_t x = 0; x < n && next < num_msgs; ++x)
            if (gs_coin(net.seed(), net.epoch(), rnd, x)) net.send_new(x, next++);
        processed = net.next_round();
    }
    // Statistics::add over every gossiper, rounds = the last one's (:241-245),
    // as device reductions; messages().len() per node as a device popcount
    Metric m{0, 0, net.statistics_reduce(GS_REDUCE_SUM)};
    m.stats.rounds = net.statistics(n - 1).rounds;
    const std::vector<uint32_t> counts = net.known_popcounts();
    for (uint32_t x = 0; x < n; ++x) {
        const uint32_t c = counts[x];
        if (c != num_msgs) {
            m.nodes_missed += 1;
            m.msgs_missed += num_msgs - c;
        }
    }
    m.stats.empty_pull_sent -= n;
    m.stats.empty_push_sent -= n;
    net.clear(net.epoch() + 1);
    return m;
}

static void print_metric(double nodes_missed, double msgs_missed, const Statistics &s,
                         uint32_t n, uint32_t msgs) {
    printf("rounds: %" PRIu64 ", empty_pulls: %" PRIu64 ", empty_pushes: %" PRIu64
           ", full_msgs_sent: %" PRIu64 ", msgs_missed: %g (%.2f%%), nodes_missed: %g (%.2f%%)\n",
           s.rounds, s.empty_pull_sent, s.empty_push_sent, s.full_message_sent, msgs_missed,
           100.0 * msgs_missed / n / msgs, nodes_missed, 100.0 * nodes_missed / n / msgs);
}

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 2000;
    const uint32_t iterations = argc > 2 ? (uint32_t)atoi(argv[2]) : 1000;
    const uint32_t msgs = argc > 3 ? (uint32_t)atoi(argv[3]) : 1;
    const bool two_phase = argc > 4 && std::string(argv[4]) == "2P";
    try {
        Network net(n, msgs, 0x5AFE6055ull, 0, 0, two_phase ? GS_SCHED_2P : GS_SCHED_SEQ);
        printf("Network of %u nodes (%s schedule):\n", n, two_phase ? "2P" : "SEQ");
        Statistics avg, mx, mn = Statistics::new_max();
        double nm_avg = 0, mm_avg = 0;
        uint64_t nm_max = 0, nm_min = UINT64_MAX, mm_max = 0, mm_min = UINT64_MAX;
        for (uint32_t i = 0; i < iterations; ++i) {
            Metric m = send_messages(net, msgs);
            nm_avg += (double)m.nodes_missed;
            mm_avg += (double)m.msgs_missed;
            nm_max = std::max(nm_max, m.nodes_missed);
            nm_min = std::min(nm_min, m.nodes_missed);
            mm_max = std::max(mm_max, m.msgs_missed);
            mm_min = std::min(mm_min, m.msgs_missed);
            avg.add(m.stats);
            mx.max(m.stats);
            mn.min(m.stats);
        }
        nm_avg /= iterations;
        mm_avg /= iterations;
        avg.rounds /= iterations;
        avg.empty_pull_sent /= iterations;
        avg.empty_push_sent /= iterations;
        avg.full_message_sent /= iterations;
        avg.full_message_received /= iterations;
        printf("    AVERAGE ---- ");
        print_metric(nm_avg, mm_avg, avg, n, msgs);
        printf("    MIN -------- ");
        print_metric((double)nm_min, (double)mm_min, mn, n, msgs);
        printf("    MAX -------- ");
        print_metric((double)nm_max, (double)mm_max, mx, n, msgs);
    } catch (const safe_gossip::GossipError &e) {
        fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
